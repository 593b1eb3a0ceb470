// sdhip_point.h -- per-point device helpers shared by the gfx950 field kernels
// (sdhip_field.hip: grid-space MLP; sdhip_proj.hip: projected-grid MLP).
#pragma once
#include "sdhip_common.h"

extern "C" void sd_set_error(const char *msg);

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;


// ---------------------------------------------------------------------------
// per-point geometry
// ---------------------------------------------------------------------------
struct PointGeo {
    Taps t;
    float v[3];   // [x, y, z~] inputs of the positional code (after clamp(-2,2))
    bool inv_f;   // outside the encoder frustum
};

// FASTZ (16-bit modes): z~ with a hardware reciprocal; it only feeds the positional
// code, never the masks or taps.
template <bool FASTZ = false, typename CP>
__device__ __forceinline__ PointGeo sd_point_geo(CP cam, float px, float py,
                                                 float pz, int Wf, int Hf) {
    PointGeo g;
    float x, y, zc;
    sd_project(cam, px, py, pz, x, y, zc);
    g.inv_f = sd_outside(x, y, zc);
    x = fminf(fmaxf(x, -2.f), 2.f);
    y = fminf(fmaxf(y, -2.f), 2.f);
    // encoding_mode._z, inv_z, d_min=3, d_max=80 (positional_encoding.py:13-21).
    // (1/d_min - 1/d_max) is a Python double rounded once to fp32, as in the reference.
    float zt = FASTZ
        ? (__builtin_amdgcn_rcpf(fmaxf(zc, SD_EPS)) - (float)(1.0 / 80.0)) * (float)(1.0 / (1.0 / 3.0 - 1.0 / 80.0))
        : (1.f / fmaxf(zc, SD_EPS) - (float)(1.0 / 80.0)) / (float)(1.0 / 3.0 - 1.0 / 80.0);
    zt = 2.f * zt - 1.f;
    g.v[0] = x; g.v[1] = y; g.v[2] = zt;
    g.t = sd_taps(x, y, Wf, Hf);
    return g;
}


// 16-bit render modes: projection through the fused record P = K . w2c[:3]
// (SD_CAM_WORDS layout, words 24..35) with fmaf and one hardware reciprocal -- a few ulp
// from the two-step pts_into_camera / project_to_image, far below the 16-bit operands.
// x, y, zc as sd_project; rz = 1 / max(zc, eps) (the z~ input of the code).
template <typename CP>
__device__ __forceinline__ void sd_project_fast(CP cam, float px, float py, float pz, float &x,
                                                float &y, float &zc, float &rz) {
    CP P = cam + 24;
    const float i0 = fmaf(P[0], px, fmaf(P[1], py, fmaf(P[2], pz, P[3])));
    const float i1 = fmaf(P[4], px, fmaf(P[5], py, fmaf(P[6], pz, P[7])));
    const float i2 = fmaf(P[8], px, fmaf(P[9], py, fmaf(P[10], pz, P[11])));
    rz = __builtin_amdgcn_rcpf(fmaxf(i2, SD_EPS));
    x = i0 * rz;
    y = i1 * rz;
    zc = i2;
}

// Frustum mask of a fast projection, bit-exact with sd_outside on the two-step one: only
// points within 1e-4 of a frustum plane can differ, and those (a divergent, rarely taken
// branch) are re-projected the reference way.
template <typename CP>
__device__ __forceinline__ bool sd_outside_exact(CP cam, float px, float py, float pz, float x,
                                                 float y, float zc) {
    bool inv = sd_outside(x, y, zc);
    const bool edge = fabsf(fabsf(x) - 1.f) < 1e-4f || fabsf(fabsf(y) - 1.f) < 1e-4f ||
                      fabsf(zc - SD_EPS) < 1e-4f;
    if (edge) {
        float xe, ye, ze;
        sd_project(cam, px, py, pz, xe, ye, ze);
        inv = sd_outside(xe, ye, ze);
    }
    return inv;
}

template <typename CP>
__device__ __forceinline__ PointGeo sd_point_geo_fast(CP cam, float px, float py, float pz, int Wf,
                                                      int Hf) {
    PointGeo g;
    float x, y, zc, rz;
    sd_project_fast(cam, px, py, pz, x, y, zc, rz);
    g.inv_f = sd_outside_exact(cam, px, py, pz, x, y, zc);
    x = fminf(fmaxf(x, -2.f), 2.f);
    y = fminf(fmaxf(y, -2.f), 2.f);
    const float zt = (rz - (float)(1.0 / 80.0)) * (float)(1.0 / (1.0 / 3.0 - 1.0 / 80.0));
    g.v[0] = x; g.v[1] = y; g.v[2] = 2.f * zt - 1.f;
    g.t = sd_taps(x, y, Wf, Hf);
    return g;
}

template <typename CP>
__device__ __forceinline__ Taps sd_color_taps_fast(CP cam, int Wc, int Hc, float px, float py,
                                                   float pz, bool &inv) {
    float x, y, zc, rz;
    sd_project_fast(cam, px, py, pz, x, y, zc, rz);
    inv = sd_outside_exact(cam, px, py, pz, x, y, zc);  // (clamping x, y to +-2 keeps it)
    x = fminf(fmaxf(x, -2.f), 2.f);
    y = fminf(fmaxf(y, -2.f), 2.f);
    return sd_taps(x, y, Wc, Hc);
}

__device__ __forceinline__ uint4 sd_ld128(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
#if SD_ABL_NOLOAD  // diagnostic timing build only: the gather replaced by register values
    (void)rs;
    return uint4{voff & 0x3c003c00u, soff & 0x3c003c00u, (voff ^ soff) & 0x3c003c00u, 0x3c003c00u};
#else
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
#endif
}


// Buffer descriptor over one batch element's grid plane (wave-uniform inputs).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sd_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}

// ReLU without the canonicalising v_max hipcc adds in front of fmaxf on MFMA results
__device__ __forceinline__ float sd_relu(float x) {
    return __builtin_amdgcn_fmed3f(x, 0.f, __builtin_inff());
}


// An opaque zero: indexing LDS with it stops LICM from hoisting the per-sub-tile
// weight reads out of the loop (which would pin ~100 VGPRs and spill).
__device__ __forceinline__ int sd_opaque0() {
    int z = 0;
    asm volatile("" : "+v"(z));
    return z;
}


// torch.nn.functional.softplus(beta=1, threshold=20)
__device__ __forceinline__ float sd_softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

__device__ __forceinline__ void sd_sample_rgb(const float *__restrict__ img, const Taps &t,
                                              float out[3]) {
    f32x4 a = *(const f32x4 *)(img + (int64_t)t.i00 * 4);
    f32x4 b = *(const f32x4 *)(img + (int64_t)t.i01 * 4);
    f32x4 c = *(const f32x4 *)(img + (int64_t)t.i10 * 4);
    f32x4 d = *(const f32x4 *)(img + (int64_t)t.i11 * 4);
#pragma unroll
    for (int i = 0; i < 3; ++i)
        out[i] = ((a[i] * t.w00 + b[i] * t.w01) + c[i] * t.w10) + d[i] * t.w11;
}

// colour-sample taps + validity in a render view (bts.py:336-346; clamp before the
// frustum test)
template <typename CP>
__device__ __forceinline__ Taps sd_color_taps(CP cam, int Wc, int Hc, float px, float py, float pz,
                                              bool &inv) {
    float x, y, zc;
    sd_project(cam, px, py, pz, x, y, zc);
    x = fminf(fmaxf(x, -2.f), 2.f);
    y = fminf(fmaxf(y, -2.f), 2.f);
    inv = sd_outside(x, y, zc);
    return sd_taps(x, y, Wc, Hc);
}

template <typename CP>
__device__ __forceinline__ bool sd_color_view(CP cam, const float *img, int Wc, int Hc,
                                              float px, float py, float pz, float col[3]) {
    bool inv;
    const Taps tc = sd_color_taps(cam, Wc, Hc, px, py, pz, inv);
    sd_sample_rgb(img, tc, col);
    return inv;
}

// colour sample split in two: the four texel loads issued now, the blend later (after
// other work has hidden their latency)
struct ColPend {
    f32x4 a, b, c, d;
    float w00, w01, w10, w11;
    float delta;
};

__device__ __forceinline__ void sd_color_issue(const float *__restrict__ img, const Taps &t,
                                               ColPend &cp) {
    cp.a = *(const f32x4 *)(img + (int64_t)t.i00 * 4);
    cp.b = *(const f32x4 *)(img + (int64_t)t.i01 * 4);
    cp.c = *(const f32x4 *)(img + (int64_t)t.i10 * 4);
    cp.d = *(const f32x4 *)(img + (int64_t)t.i11 * 4);
    cp.w00 = t.w00; cp.w01 = t.w01; cp.w10 = t.w10; cp.w11 = t.w11;
}

// same arithmetic and order as sd_sample_rgb
__device__ __forceinline__ void sd_color_finish(const ColPend &cp, float out[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
        out[i] = ((cp.a[i] * cp.w00 + cp.b[i] * cp.w01) + cp.c[i] * cp.w10) + cp.d[i] * cp.w11;
}


// CUs left to other kernels by the persistent grids (sd_reserve_cus; defined in
// sdhip_field.hip): the multi-GPU step runs RCCL's all-gather of the previous frame beside the
// render, one workgroup per channel, and a persistent workgroup whose CU is held waits for it
extern int sd_g_cu_reserve;

// Workgroups of a persistent one-per-CU grid: the device's CUs minus the reservation, rounded
// down to a multiple of 8 (the kernels' XCD-aware ranges assume gridDim.x % 8 == 0)
static int sd_num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    const int r = sd_g_cu_reserve;
    if (r <= 0) return n;
    const int m = ((n - r) / 8) * 8;
    return m >= 8 ? m : n;
}


// Wave-uniform position of a persistent wave's work item: ray (< 2^31), sub-tile of
// the ray and the ray's super-batch (batch element) index.  Advanced without integer
// division (a 64-bit divide is ~100 scalar instructions); clamps at the wave's last
// item, which the software pipelines then only re-open for prefetch.
struct ItemCursor {
    int ray, sub, sbi;
};

__device__ __forceinline__ ItemCursor sd_cursor0(int ray0, int rays_per_sb) {
    return {ray0, 0, (int)((unsigned)ray0 / (unsigned)rays_per_sb)};
}

__device__ __forceinline__ ItemCursor sd_advance(ItemCursor c, int nsub, int nwaves, int R,
                                                 int rays_per_sb) {
    if (c.sub + 1 < nsub) {
        c.sub++;
    } else if (c.ray + nwaves < R) {
        c.ray += nwaves;
        c.sub = 0;
        c.sbi = (int)((unsigned)c.ray / (unsigned)rays_per_sb);
    }
    return c;
}
