// sdhip_common.h -- shared device helpers for the gfx950 SceneDINO kernels.
// Compiled with -ffp-contract=off: every fused multiply-add is an explicit fmaf()
// so that the bit-exact kernels (ray generation, z sampling) reproduce the
// reference's separately rounded fp32 arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sdhip.h"

#include <mutex>
#include <unordered_map>

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel) (and on growth),
// not per launch: a host call on every launch of the latency-bound eager paths otherwise
// (ADVICE r4).  Keyed by the current device too: the attribute is set while a device is
// current, so a process driving several GPUs sets it once on each.
static inline void sd_lds_attr(const void *kern, int bytes) {
    static std::mutex mu;
    static std::unordered_map<const void *, int> set[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    std::lock_guard<std::mutex> g(mu);
    auto it = set[dev].find(kern);
    if (it != set[dev].end() && it->second >= bytes) return;
    (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    set[dev][kern] = bytes;
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// Per-frame render inputs (sd_frame_inputs): work item gid < N H W packs pixel gid of the
// NCHW colour images into NHWC4; gid - N H W < n SD_CAM_WORDS writes one camera-record word
// (the fused projection K . w2c[:3] accumulated in f64, rounded once)
__device__ __forceinline__ void sd_cam_word(const float *__restrict__ w2c, int64_t s_w,
                                            const float *__restrict__ Ks, int64_t s_k, int64_t n,
                                            float *__restrict__ out, int64_t gid) {
    if (gid >= n * SD_CAM_WORDS) return;
    const int64_t v = gid / SD_CAM_WORDS;
    const int e = (int)(gid - v * SD_CAM_WORDS);
    const float *w = w2c + v * s_w, *k = Ks + v * s_k;
    float r;
    if (e < 12) {
        r = w[e];
    } else if (e < 21) {
        r = k[e - 12];
    } else if (e < 24) {
        r = 0.f;
    } else {
        const int i = (e - 24) >> 2, c = (e - 24) & 3;
        r = (float)((double)k[3 * i] * w[c] + (double)k[3 * i + 1] * w[4 + c] +
                    (double)k[3 * i + 2] * w[8 + c]);
    }
    out[gid] = r;
}
__device__ __forceinline__ void sd_frame_item(const sd_frame_args &fa, int64_t gid) {
    const int64_t hw = fa.H * fa.W, np = fa.N * hw;
    if (gid >= np) {
        sd_cam_word(fa.w2c, fa.s_w, fa.Ks, fa.s_k, fa.n, fa.out_cam, gid - np);
        return;
    }
    const int64_t b = gid / hw, p = gid - b * hw;
    const float *s = fa.img_nchw + b * 3 * hw + p;
    typedef __attribute__((ext_vector_type(4))) float f4;
    *(f4 *)(fa.out_nhwc4 + gid * 4) = f4{s[0], s[hw], s[2 * hw], 0.f};
}
__host__ __device__ inline int64_t sd_frame_items(const sd_frame_args &fa) {
    return fa.N * fa.H * fa.W + fa.n * SD_CAM_WORDS;
}

#define SD_WAVE 64
#define SD_DH 128          // ResnetFC d_hidden (configs/model/dino_downsampler.yaml:39)
#define SD_PE_CHUNKS 3     // 39 positional-code features padded to 48 = 3 x 16
#define SD_EPS 1e-3f       // scenedino/common/cameras/pinhole.py:3
#define SD_MAX_NV 4        // colour (render) views handled by the fused kernels

// torch.linspace(start, end, n)[i] in fp32 (identical on CPU and CUDA builds of
// torch; verified against the reference's rays bit for bit, tests/golden).
// I: int64_t, or int where n fits (the render kernels' K: 32-bit compare / convert); the
// float results are the same for every n, i < 2^24
template <typename I>
__device__ __forceinline__ float sd_linspace_at(float start, float end, I n, I i) {
    if (n == 1) return start;
    float step = (end - start) / (float)(n - 1);
    int64_t half = n / 2;
    if (i < half) return fmaf(step, (float)i, start);
    return fmaf(-step, (float)(n - 1 - i), end);
}

__device__ __forceinline__ float bf16lo(uint32_t d) { return __uint_as_float(d << 16); }
__device__ __forceinline__ float bf16hi(uint32_t d) { return __uint_as_float(d & 0xffff0000u); }

// Camera record: w2c rows 0..2 (3x4) then normalised K (3x3).
// pts_into_camera (pinhole.py:40-59) followed by project_to_image (pinhole.py:62-84).
// CP: const float * or a constant-address-space pointer (scalar loads of a
// wave-uniform record).
typedef __attribute__((address_space(4))) const float sd_cfloat;
template <typename CP>
__device__ __forceinline__ void sd_project(CP cam, float px, float py,
                                           float pz, float &x, float &y, float &zc) {
    float c0 = ((cam[0] * px + cam[1] * py) + cam[2] * pz) + cam[3];
    float c1 = ((cam[4] * px + cam[5] * py) + cam[6] * pz) + cam[7];
    float c2 = ((cam[8] * px + cam[9] * py) + cam[10] * pz) + cam[11];
    CP K = cam + 12;
    float i0 = (K[0] * c0 + K[1] * c1) + K[2] * c2;
    float i1 = (K[3] * c0 + K[4] * c1) + K[5] * c2;
    float i2 = (K[6] * c0 + K[7] * c1) + K[8] * c2;
    float zd = fmaxf(i2, SD_EPS);
    x = i0 / zd;
    y = i1 / zd;
    zc = i2;
}

// outside_frustum (pinhole.py:87-112)
__device__ __forceinline__ bool sd_outside(float x, float y, float zc) {
    return (zc <= SD_EPS) | (x < -1.f) | (x > 1.f) | (y < -1.f) | (y > 1.f);
}

// Bilinear tap setup of F.grid_sample(mode=bilinear, padding_mode=border,
// align_corners=False) for normalised coords (x, y) on an (h, w) image.
struct Taps {
    int i00, i01, i10, i11;   // pixel indices (row-major y*w + x) of nw, ne, sw, se
    float w00, w01, w10, w11; // bilinear weights
    int x0, y0;               // column / row of the nw tap
};

__device__ __forceinline__ Taps sd_taps(float x, float y, int w, int h) {
    float ix = ((x + 1.f) * (float)w - 1.f) / 2.f;
    float iy = ((y + 1.f) * (float)h - 1.f) / 2.f;
    ix = fminf((float)(w - 1), fmaxf(ix, 0.f));
    iy = fminf((float)(h - 1), fmaxf(iy, 0.f));
    float fx0 = floorf(ix), fy0 = floorf(iy);
    int x0 = (int)fx0, y0 = (int)fy0;
    x0 = min(max(x0, 0), w - 1);
    y0 = min(max(y0, 0), h - 1);
    int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, h - 1);
    float ex = (fx0 + 1.f) - ix, wx = ix - fx0;  // weight of x0 / x1 column
    float ey = (fy0 + 1.f) - iy, wy = iy - fy0;
    Taps t;
    t.i00 = y0 * w + x0; t.i01 = y0 * w + x1; t.i10 = y1 * w + x0; t.i11 = y1 * w + x1;
    t.w00 = ex * ey; t.w01 = wx * ey; t.w10 = ex * wy; t.w11 = wx * wy;
    t.x0 = x0; t.y0 = y0;
    return t;
}

// NeRFRenderer.sample_coarse for sample k of a ray (nerf.py:121-141) given its jitter
// uu: t = linspace(0, 1 - 1/K, K)[k] + uu / K, then lindisp / linear depth.  Every
// operation separately rounded (bit-exact with the reference, tests/golden).
template <typename I>
__device__ __forceinline__ float sd_z_sample(float near, float far, I K, I k, float uu,
                                             float step, float t_end, int lindisp) {
    const float t = sd_linspace_at(0.0f, t_end, K, k) + uu * step;
    if (lindisp) {
        const float a = (1.0f / near) * (1.0f - t);
        const float b = (1.0f / far) * t;
        return 1.0f / (a + b);
    }
    return near * (1.0f - t) + far * t;
}

// The same stratified sample for the counter-RNG jitter (perf mode: sd_sample_z with
// u == NULL and the render kernels' in-kernel depths, which no reference value pins --
// any uniform stream is a valid draw): hardware reciprocals instead of the three IEEE
// divisions of the reference recipe (within 1-2 ulp of it).
template <typename I>
__device__ __forceinline__ float sd_z_sample_rng(float near, float far, I K, I k, float uu,
                                                 float step, float t_end, int lindisp) {
    const float t = sd_linspace_at(0.0f, t_end, K, k) + uu * step;
    if (lindisp) {
        const float a = __builtin_amdgcn_rcpf(near) * (1.0f - t);
        return __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_rcpf(far), t, a));
    }
    return near * (1.0f - t) + far * t;
}

// Counter-based uniform [0,1) (24-bit mantissa) for perf-mode jitter: murmur3's 32-bit
// finaliser over the counter, keyed by both halves of the 64-bit seed (the reference draws
// torch.rand_like, nerf.py:134; any uniform stream is a valid stratified sample).
__device__ __forceinline__ float sd_uniform(uint64_t seed, uint64_t ctr) {
    uint32_t x = (uint32_t)ctr ^ (uint32_t)seed;
    x = (x ^ (uint32_t)(ctr >> 32)) * 0x9E3779B1u + (uint32_t)(seed >> 32);
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}
