// sdhip_down.hip -- PatchSalienceDownsampler (the "featup" downsampler of the training
// loss, scenedino/models/backbones/dino/downsampler.py:31-98) forward and backward.
//
// Per patch of S = ph * pw rendered feature vectors x_i (C channels):
//   s_i = w . x_i + b                      (1x1 conv C -> 1, :88)
//   l_i = s_i * pw_i + pb_i                (per-position weight / bias, :90)
//   a   = softmax(l)                       (:91)
//   y   = sum_i a_i x_i ;  out = y / |y|   (:94-96, normalize_features)
// Backward (gradients of out, optionally of the salience / weight maps):
//   g_y = (g_out - out (out . g_out)) / |y|   (or g_out without normalisation)
//   g_a_i = g_y . x_i + g_wmap_i ;  g_l_i = a_i (g_a_i - sum_j a_j g_a_j)
//   g_s_i = g_l_i pw_i + g_sal_i ;  g_x_i = a_i g_y + g_s_i w
//   g_w = sum g_s_i x_i,  g_b = sum g_s_i,  g_pw_i = sum g_l_i s_i,  g_pb_i = sum g_l_i
// (the parameter gradients as per-patch partial rows, summed by the caller: deterministic).
//
// Work unit: one 256-thread workgroup per patch.  The two passes over the patch are laid
// out for coalescing: per-pixel dot products (a wave per pixel, lanes over channels, 16-B
// loads, DPP-free shuffle reduction), then channel sums (a thread per 4 channels, pixels
// streamed); the softmax and the per-pixel scalars live in LDS.  HBM-bound: the patch is
// read twice (the second read mostly from L2), the result written once.
#include "sdhip_common.h"

extern "C" void sd_set_error(const char *msg);

#define DS_T 256
#define DS_MAX_S 1024
#define DS_MAX_C 1024

__device__ __forceinline__ float ds_wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ float ds_wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// block-wide sum of one value per thread (256 threads, 4 waves); result to every thread
__device__ __forceinline__ float ds_block_sum(float v, float *red) {
    v = ds_wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// dot(vec, x_i) for pixels i = wave, wave + 4, ...: lanes over 4-channel groups
__device__ __forceinline__ float ds_dot(const float *__restrict__ xi, const float *vec, int C,
                                        int lane) {
    float acc = 0.f;
    for (int c = 4 * lane; c < C; c += 256) {
        const float4 xv = *(const float4 *)(xi + c);
        const float4 wv = *(const float4 *)(vec + c);
        acc = fmaf(xv.x, wv.x, acc);
        acc = fmaf(xv.y, wv.y, acc);
        acc = fmaf(xv.z, wv.z, acc);
        acc = fmaf(xv.w, wv.w, acc);
    }
    return ds_wave_sum(acc);
}

// softmax of l (S values in LDS) into a, by wave 0
__device__ __forceinline__ void ds_softmax(const float *l, float *a, int S, int lane) {
    float m = -INFINITY;
    for (int i = lane; i < S; i += 64) m = fmaxf(m, l[i]);
    m = ds_wave_max(m);
    float sum = 0.f;
    for (int i = lane; i < S; i += 64) {
        const float e = expf(l[i] - m);
        a[i] = e;
        sum += e;
    }
    sum = ds_wave_sum(sum);
    const float inv = 1.f / sum;
    for (int i = lane; i < S; i += 64) a[i] = a[i] * inv;
}

__global__ void __launch_bounds__(DS_T) k_salience_fwd(const sd_salience_args g) {
    __shared__ float s_w[DS_MAX_C];
    __shared__ float s_s[DS_MAX_S], s_a[DS_MAX_S];
    __shared__ float red[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int S = g.S, C = g.C;
    const int64_t patch = blockIdx.x;
    const float *xp = g.x + patch * (int64_t)S * C;
    for (int c = tid; c < C; c += DS_T) s_w[c] = g.w[c];
    __syncthreads();
    // pass 1: salience and logits
    for (int i = wave; i < S; i += 4) {
        const float d = ds_dot(xp + (int64_t)i * C, s_w, C, lane);
        if (lane == 0) {
            const float s = d + (g.b ? g.b[0] : 0.f);
            s_s[i] = s;
            s_a[i] = fmaf(s, g.pw[i], g.pb[i]);
        }
    }
    __syncthreads();
    if (wave == 0) ds_softmax(s_a, s_a, S, lane);
    __syncthreads();
    for (int i = tid; i < S; i += DS_T) {
        if (g.sal) g.sal[patch * S + i] = s_s[i];
        if (g.wmap) g.wmap[patch * S + i] = s_a[i];
    }
    // pass 2: y = sum_i a_i x_i, thread = 4 channels (C <= 1024)
    const int c4 = 4 * tid;
    float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c4 < C) {
        for (int i = 0; i < S; ++i) {
            const float ai = s_a[i];
            const float4 xv = *(const float4 *)(xp + (int64_t)i * C + c4);
            y.x = fmaf(ai, xv.x, y.x);
            y.y = fmaf(ai, xv.y, y.y);
            y.z = fmaf(ai, xv.z, y.z);
            y.w = fmaf(ai, xv.w, y.w);
        }
    }
    float nrm = 1.f;
    if (g.normalize) {
        nrm = sqrtf(ds_block_sum(y.x * y.x + y.y * y.y + y.z * y.z + y.w * y.w, red));
        if (tid == 0) g.ynorm[patch] = nrm;
    }
    if (c4 < C) {  // patched / norm, a division as the reference
        const float4 o = g.normalize ? make_float4(y.x / nrm, y.y / nrm, y.z / nrm, y.w / nrm) : y;
        *(float4 *)(g.out + patch * C + c4) = o;
    }
}

__global__ void __launch_bounds__(DS_T) k_salience_bwd(const sd_salience_args g) {
    __shared__ float s_gy[DS_MAX_C], s_w[DS_MAX_C];
    __shared__ float s_a[DS_MAX_S], s_ga[DS_MAX_S], s_gs[DS_MAX_S];
    __shared__ float red[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int S = g.S, C = g.C;
    const int64_t patch = blockIdx.x;
    const float *xp = g.x + patch * (int64_t)S * C;
    const int c4 = 4 * tid;
    // g_y
    float4 go = make_float4(0.f, 0.f, 0.f, 0.f), u = go;
    if (c4 < C) {
        go = *(const float4 *)(g.g_out + patch * C + c4);
        u = *(const float4 *)(g.out + patch * C + c4);
    }
    float4 gy = go;
    if (g.normalize) {
        const float ug = ds_block_sum(u.x * go.x + u.y * go.y + u.z * go.z + u.w * go.w, red);
        const float inv = 1.f / g.ynorm[patch];
        gy = make_float4((go.x - u.x * ug) * inv, (go.y - u.y * ug) * inv,
                         (go.z - u.z * ug) * inv, (go.w - u.w * ug) * inv);
    }
    if (c4 < C) {
        *(float4 *)(s_gy + c4) = gy;
        *(float4 *)(s_w + c4) = *(const float4 *)(g.w + c4);
    }
    for (int i = tid; i < S; i += DS_T) s_a[i] = g.wmap[patch * S + i];
    __syncthreads();
    // pass A: g_a_i = g_y . x_i (+ g_wmap_i)
    for (int i = wave; i < S; i += 4) {
        const float d = ds_dot(xp + (int64_t)i * C, s_gy, C, lane);
        if (lane == 0) s_ga[i] = d + (g.g_wmap ? g.g_wmap[patch * S + i] : 0.f);
    }
    __syncthreads();
    if (wave == 0) {
        float t = 0.f;
        for (int i = lane; i < S; i += 64) t = fmaf(s_a[i], s_ga[i], t);
        t = ds_wave_sum(t);
        float gb = 0.f;
        for (int i = lane; i < S; i += 64) {
            const float gl = s_a[i] * (s_ga[i] - t);
            const float gs = fmaf(gl, g.pw[i], g.g_sal ? g.g_sal[patch * S + i] : 0.f);
            s_gs[i] = gs;
            gb += gs;
            g.gpw_part[patch * S + i] = gl * g.sal[patch * S + i];
            g.gpb_part[patch * S + i] = gl;
        }
        gb = ds_wave_sum(gb);
        if (lane == 0) g.gb_part[patch] = gb;
    }
    __syncthreads();
    // pass B: g_x_i = a_i g_y + g_s_i w ; g_w partial = sum_i g_s_i x_i
    if (c4 < C) {
        const float4 wv = *(const float4 *)(s_w + c4);
        float4 gw = make_float4(0.f, 0.f, 0.f, 0.f);
        float *gxp = g.gx + patch * (int64_t)S * C;
        for (int i = 0; i < S; ++i) {
            const float ai = s_a[i], gs = s_gs[i];
            const float4 xv = *(const float4 *)(xp + (int64_t)i * C + c4);
            gw.x = fmaf(gs, xv.x, gw.x);
            gw.y = fmaf(gs, xv.y, gw.y);
            gw.z = fmaf(gs, xv.z, gw.z);
            gw.w = fmaf(gs, xv.w, gw.w);
            *(float4 *)(gxp + (int64_t)i * C + c4) =
                make_float4(fmaf(ai, gy.x, gs * wv.x), fmaf(ai, gy.y, gs * wv.y),
                            fmaf(ai, gy.z, gs * wv.z), fmaf(ai, gy.w, gs * wv.w));
        }
        *(float4 *)(g.gw_part + patch * C + c4) = gw;
    }
}

static int ds_check(const sd_salience_args *g, const char *name) {
    if (!g || !g->x || !g->w || !g->pw || !g->pb || g->N < 0 || g->S <= 0 || g->S > DS_MAX_S ||
        g->C <= 0 || g->C > DS_MAX_C || g->C % 4 ||
        (((uintptr_t)g->x | (uintptr_t)g->w) & 15)) {
        sd_set_error(name);
        return -1;
    }
    return 0;
}

extern "C" int sd_salience_fwd(const sd_salience_args *g, void *stream) {
    if (ds_check(g, "sd_salience_fwd: invalid argument (S <= 1024, C <= 1024, C % 4 == 0, "
                    "16-byte aligned x / w)"))
        return -1;
    if (!g->out || ((uintptr_t)g->out & 15) || (g->normalize && !g->ynorm)) {
        sd_set_error("sd_salience_fwd: out (16-byte aligned) and, if normalising, ynorm needed");
        return -1;
    }
    if (g->N == 0) return 0;
    hipLaunchKernelGGL(k_salience_fwd, dim3((unsigned)g->N), dim3(DS_T), 0, (hipStream_t)stream,
                       *g);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_salience_fwd: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_salience_bwd(const sd_salience_args *g, void *stream) {
    if (ds_check(g, "sd_salience_bwd: invalid argument") || !g->out || !g->g_out || !g->sal ||
        !g->wmap || !g->gx || !g->gw_part || !g->gpw_part || !g->gpb_part || !g->gb_part ||
        (g->normalize && !g->ynorm) ||
        (((uintptr_t)g->out | (uintptr_t)g->g_out | (uintptr_t)g->gx | (uintptr_t)g->gw_part) & 15)) {
        sd_set_error("sd_salience_bwd: invalid argument");
        return -1;
    }
    if (g->N == 0) return 0;
    hipLaunchKernelGGL(k_salience_bwd, dim3((unsigned)g->N), dim3(DS_T), 0, (hipStream_t)stream,
                       *g);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_salience_bwd: launch failed");
        return -2;
    }
    return 0;
}
