// sdhip_field.hip -- fused feature-field render (gfx950 / CDNA4).
//
// One wave owns a tile of 32 rays and walks their K samples in order
// (sample-major).  Per sample the 32 points form the N=32 side of 32x32 MFMA
// tiles of the first ResnetFC layer, computed transposed (H^T = W_in X^T) so that
// every lane's accumulator column is "its" ray:
//   * lane l (ray l&31, half h=l>>5) gathers 8 consecutive channels of its point
//     from the NHWC grid for each 16-channel chunk -> B fragment, bilinear blend
//     in fp32 registers (F.grid_sample bilinear/border/align_corners=False);
//   * W_in fragments live in LDS (staged once per workgroup);
//   * the 39-d positional code is computed in registers (3 more K chunks);
//   * epilogue: +b_in, ReLU, sigma = w_sigma . h (fp32 dot + one cross-half add),
//     softplus, alpha, sequential transmittance (exactly torch.cumprod's order),
//     and the weighted sum  Hacc += w_k * relu(h_k)  in fp32 registers.
// The DINO head is linear in h, so  sum_k w_k (W_out h_k + b) = W_out Hacc + (sum w) b:
// the second layer runs ONCE per ray tile on the accumulated Hacc (16 MFMAs per 64
// dims) instead of once per sample.  Colours are sampled per sample in the render
// views (NHWC4 fp32) and composited in registers.
//
// Reference: NeRFRenderer.composite (scenedino/renderer/nerf.py:230-449),
// BTSNet.forward / sample_features / sample_colors (scenedino/models/bts.py:271-595),
// ResnetFC.forward (models/prediction_heads/resnetfc.py:135-203),
// PositionalEncoding + encoding_mode._z (common/positional_encoding.py:13-80),
// pinhole projection (common/cameras/pinhole.py:40-112).
#include "sdhip_common.h"

#include <string.h>
#include <type_traits>

static thread_local char g_err[512] = "";
extern "C" void sd_set_error(const char *msg) {
    strncpy(g_err, msg, sizeof(g_err) - 1);
    g_err[sizeof(g_err) - 1] = 0;
}
extern "C" const char *sd_last_error(void) { return g_err; }
extern "C" int sd_abi_version(void) { return 1; }

template <int DT> struct GridT;
template <> struct GridT<SD_BF16> { typedef uint16_t T; };
template <> struct GridT<SD_F32> { typedef float T; };

// ---------------------------------------------------------------------------
// per-point geometry: projection into the encoder view, taps, positional code
// ---------------------------------------------------------------------------
struct PointGeo {
    Taps t;
    float v[3];   // [x, y, z~] inputs of the positional code (after clamp(-2,2))
    bool inv_f;   // outside the encoder frustum
};

__device__ __forceinline__ PointGeo sd_point_geo(const float *__restrict__ cam, float px, float py,
                                                 float pz, int Wf, int Hf) {
    PointGeo g;
    float x, y, zc;
    sd_project(cam, px, py, pz, x, y, zc);
    g.inv_f = sd_outside(x, y, zc);
    x = fminf(fmaxf(x, -2.f), 2.f);
    y = fminf(fmaxf(y, -2.f), 2.f);
    // encoding_mode._z with inv_z, d_min=3, d_max=80 (positional_encoding.py:13-21)
    float zt = (1.f / fmaxf(zc, SD_EPS) - 1.f / 80.f) / (1.f / 3.f - 1.f / 80.f);
    zt = 2.f * zt - 1.f;
    g.v[0] = x; g.v[1] = y; g.v[2] = zt;
    g.t = sd_taps(x, y, Wf, Hf);
    return g;
}

// Positional-code chunk pc (0..2) for lane half h: element j of the fragment is
// slot s = 8*pc + j.  s < 18: freq index s/3 (f = 1.5 * 2^(s/3)), input dim s%3,
// phase h*pi/2 (h=0 -> sin, h=1 -> cos as sin(x + pi/2), as the reference).  s in
// 18..20 (h == 0): the raw inputs.  Everything else: 0.  The host packs W_in's 39
// code columns in this order (scenedino_amd/mlp_pack.py).
template <bool FAST>
__device__ __forceinline__ void sd_pe_chunk(const float v[3], int pc, int h, float out[8]) {
    const float phase = h ? 1.5707963705062866f : 0.f;  // float32(pi/2), positional_encoding.py:65
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int s = 8 * pc + j;
        float r = 0.f;
        if (s < 18) {
            float f = 1.5f * (float)(1 << (s / 3));
            float a = phase + v[s % 3] * f;
            r = FAST ? __sinf(a) : sinf(a);
        } else if (s < 21) {
            r = h ? 0.f : v[s - 18];
        }
        out[j] = r;
    }
}

// ---------------------------------------------------------------------------
// first layer: acc[ht] (32 hidden x 32 points) += W_in[ht] . X^T over C + 48 k
// ---------------------------------------------------------------------------
template <int DT> struct Layer1;

template <> struct Layer1<SD_BF16> {
    struct TapRaw { uint4 a, b, c, d; };
    static __device__ __forceinline__ TapRaw load(const uint16_t *__restrict__ g, const Taps &t,
                                                  int C, int coff) {
        TapRaw r;
        r.a = *(const uint4 *)(g + (int64_t)t.i00 * C + coff);
        r.b = *(const uint4 *)(g + (int64_t)t.i01 * C + coff);
        r.c = *(const uint4 *)(g + (int64_t)t.i10 * C + coff);
        r.d = *(const uint4 *)(g + (int64_t)t.i11 * C + coff);
        return r;
    }
    static __device__ __forceinline__ float blend1(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                                   bool hi, const Taps &t) {
        float va = hi ? bf16hi(a) : bf16lo(a), vb = hi ? bf16hi(b) : bf16lo(b);
        float vc = hi ? bf16hi(c) : bf16lo(c), vd = hi ? bf16hi(d) : bf16lo(d);
        return fmaf(vd, t.w11, fmaf(vc, t.w10, fmaf(vb, t.w01, va * t.w00)));
    }
    static __device__ __forceinline__ bf16x8 blend(const TapRaw &r, const Taps &t) {
        float f[8];
        uint32_t A[4] = {r.a.x, r.a.y, r.a.z, r.a.w}, B[4] = {r.b.x, r.b.y, r.b.z, r.b.w};
        uint32_t Cc[4] = {r.c.x, r.c.y, r.c.z, r.c.w}, D[4] = {r.d.x, r.d.y, r.d.z, r.d.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[2 * i] = blend1(A[i], B[i], Cc[i], D[i], false, t);
            f[2 * i + 1] = blend1(A[i], B[i], Cc[i], D[i], true, t);
        }
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (__bf16)f[i];
        return o;
    }
    // acc[ht] += A(q, ht) . B
    static __device__ __forceinline__ void mma(const uint8_t *lds_w, int q, int lane,
                                               const bf16x8 &b, f32x16 acc[4]) {
        const bf16x8 *w = (const bf16x8 *)lds_w + (q * 4) * SD_WAVE + lane;
#pragma unroll
        for (int ht = 0; ht < 4; ++ht)
            acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[ht * SD_WAVE], b, acc[ht], 0, 0, 0);
    }
    static __device__ __forceinline__ void mma_f(const uint8_t *lds_w, int q, int lane,
                                                 const float f[8], f32x16 acc[4]) {
        bf16x8 b;
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = (__bf16)f[i];
        mma(lds_w, q, lane, b, acc);
    }

    template <bool FAST_PE>
    static __device__ __forceinline__ void run(const uint16_t *__restrict__ g, int C,
                                               const PointGeo &geo, const uint8_t *lds_w,
                                               int lane, f32x16 acc[4]) {
        const int h = lane >> 5;
        const int nq = C >> 4;
        int coff = 8 * h;
        TapRaw cur = load(g, geo.t, C, coff);
        for (int q = 0; q < nq; ++q) {
            TapRaw nxt = cur;
            if (q + 1 < nq) nxt = load(g, geo.t, C, coff + 16);
            bf16x8 b = blend(cur, geo.t);
            mma(lds_w, q, lane, b, acc);
            cur = nxt;
            coff += 16;
        }
#pragma unroll
        for (int pc = 0; pc < SD_PE_CHUNKS; ++pc) {
            float f[8];
            sd_pe_chunk<FAST_PE>(geo.v, pc, h, f);
            mma_f(lds_w, nq + pc, lane, f, acc);
        }
    }
};

template <> struct Layer1<SD_F32> {
    struct TapRaw { f32x4 a0, a1, b0, b1, c0, c1, d0, d1; };
    static __device__ __forceinline__ TapRaw load(const float *__restrict__ g, const Taps &t, int C,
                                                  int coff) {
        TapRaw r;
        const float *pa = g + (int64_t)t.i00 * C + coff, *pb = g + (int64_t)t.i01 * C + coff;
        const float *pc = g + (int64_t)t.i10 * C + coff, *pd = g + (int64_t)t.i11 * C + coff;
        r.a0 = *(const f32x4 *)pa; r.a1 = *(const f32x4 *)(pa + 4);
        r.b0 = *(const f32x4 *)pb; r.b1 = *(const f32x4 *)(pb + 4);
        r.c0 = *(const f32x4 *)pc; r.c1 = *(const f32x4 *)(pc + 4);
        r.d0 = *(const f32x4 *)pd; r.d1 = *(const f32x4 *)(pd + 4);
        return r;
    }
    // grid_sample order: nw, ne, sw, se accumulated left to right.
    static __device__ __forceinline__ void blend(const TapRaw &r, const Taps &t, float f[8]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[i] = ((r.a0[i] * t.w00 + r.b0[i] * t.w01) + r.c0[i] * t.w10) + r.d0[i] * t.w11;
            f[4 + i] = ((r.a1[i] * t.w00 + r.b1[i] * t.w01) + r.c1[i] * t.w10) + r.d1[i] * t.w11;
        }
    }
    static __device__ __forceinline__ void mma_f(const uint8_t *lds_w, int q, int lane,
                                                 const float f[8], f32x16 acc[4]) {
        const f32x4 *w = (const f32x4 *)lds_w + ((q * 4) * SD_WAVE + lane) * 2;
#pragma unroll
        for (int ht = 0; ht < 4; ++ht) {
            f32x4 w0 = w[ht * SD_WAVE * 2], w1 = w[ht * SD_WAVE * 2 + 1];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[i], f[i], acc[ht], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[i], f[4 + i], acc[ht], 0, 0, 0);
        }
    }
    template <bool FAST_PE>
    static __device__ __forceinline__ void run(const float *__restrict__ g, int C,
                                               const PointGeo &geo, const uint8_t *lds_w,
                                               int lane, f32x16 acc[4]) {
        const int h = lane >> 5;
        const int nq = C >> 4;
        int coff = 8 * h;
        for (int q = 0; q < nq; ++q) {
            TapRaw r = load(g, geo.t, C, coff);
            float f[8];
            blend(r, geo.t, f);
            mma_f(lds_w, q, lane, f, acc);
            coff += 16;
        }
#pragma unroll
        for (int pc = 0; pc < SD_PE_CHUNKS; ++pc) {
            float f[8];
            sd_pe_chunk<FAST_PE>(geo.v, pc, h, f);
            mma_f(lds_w, nq + pc, lane, f, acc);
        }
    }
};

// ---------------------------------------------------------------------------
// second layer on an accumulator-layout operand X (32 hidden rows per tile t in
// registers, point/ray on the lane):  out^T (32 dims x 32 points) = W[dt] . X
// ---------------------------------------------------------------------------
template <int DT> struct Layer2;
template <> struct Layer2<SD_BF16> {
    // A fragments: [dt][t][s][lane][8] bf16
    static __device__ __forceinline__ f32x16 run(const bf16x8 *__restrict__ w, int dt,
                                                 const f32x16 X[4], int lane) {
        f32x16 acc = {};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 b;
#pragma unroll
                for (int j = 0; j < 8; ++j) b[j] = (__bf16)X[t][8 * s + j];
                bf16x8 a = w[((dt * 4 + t) * 2 + s) * SD_WAVE + lane];
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
            }
        }
        return acc;
    }
};
template <> struct Layer2<SD_F32> {
    // A values: [dt][t][lane][16] f32
    static __device__ __forceinline__ f32x16 run(const float *__restrict__ w, int dt,
                                                 const f32x16 X[4], int lane) {
        f32x16 acc = {};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f32x4 *wp = (const f32x4 *)(w + ((int64_t)(dt * 4 + t) * SD_WAVE + lane) * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4 a = wp[q];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], X[t][4 * q + i], acc, 0, 0, 0);
            }
        }
        return acc;
    }
};

// relu(acc + b_in) in place; returns this lane's half of w_sigma . h
__device__ __forceinline__ float sd_bias_relu_sigma(f32x16 acc[4], const float *lds_b,
                                                    const float *lds_ws, int h) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const f32x4 *bb = (const f32x4 *)(lds_b + (t * 2 + h) * 16);
        const f32x4 *ww = (const f32x4 *)(lds_ws + (t * 2 + h) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 b = bb[q], w = ww[q];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = fmaxf(acc[t][4 * q + i] + b[i], 0.f);
                acc[t][4 * q + i] = v;
                s = fmaf(v, w[i], s);
            }
        }
    }
    return s;
}

// torch.nn.functional.softplus(beta=1, threshold=20)
__device__ __forceinline__ float sd_softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// bilinear sample of an NHWC4 colour image (grid_sample, border, align_corners=False)
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

// Stage W_in fragments + bias / sigma rows into LDS (one pass per workgroup).
// An opaque zero: indexing LDS with it stops LICM from hoisting the per-sample
// weight reads out of the sample loop (which would pin ~100 VGPRs and spill).
__device__ __forceinline__ int sd_opaque0() {
    int z = 0;
    asm volatile("" : "+v"(z));
    return z;
}

__device__ __forceinline__ void sd_stage_weights(uint8_t *lds, const sd_mlp &m, int win_bytes) {
    const uint4 *src = (const uint4 *)m.w_in;
    uint4 *dst = (uint4 *)lds;
    for (int i = threadIdx.x; i < win_bytes / 16; i += blockDim.x) dst[i] = src[i];
    float *fb = (float *)(lds + win_bytes);
    for (int i = threadIdx.x; i < 128; i += blockDim.x) {
        fb[i] = m.b_in_h[i];
        fb[128 + i] = m.w_sig_h[i];
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// fused render kernel
// ---------------------------------------------------------------------------
template <int DT, bool FAST_PE>
__global__ void __launch_bounds__(256, DT == SD_BF16 ? 2 : 1)
k_render(const sd_render_args a, const sd_mlp m, int win_bytes) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    typedef typename GridT<DT>::T G;
    sd_stage_weights(lds, m, win_bytes);
    const float *lds_b = (const float *)(lds + win_bytes);
    const float *lds_ws = lds_b + 128;

    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int wave = threadIdx.x >> 6;
    const int64_t ntiles = (a.R + 31) / 32;
    const int K = a.K, C = m.C, nv = a.nv;
    const int64_t plane = (int64_t)a.Hf * a.Wf * C;
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;

    for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles;
         tile += (int64_t)gridDim.x * 4) {
        const int64_t ray_u = tile * 32 + (lane & 31);
        const bool valid = ray_u < a.R;
        const int64_t ray = valid ? ray_u : a.R - 1;
        const int64_t sbi = ray / a.rays_per_sb;
        const float *rr = a.rays + ray * a.ray_dim;
        const float ox = rr[0], oy = rr[1], oz = rr[2], dx = rr[3], dy = rr[4], dz = rr[5];
        const float *zr = a.z + ray * K;
        const G *grid = (const G *)a.grid + sbi * plane;
        const float *camf = a.cam_f + sbi * 21;

        f32x16 hacc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) hacc[t] = f32x16{};
        float T = 1.f, wsum = 0.f, depth = 0.f;
        float rgbacc[3 * SD_MAX_NV];
#pragma unroll
        for (int i = 0; i < 3 * SD_MAX_NV; ++i) rgbacc[i] = 0.f;

        float zk = zr[0];
        for (int k = 0; k < K; ++k) {
            const float zn = (k + 1 < K) ? zr[k + 1] : 0.f;
            const float delta = (k + 1 < K) ? (zn - zk) : 1e10f;
            // points = o + z*d (nerf.py:252)
            const float px = ox + zk * dx, py = oy + zk * dy, pz = oz + zk * dz;
            PointGeo geo = sd_point_geo(camf, px, py, pz, a.Wf, a.Hf);

            f32x16 acc[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = f32x16{};
            const int lo = sd_opaque0();
            Layer1<DT>::template run<FAST_PE>(grid, C, geo, lds + lo, lane, acc);

            float s = sd_bias_relu_sigma(acc, lds_b + lo, lds_ws + lo, h);
            s += __shfl_xor(s, 32);
            const float sigma = sd_softplus(s + m.b_sigma);

            // alpha compositing (nerf.py:376-389)
            float alpha = 1.f - expf(-fabsf(delta) * fmaxf(sigma, 0.f));
            if (a.hard_alpha_cap && k == K - 1) alpha = 1.f;
            const float w = alpha * T;
            T = T * ((1.f - alpha) + 1e-10f);
            wsum += w;
            depth += w * zk;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) hacc[t][r] = fmaf(w, acc[t][r], hacc[t][r]);

            // colours in the render views (bts.py:330-441)
            bool inv_any_c[SD_MAX_NV];
            float col[3 * SD_MAX_NV];
#pragma unroll
            for (int v = 0; v < SD_MAX_NV; ++v) {
                inv_any_c[v] = false;
                col[3 * v] = col[3 * v + 1] = col[3 * v + 2] = 0.f;
                if (v < nv) {
                    float x, y, zc;
                    sd_project(a.cam_c + (sbi * nv + v) * 21, px, py, pz, x, y, zc);
                    x = fminf(fmaxf(x, -2.f), 2.f);
                    y = fminf(fmaxf(y, -2.f), 2.f);
                    inv_any_c[v] = sd_outside(x, y, zc);
                    Taps tc = sd_taps(x, y, a.Wc, a.Hc);
                    sd_sample_rgb(a.img + (sbi * nv + v) * cplane, tc, col + 3 * v);
                    rgbacc[3 * v] += w * col[3 * v];
                    rgbacc[3 * v + 1] += w * col[3 * v + 1];
                    rgbacc[3 * v + 2] += w * col[3 * v + 2];
                }
            }

            if (valid) {
                const int64_t o = ray * K + k;
                if (h == 0) {
                    if (a.weights) a.weights[o] = w;
                    if (a.alphas) a.alphas[o] = alpha;
                    if (a.invalid_f) a.invalid_f[o] = geo.inv_f ? 1 : 0;
                } else {
#pragma unroll
                    for (int v = 0; v < SD_MAX_NV; ++v) {
                        if (v < nv) {
                            if (a.invalid) a.invalid[o * nv + v] = (inv_any_c[v] | geo.inv_f) ? 1.f : 0.f;
                            if (a.rgb_samps) {
                                a.rgb_samps[(o * nv + v) * 3] = col[3 * v];
                                a.rgb_samps[(o * nv + v) * 3 + 1] = col[3 * v + 1];
                                a.rgb_samps[(o * nv + v) * 3 + 2] = col[3 * v + 2];
                            }
                        }
                    }
                }
            }
            zk = zn;
        }

        // DINO head on the accumulated hidden state: dino = W_out Hacc + wsum * b
        const int ndt = m.D >> 5;
        for (int dt = 0; dt < ndt; ++dt) {
            f32x16 o = Layer2<DT>::run((const typename std::conditional<DT == SD_BF16, bf16x8, float>::type *)m.w_out,
                                       dt, hacc, lane);
            if (valid) {
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    int dim = dt * 32 + 8 * g4 + 4 * h;
                    f32x4 bb = *(const f32x4 *)(m.b_dino + dim);
                    f32x4 val;
#pragma unroll
                    for (int i = 0; i < 4; ++i) val[i] = o[4 * g4 + i] + wsum * bb[i];
                    *(f32x4 *)(a.dino + ray * m.D + dim) = val;
                }
            }
        }
        if (valid && h == 0) {
            a.depth[ray] = depth;
#pragma unroll
            for (int v = 0; v < SD_MAX_NV; ++v)
                if (v < nv) {
                    a.rgb[ray * 3 * nv + 3 * v] = rgbacc[3 * v];
                    a.rgb[ray * 3 * nv + 3 * v + 1] = rgbacc[3 * v + 1];
                    a.rgb[ray * 3 * nv + 3 * v + 2] = rgbacc[3 * v + 2];
                }
        }
    }
}

// ---------------------------------------------------------------------------
// per-point field query (no compositing): 32 consecutive points per wave step
// ---------------------------------------------------------------------------
template <int DT, bool FAST_PE>
__global__ void __launch_bounds__(256, DT == SD_BF16 ? 2 : 1)
k_field(const sd_field_args a, const sd_mlp m, int win_bytes) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    typedef typename GridT<DT>::T G;
    sd_stage_weights(lds, m, win_bytes);
    const float *lds_b = (const float *)(lds + win_bytes);
    const float *lds_ws = lds_b + 128;

    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int wave = threadIdx.x >> 6;
    const int64_t NP = a.B * a.P;
    const int64_t ntiles = (NP + 31) / 32;
    const int C = m.C, nv = a.nv;
    const int64_t plane = (int64_t)a.Hf * a.Wf * C;
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;

    for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < ntiles;
         tile += (int64_t)gridDim.x * 4) {
        const int64_t pu = tile * 32 + (lane & 31);
        const bool valid = pu < NP;
        const int64_t p = valid ? pu : NP - 1;
        const int64_t b = p / a.P;
        const float px = a.xyz[p * 3], py = a.xyz[p * 3 + 1], pz = a.xyz[p * 3 + 2];
        const G *grid = (const G *)a.grid + b * plane;
        PointGeo geo = sd_point_geo(a.cam_f + b * 21, px, py, pz, a.Wf, a.Hf);

        f32x16 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = f32x16{};
        const int lo = sd_opaque0();
        Layer1<DT>::template run<FAST_PE>(grid, C, geo, lds + lo, lane, acc);
        float s = sd_bias_relu_sigma(acc, lds_b + lo, lds_ws + lo, h);
        s += __shfl_xor(s, 32);
        const float sigma = sd_softplus(s + m.b_sigma);

        const int ndt = m.D >> 5;
        for (int dt = 0; dt < ndt; ++dt) {
            f32x16 o = Layer2<DT>::run((const typename std::conditional<DT == SD_BF16, bf16x8, float>::type *)m.w_out,
                                       dt, acc, lane);
            if (valid) {
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    int dim = dt * 32 + 8 * g4 + 4 * h;
                    f32x4 bb = *(const f32x4 *)(m.b_dino + dim);
                    f32x4 val;
#pragma unroll
                    for (int i = 0; i < 4; ++i) val[i] = o[4 * g4 + i] + bb[i];
                    *(f32x4 *)(a.dino + p * m.D + dim) = val;
                }
            }
        }
        if (valid && h == 0) {
            a.sigma[p] = sigma;
            if (a.invalid_f) a.invalid_f[p] = geo.inv_f ? 1 : 0;
        }
        if (valid && h == 1 && nv > 0 && (a.rgb || a.invalid)) {
#pragma unroll
            for (int v = 0; v < SD_MAX_NV; ++v) {
                if (v < nv) {
                    float x, y, zc, col[3];
                    sd_project(a.cam_c + (b * nv + v) * 21, px, py, pz, x, y, zc);
                    x = fminf(fmaxf(x, -2.f), 2.f);
                    y = fminf(fmaxf(y, -2.f), 2.f);
                    bool ic = sd_outside(x, y, zc);
                    Taps tc = sd_taps(x, y, a.Wc, a.Hc);
                    sd_sample_rgb(a.img + (b * nv + v) * cplane, tc, col);
                    if (a.rgb) {
                        a.rgb[(p * nv + v) * 3] = col[0];
                        a.rgb[(p * nv + v) * 3 + 1] = col[1];
                        a.rgb[(p * nv + v) * 3 + 2] = col[2];
                    }
                    if (a.invalid) a.invalid[p * nv + v] = (ic | geo.inv_f) ? 1.f : 0.f;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// standalone compositor: one wave per ray, lane = feature column
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_composite(const float *__restrict__ z, const float *__restrict__ sigma,
            const float *__restrict__ feat, int64_t F, const float *__restrict__ rgb, int64_t Cc,
            int64_t R, int K, int hard_cap, float *__restrict__ weights,
            float *__restrict__ alphas, float *__restrict__ depth, float *__restrict__ feat_out,
            float *__restrict__ rgb_out) {
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= R) return;
    const float *zr = z + ray * K, *sr = sigma + ray * K;
    float T = 1.f, dep = 0.f;
    const int nf = (int)((F + 63) / 64);
    float facc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float cacc = 0.f;
    for (int k = 0; k < K; ++k) {
        float zk = zr[k];
        float delta = (k + 1 < K) ? zr[k + 1] - zk : 1e10f;
        float alpha = 1.f - expf(-fabsf(delta) * fmaxf(sr[k], 0.f));
        if (hard_cap && k == K - 1) alpha = 1.f;
        float w = alpha * T;
        T = T * ((1.f - alpha) + 1e-10f);
        dep += w * zk;
        if (lane == 0) {
            if (weights) weights[ray * K + k] = w;
            if (alphas) alphas[ray * K + k] = alpha;
        }
        if (feat) {
            const float *fr = feat + (ray * K + k) * F;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < nf && lane + 64 * j < F) facc[j] += fr[lane + 64 * j] * w;
        }
        if (rgb && lane < Cc) cacc += w * rgb[(ray * K + k) * Cc + lane];
    }
    if (lane == 0 && depth) depth[ray] = dep;
    if (feat && feat_out) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j < nf && lane + 64 * j < F) feat_out[ray * F + lane + 64 * j] = facc[j];
    }
    if (rgb && rgb_out && lane < Cc) rgb_out[ray * Cc + lane] = cacc;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int sd_num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

static int sd_check_mlp(const sd_mlp *m, int *win_bytes, int *lds_bytes) {
    if (!m || !m->w_in || !m->b_in_h || !m->w_sig_h || !m->w_out || !m->b_dino) {
        sd_set_error("sd_mlp: null parameter pointer");
        return -1;
    }
    if (m->d_hidden != SD_DH || m->C <= 0 || (m->C % 16) || m->D <= 0 || (m->D % 32) ||
        (m->dtype != SD_BF16 && m->dtype != SD_F32)) {
        sd_set_error("sd_mlp: unsupported shape (need d_hidden=128, C%16==0, D%32==0)");
        return -1;
    }
    int nq = m->C / 16 + SD_PE_CHUNKS;
    int esz = m->dtype == SD_BF16 ? 2 : 4;
    *win_bytes = nq * 4 * SD_WAVE * 8 * esz;
    *lds_bytes = *win_bytes + 256 * 4;
    if (*lds_bytes > 160 * 1024) {
        sd_set_error("sd_mlp: W_in fragments exceed LDS (reduce C or use bf16)");
        return -1;
    }
    return 0;
}

#define SD_LAUNCH_FIELD(KERN, DT, GRID, LDS, STREAM, ...)                                    \
    do {                                                                                     \
        static bool attr_set_##KERN##DT = false;                                             \
        if (!attr_set_##KERN##DT) {                                                          \
            (void)hipFuncSetAttribute((const void *)KERN<DT, SD_FASTPE>,                               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS > 65536 ? 163840 : 65536); \
            attr_set_##KERN##DT = true;                                                      \
        }                                                                                    \
        hipLaunchKernelGGL((KERN<DT, SD_FASTPE>), GRID, dim3(256), LDS, STREAM, __VA_ARGS__);    \
    } while (0)

extern "C" int sd_render_fused(const sd_render_args *args, const sd_mlp *mlp, void *stream) {
    int win = 0, lds = 0;
    if (!args) {
        sd_set_error("sd_render_fused: null args");
        return -1;
    }
    if (sd_check_mlp(mlp, &win, &lds)) return -1;
    const sd_render_args &a = *args;
    if (a.R < 0 || a.K <= 0 || a.ray_dim < 6 || a.rays_per_sb <= 0 || !a.rays || !a.z ||
        !a.grid || !a.cam_f || !a.depth || !a.dino || a.Hf <= 0 || a.Wf <= 0 || a.nv < 0 ||
        a.nv > SD_MAX_NV || (a.nv > 0 && (!a.img || !a.cam_c || !a.rgb || a.Hc <= 0 || a.Wc <= 0))) {
        sd_set_error("sd_render_fused: invalid argument (nv must be 0..4)");
        return -1;
    }
    if (a.R == 0) return 0;
    int64_t ntiles = (a.R + 31) / 32;
    int per_cu = mlp->dtype == SD_BF16 ? 2 : 1;
    int64_t nblk = (ntiles + 3) / 4;
    int64_t cap = (int64_t)sd_num_cus() * per_cu;
    if (nblk > cap) nblk = cap;
    dim3 grid((unsigned)nblk);
    hipStream_t s = (hipStream_t)stream;
    if (mlp->dtype == SD_BF16)
        SD_LAUNCH_FIELD(k_render, SD_BF16, grid, lds, s, a, *mlp, win);
    else
        SD_LAUNCH_FIELD(k_render, SD_F32, grid, lds, s, a, *mlp, win);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        return -2;
    }
    return 0;
}

extern "C" int sd_field_query(const sd_field_args *args, const sd_mlp *mlp, void *stream) {
    int win = 0, lds = 0;
    if (!args) {
        sd_set_error("sd_field_query: null args");
        return -1;
    }
    if (sd_check_mlp(mlp, &win, &lds)) return -1;
    const sd_field_args &a = *args;
    if (a.B <= 0 || a.P < 0 || !a.xyz || !a.grid || !a.cam_f || !a.sigma || !a.dino ||
        a.Hf <= 0 || a.Wf <= 0 || a.nv < 0 || a.nv > SD_MAX_NV ||
        (a.nv > 0 && (a.rgb || a.invalid) && (!a.img || !a.cam_c || a.Hc <= 0 || a.Wc <= 0))) {
        sd_set_error("sd_field_query: invalid argument");
        return -1;
    }
    if (a.P == 0) return 0;
    int64_t ntiles = (a.B * a.P + 31) / 32;
    int per_cu = mlp->dtype == SD_BF16 ? 2 : 1;
    int64_t nblk = (ntiles + 3) / 4;
    int64_t cap = (int64_t)sd_num_cus() * per_cu * 4;
    if (nblk > cap) nblk = cap;
    dim3 grid((unsigned)nblk);
    hipStream_t s = (hipStream_t)stream;
    if (mlp->dtype == SD_BF16)
        SD_LAUNCH_FIELD(k_field, SD_BF16, grid, lds, s, a, *mlp, win);
    else
        SD_LAUNCH_FIELD(k_field, SD_F32, grid, lds, s, a, *mlp, win);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        return -2;
    }
    return 0;
}

extern "C" int sd_composite(const float *z, const float *sigma, const float *feat, int64_t F,
                            const float *rgb, int64_t Cc, int64_t R, int32_t K,
                            int32_t hard_alpha_cap, float *weights, float *alphas, float *depth,
                            float *feat_out, float *rgb_out, void *stream) {
    if (!z || !sigma || R < 0 || K <= 0 || F < 0 || F > 512 || Cc < 0 || Cc > 64 ||
        (feat && !feat_out) || (rgb && !rgb_out)) {
        sd_set_error("sd_composite: invalid argument (F<=512, Cc<=64)");
        return -1;
    }
    if (R == 0) return 0;
    hipLaunchKernelGGL(k_composite, dim3((unsigned)((R + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, z, sigma, feat, F, rgb, Cc, R, K, hard_alpha_cap,
                       weights, alphas, depth, feat_out, rgb_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        return -2;
    }
    return 0;
}
