// sdhip_field.hip -- fused feature-field render and field query (gfx950 / CDNA4).
//
// Work unit: one wave = 32 consecutive points (lanes l and l+32 share point l&31;
// lane half h = l>>5 supplies the other 8 channels of every 16-channel K chunk).
//   * render kernel: the 32 points are 32 consecutive samples of ONE ray (ray-major),
//     so the bilinear taps of a sub-tile are spatially coherent (identical for the
//     render-from-encoder-view case of the demo / SSCBench) and every per-sample
//     store is coalesced;
//   * field kernel: 32 consecutive query points.
// First ResnetFC layer, transposed:  H^T (128 hidden x 32 points) = W_in . X^T as
// 4 tiles of 32x32 MFMA; W_in fragments staged once per workgroup in LDS; the lane's
// B fragment = bilinear blend of 8 NHWC channels from the 4 taps (F.grid_sample
// bilinear/border/align_corners=False) or 8 values of the 39-d positional code.
// Epilogue (accumulator layout: lane = point): +b_in via the initial accumulator,
// ReLU, sigma = w_sigma . h (fp32 dot + one cross-half add), softplus.
// Render kernel compositing: alpha, wave-level prefix product of (1-alpha+1e-10)
// across the 32 lanes (+ carry across sub-tiles) = transmittance, weights, and the
// DINO head folded into the compositing sum:
//     sum_k w_k (W_out h_k + b) = sum_k (w_k h_k) W_out^T + (sum_k w_k) b
// i.e. the second-layer MFMA consumes w-scaled hidden states and ACCUMULATES over
// all samples of the ray in its accumulator (O layout: points summed in registers,
// dims on lanes).  Colours: bilinear NHWC4 fp32 in each render view.
//
// Precision modes (template P): SD_F32 (f32 grid, exact-f32 MFMA 32x32x2, accurate
// sinf), SD_F16 (f16 grid, packed-f16 blend, f16 MFMA), SD_BF16 (as SD_F16 up to sigma,
// the DINO output layer on bf16 MFMA: RMode in sdhip_render.h).  All modes accumulate in fp32 and keep geometry, alpha and
// transmittance in fp32.
//
// Reference: NeRFRenderer.composite (scenedino/renderer/nerf.py:230-449),
// BTSNet.forward / sample_features / sample_colors (scenedino/models/bts.py:271-595),
// ResnetFC.forward (models/prediction_heads/resnetfc.py:135-203),
// PositionalEncoding + encoding_mode._z (common/positional_encoding.py:13-80),
// pinhole projection (common/cameras/pinhole.py:40-112).
#include "sdhip_point.h"
#include "sdhip_render.h"

#include <string.h>

static thread_local char g_err[512] = "";
extern "C" void sd_set_error(const char *msg) {
    strncpy(g_err, msg, sizeof(g_err) - 1);
    g_err[sizeof(g_err) - 1] = 0;
}
extern "C" const char *sd_last_error(void) { return g_err; }
extern "C" int sd_abi_version(void) { return 11; }

int sd_g_cu_reserve = 0;

extern "C" int32_t sd_reserve_cus(int32_t n) {
    const int prev = sd_g_cu_reserve;
    sd_g_cu_reserve = n > 0 ? n : 0;
    return prev;
}

// diagnostic: nblocks single-wave workgroups with 32 KiB of LDS each that hold a CU for `us`
// microseconds (the constant 100 MHz wall clock), bounded -- the CU occupancy of another
// stream's kernel (tools/contention_ab.py stands in for RCCL's all-gather with it: its blocks
// hold shared memory, and the persistent render workgroups need nearly all of a CU's LDS)
__global__ void __launch_bounds__(64) k_spin(int64_t ticks) {
    extern __shared__ float spin_lds[];  // holds LDS like RCCL's per-block shared state
    const uint64_t t0 = wall_clock64();
    while ((int64_t)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
    if (ticks < 0) spin_lds[threadIdx.x] = 0.f;
}

extern "C" int sd_spin(int32_t nblocks, float us, void *stream) {
    if (nblocks <= 0 || nblocks > 4096 || !(us >= 0.f) || us > 1e6f) {
        sd_set_error("sd_spin: invalid argument (1..4096 blocks, 0..1e6 us)");
        return -1;
    }
    hipLaunchKernelGGL(k_spin, dim3((unsigned)nblocks), dim3(64), 32768, (hipStream_t)stream,
                       (int64_t)(us * 100.f));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        return -2;
    }
    return 0;
}

extern "C" int sd_field_dtype(int dtype) {
    // Prec<SD_BF16> inherits Prec<SD_F16>: the bf16 mode reads its grids, W_in and the
    // projected grid as f16 (only the DINO output layer is bf16)
    return dtype == SD_F32 ? SD_F32 : (dtype == SD_BF16 || dtype == SD_F16) ? SD_F16 : -1;
}

// Threads per workgroup, one workgroup per CU: 16-bit kernels run 8 waves (2 per SIMD,
// <= 256 VGPRs each); the f32 parity kernels run 4 waves (1 per SIMD, 512 VGPRs).
template <int P> struct WG {
    static constexpr int T = P == SD_F32 ? 256 : 512;
    static constexpr int W = T / 64;
};

// Positional-code chunk pc (0..2) for lane half h: fragment element j = slot s = 8pc+j.
// s < 18: sin(phase_h + v[s%3] * 1.5*2^(s/3)) with phase_h = h*float32(pi/2) (cos as
// sin(x+pi/2), as the reference); s = 18..20 (h == 0): the raw inputs; else 0.
// The host packs W_in's 39 code columns in this order (scenedino_amd/mlp_pack.py).
template <bool FAST>
__device__ __forceinline__ void sd_pe_chunk(const float v[3], int pc, int h, float out[8]) {
    const float phase = h ? 1.5707963705062866f : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int s = 8 * pc + j;
        float r = 0.f;
        if (s < 18) {
            float f = 1.5f * (float)(1 << (s / 3));
            float a = fmaf(v[s % 3], f, phase);  // torch.addcmul is a fused multiply-add
            r = FAST ? __sinf(a) : sinf(a);
        } else if (s < 21) {
            r = h ? 0.f : v[s - 18];
        }
        out[j] = r;
    }
}

// ---------------------------------------------------------------------------
// precision traits: grid storage, tap loads, blend, layer-1 / layer-2 MFMA
// ---------------------------------------------------------------------------
template <int P> struct Prec;

struct Raw16 { uint4 a, b, c, d; };  // 4 taps x 8 x 16-bit channels

// Byte offsets (within the grid plane of this ray's batch element) of the lane's
// channel slice in the 4 taps at chunk 0; chunk q adds q * 16 * esz bytes, which is
// wave-uniform and goes into the buffer load's scalar offset (no per-load VALU).
struct TapOff { uint32_t o00, o01, o10, o11; };

__device__ __forceinline__ TapOff sd_tapoff(const Taps &t, int C, int esz, int h,
                                           uint32_t base = 0) {
    const uint32_t row = (uint32_t)C * esz, lo = (uint32_t)(8 * esz * h) + base;
    return {t.i00 * row + lo, t.i01 * row + lo, t.i10 * row + lo, t.i11 * row + lo};
}

__device__ __forceinline__ Raw16 sd_load16(__amdgpu_buffer_rsrc_t rs, const TapOff &o, int q) {
    const uint32_t s = (uint32_t)q * 32u;
    Raw16 r;
    r.a = sd_ld128(rs, o.o00, s);
    r.b = sd_ld128(rs, o.o01, s);
    r.c = sd_ld128(rs, o.o10, s);
    r.d = sd_ld128(rs, o.o11, s);
    return r;
}

// 16-bit field blend: packed-f16 FMAs over the four taps (4 v_pk_fma per channel pair)
template <> struct Prec<SD_F16> {
    typedef uint16_t G;
    typedef Raw16 Raw;
    typedef f16x8 Frag;
    static constexpr bool FAST_PE = true;
    static constexpr int ESZ = 2, DEPTH = 4;
    static __device__ __forceinline__ Raw load(__amdgpu_buffer_rsrc_t rs, const TapOff &o, int q) {
        return sd_load16(rs, o, q);
    }
    static __device__ __forceinline__ Frag blend(const Raw &r, const Taps &t) {
        const f16x2 w0 = {(_Float16)t.w00, (_Float16)t.w00}, w1 = {(_Float16)t.w01, (_Float16)t.w01};
        const f16x2 w2 = {(_Float16)t.w10, (_Float16)t.w10}, w3 = {(_Float16)t.w11, (_Float16)t.w11};
        uint32_t A[4] = {r.a.x, r.a.y, r.a.z, r.a.w}, B[4] = {r.b.x, r.b.y, r.b.z, r.b.w};
        uint32_t Cc[4] = {r.c.x, r.c.y, r.c.z, r.c.w}, D[4] = {r.d.x, r.d.y, r.d.z, r.d.w};
        Frag o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f16x2 v = __builtin_bit_cast(f16x2, A[i]) * w0;
            v = __builtin_elementwise_fma(__builtin_bit_cast(f16x2, B[i]), w1, v);
            v = __builtin_elementwise_fma(__builtin_bit_cast(f16x2, Cc[i]), w2, v);
            v = __builtin_elementwise_fma(__builtin_bit_cast(f16x2, D[i]), w3, v);
            o[2 * i] = v[0];
            o[2 * i + 1] = v[1];
        }
        return o;
    }
    static __device__ __forceinline__ Frag from_f(const float f[8]) {
        Frag o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (_Float16)f[i];
        return o;
    }
    static __device__ __forceinline__ void mma1(const uint8_t *lw, int q, int lane, const Frag &b,
                                                f32x16 acc[4]) {
        const Frag *w = (const Frag *)lw + (q * 4) * SD_WAVE + lane;
#pragma unroll
        for (int ht = 0; ht < 4; ++ht)
            acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_f16(w[ht * SD_WAVE], b, acc[ht], 0, 0, 0);
    }
    static __device__ __forceinline__ void mma2(const uint8_t *w_out, int dt, const f32x16 X[4],
                                                int lane, f32x16 &out) {
        const Frag *w = (const Frag *)w_out + (dt * 8) * SD_WAVE + lane;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                Frag a;
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = (_Float16)X[t][8 * s + j];
                out = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, w[(t * 2 + s) * SD_WAVE], out, 0, 0, 0);
            }
    }
};

// bf16 mode (RMode, sdhip_render.h): the grid, its blend, layer 1 and sigma as the fp16
// mode (an f16 grid); only the DINO output layer on bf16 operands
template <> struct Prec<SD_BF16> : Prec<SD_F16> {
    // out (32 points x 32 dims, O layout) += X^T . W_out^T[dt]; X in accumulator layout.
    // w_out: [dt][t][s][lane] x 16 B
    static __device__ __forceinline__ void mma2(const uint8_t *w_out, int dt, const f32x16 X[4],
                                                int lane, f32x16 &out) {
        const bf16x8 *w = (const bf16x8 *)w_out + (dt * 8) * SD_WAVE + lane;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                bf16x8 a;
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = (__bf16)X[t][8 * s + j];
                out = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, w[(t * 2 + s) * SD_WAVE], out, 0, 0, 0);
            }
    }
};

template <> struct Prec<SD_F32> {
    typedef float G;
    struct Raw { f32x4 a0, a1, b0, b1, c0, c1, d0, d1; };
    struct Frag { float f[8]; };
    static constexpr bool FAST_PE = false;
    static constexpr int ESZ = 4, DEPTH = 2;
    static __device__ __forceinline__ f32x4 ld(__amdgpu_buffer_rsrc_t rs, uint32_t v, uint32_t s) {
        return __builtin_bit_cast(f32x4, sd_ld128(rs, v, s));
    }
    static __device__ __forceinline__ Raw load(__amdgpu_buffer_rsrc_t rs, const TapOff &o, int q) {
        const uint32_t s = (uint32_t)q * 64u;
        Raw r;
        r.a0 = ld(rs, o.o00, s); r.a1 = ld(rs, o.o00, s + 16);
        r.b0 = ld(rs, o.o01, s); r.b1 = ld(rs, o.o01, s + 16);
        r.c0 = ld(rs, o.o10, s); r.c1 = ld(rs, o.o10, s + 16);
        r.d0 = ld(rs, o.o11, s); r.d1 = ld(rs, o.o11, s + 16);
        return r;
    }
    // grid_sample order: nw, ne, sw, se accumulated left to right, separately rounded.
    static __device__ __forceinline__ Frag blend(const Raw &r, const Taps &t) {
        Frag o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o.f[i] = ((r.a0[i] * t.w00 + r.b0[i] * t.w01) + r.c0[i] * t.w10) + r.d0[i] * t.w11;
            o.f[4 + i] = ((r.a1[i] * t.w00 + r.b1[i] * t.w01) + r.c1[i] * t.w10) + r.d1[i] * t.w11;
        }
        return o;
    }
    static __device__ __forceinline__ Frag from_f(const float f[8]) {
        Frag o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o.f[i] = f[i];
        return o;
    }
    // f32 A values: [q][ht][lane][8]; 8 exact-f32 32x32x2 MFMAs per (chunk, ht)
    static __device__ __forceinline__ void mma1(const uint8_t *lw, int q, int lane, const Frag &b,
                                                f32x16 acc[4]) {
        const f32x4 *w = (const f32x4 *)lw + ((q * 4) * SD_WAVE + lane) * 2;
#pragma unroll
        for (int ht = 0; ht < 4; ++ht) {
            f32x4 w0 = w[ht * SD_WAVE * 2], w1 = w[ht * SD_WAVE * 2 + 1];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0[i], b.f[i], acc[ht], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                acc[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[i], b.f[4 + i], acc[ht], 0, 0, 0);
        }
    }
    // w_out: [dt][t][lane][16] f32;  out += X^T . W_out^T[dt]
    static __device__ __forceinline__ void mma2(const uint8_t *w_out, int dt, const f32x16 X[4],
                                                int lane, f32x16 &out) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f32x4 *wp = (const f32x4 *)w_out + ((int64_t)(dt * 4 + t) * SD_WAVE + lane) * 4;
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                f32x4 b = wp[q4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    out = __builtin_amdgcn_mfma_f32_32x32x2f32(X[t][4 * q4 + i], b[i], out, 0, 0, 0);
            }
        }
    }
};

// One pipeline step: blend chunk q from r, refill r with chunk q + DEPTH (compile-time
// LOAD: the tail steps issue no loads), then the 4 (or 32 f32) MFMAs of chunk q.
#define SD_STEP(r, qq, LOAD)                                                  \
    do {                                                                      \
        typename Pr::Frag f_ = Pr::blend(r, geo.t);                           \
        if (LOAD) r = Pr::load(rs, o, (qq) + Pr::DEPTH);                      \
        Pr::mma1(lw, (qq), lane, f_, acc);                                    \
    } while (0)

// learn_empty (bts.py:311-319): a point outside the encoder frustum sees the learned
// empty feature e instead of its grid sample, so once the grid chunks are accumulated its
// column restarts from b_in + W_in[:, :C] e (LDS rows lds_be) before the code chunks.
__device__ __forceinline__ void sd_empty_sub(f32x16 acc[4], const float *lds_be, int h, bool inv) {
    if (__builtin_amdgcn_ballot_w64(inv) == 0) return;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const f32x4 *bb = (const f32x4 *)(lds_be + (t * 2 + h) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 b = bb[q];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[t][4 * q + i] = inv ? b[i] : acc[t][4 * q + i];
        }
    }
}

// First layer over all C/16 grid chunks + 3 code chunks, with a DEPTH-deep tap-load
// pipeline held in registers (C % (16 DEPTH) == 0).  acc holds the initial
// accumulator (b_in).  rs: buffer descriptor over this batch element's grid plane.
template <int P>
__device__ __forceinline__ void sd_layer1(__amdgpu_buffer_rsrc_t rs, int C, const PointGeo &geo,
                                          const uint8_t *lw, int lane, f32x16 acc[4],
                                          uint32_t base = 0, const float *lds_be = nullptr) {
    typedef Prec<P> Pr;
    const int h = lane >> 5;
    const int nq = C >> 4;
    const TapOff o = sd_tapoff(geo.t, C, Pr::ESZ, h, base);
    if constexpr (Pr::DEPTH == 4) {
        typename Pr::Raw r0 = Pr::load(rs, o, 0), r1 = Pr::load(rs, o, 1);
        typename Pr::Raw r2 = Pr::load(rs, o, 2), r3 = Pr::load(rs, o, 3);
        int q = 0;
        for (; q + 4 < nq; q += 4) {
            SD_STEP(r0, q, true);
            SD_STEP(r1, q + 1, true);
            SD_STEP(r2, q + 2, true);
            SD_STEP(r3, q + 3, true);
        }
        SD_STEP(r0, q, false);
        SD_STEP(r1, q + 1, false);
        SD_STEP(r2, q + 2, false);
        SD_STEP(r3, q + 3, false);
    } else {
        typename Pr::Raw r0 = Pr::load(rs, o, 0), r1 = Pr::load(rs, o, 1);
        int q = 0;
        for (; q + 2 < nq; q += 2) {
            SD_STEP(r0, q, true);
            SD_STEP(r1, q + 1, true);
        }
        SD_STEP(r0, q, false);
        SD_STEP(r1, q + 1, false);
    }
    if (lds_be) sd_empty_sub(acc, lds_be, h, geo.inv_f);
#pragma unroll
    for (int pc = 0; pc < SD_PE_CHUNKS; ++pc) {
        float f[8];
        sd_pe_chunk<Pr::FAST_PE>(geo.v, pc, h, f);
        Pr::mma1(lw, nq + pc, lane, Pr::from_f(f), acc);
    }
}

// acc <- b_in rows (initial accumulator), from LDS [t][h][16]
__device__ __forceinline__ void sd_init_bias(f32x16 acc[4], const float *lds_b, int h) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const f32x4 *bb = (const f32x4 *)(lds_b + (t * 2 + h) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 b = bb[q];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[t][4 * q + i] = b[i];
        }
    }
}

// ReLU in place; returns this lane half's part of w_sigma . h
__device__ __forceinline__ float sd_relu_sigma(f32x16 acc[4], const float *lds_ws, int h) {
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const f32x4 *ww = (const f32x4 *)(lds_ws + (t * 2 + h) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 w = ww[q];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float v = sd_relu(acc[t][4 * q + i]);
                acc[t][4 * q + i] = v;
                s = fmaf(v, w[i], s);
            }
        }
    }
    return s;
}

// LDS image: [W_in fragments | W_out fragments (if they fit) | b_in rows | w_sigma rows |
// learn_empty rows]
struct LdsPlan {
    int win_bytes, wout_bytes, wout_in_lds, total;
};

__device__ __forceinline__ void sd_stage(uint8_t *lds, const sd_mlp &m, const LdsPlan &pl) {
    const uint4 *src = (const uint4 *)m.w_in;
    uint4 *dst = (uint4 *)lds;
    for (int i = threadIdx.x; i < pl.win_bytes / 16; i += blockDim.x) dst[i] = src[i];
    if (pl.wout_in_lds) {
        const uint4 *s2 = (const uint4 *)m.w_out;
        uint4 *d2 = (uint4 *)(lds + pl.win_bytes);
        for (int i = threadIdx.x; i < pl.wout_bytes / 16; i += blockDim.x) d2[i] = s2[i];
    }
    float *fb = (float *)(lds + pl.win_bytes + (pl.wout_in_lds ? pl.wout_bytes : 0));
    for (int i = threadIdx.x; i < 128; i += blockDim.x) {
        fb[i] = m.b_in_h[i];
        fb[128 + i] = m.w_sig_h[i];
        if (m.b_empty_h) fb[256 + i] = m.b_empty_h[i];
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// fused render: one wave per ray at a time, K/32 sub-tiles ("items") of 32 samples,
// software-pipelined across items: while item i runs its MLP, the z values of item
// i+1 are in flight; after item i's grid chunks, item i+1's geometry is computed and
// its first DEPTH tap loads + colour taps are issued, so the epilogue of item i (code
// chunks, sigma, compositing, DINO head) hides their latency.
// ---------------------------------------------------------------------------
struct Item {
    int ray;
    int sub;
    float zk, delta, px, py, pz;
    PointGeo geo;
    TapOff o;
    __amdgpu_buffer_rsrc_t rs;
    int sbi;
};

template <int P, int NV, int NDT>
__global__ void __launch_bounds__(WG<P>::T, 1)
k_render(const sd_render_args a, const sd_mlp m, const LdsPlan pl) {
    typedef Prec<P> Pr;
    constexpr bool WL = P != SD_F32;  // 16-bit W_out fragments live in LDS, f32 in L2
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    sd_stage(lds, m, pl);
    const uint8_t *wout_base = WL ? lds + pl.win_bytes : (const uint8_t *)m.w_out;
    const float *lds_b = (const float *)(lds + pl.win_bytes + (WL ? pl.wout_bytes : 0));
    const float *lds_ws = lds_b + 128;

    const int lane = threadIdx.x & 63, h = lane >> 5, li = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = a.K, C = m.C, nv = NV > 0 ? NV : a.nv;
    const int nsub = K >> 5, nq = C >> 4;
    const uint32_t plane_bytes = (uint32_t)a.Hf * a.Wf * C * Pr::ESZ;
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;
    const int nwaves = gridDim.x * WG<P>::W;
    const int ray0 = blockIdx.x * WG<P>::W + wave;
    const int R = (int)a.R, rps = (int)a.rays_per_sb;
    if (ray0 >= R) return;
    const int nitems = ((R - ray0 + nwaves - 1) / nwaves) * nsub;

    // z and z_next of item c for this lane
    auto load_z = [&](const ItemCursor &c, float &z0, float &z1) {
        const int k = c.sub * 32 + li;
        const float *zr = a.z + (int64_t)c.ray * K;
        z0 = zr[k];
        z1 = zr[min(k + 1, K - 1)];
    };
    // geometry, buffer descriptor and tap offsets of item c (z already loaded)
    auto open_item = [&](const ItemCursor &c, float z0, float z1, Item &it) {
        it.ray = c.ray;
        it.sub = c.sub;
        it.sbi = c.sbi;
        const int k = it.sub * 32 + li;
        sd_cfloat *rr = (sd_cfloat *)(a.rays + (int64_t)c.ray * a.ray_dim);
        it.zk = z0;
        it.delta = (k + 1 < K) ? (z1 - z0) : 1e10f;
        it.px = rr[0] + z0 * rr[3];  // points = o + z d (nerf.py:252)
        it.py = rr[1] + z0 * rr[4];
        it.pz = rr[2] + z0 * rr[5];
        it.geo = sd_point_geo((sd_cfloat *)(a.cam_f + it.sbi * SD_CAM_WORDS), it.px, it.py, it.pz, a.Wf, a.Hf);
        it.rs = sd_rsrc((const uint8_t *)a.grid + (int64_t)it.sbi * plane_bytes, plane_bytes);
        it.o = sd_tapoff(it.geo.t, C, Pr::ESZ, h);
    };
    auto colours = [&](const Item &it, float col[3 * SD_MAX_NV], bool invc[SD_MAX_NV]) {
#pragma unroll
        for (int v = 0; v < SD_MAX_NV; ++v) {
            invc[v] = false;
            col[3 * v] = col[3 * v + 1] = col[3 * v + 2] = 0.f;
            if (v < nv)
                invc[v] = sd_color_view(a.cam_c + (it.sbi * nv + v) * SD_CAM_WORDS,
                                        a.img + (int64_t)(it.sbi * nv + v) * cplane, a.Wc, a.Hc, it.px,
                                        it.py, it.pz, col + 3 * v);
        }
    };

    // prologue: item 0
    const ItemCursor c0 = sd_cursor0(ray0, rps);
    ItemCursor c1 = sd_advance(c0, nsub, nwaves, R, rps);
    Item cur;
    float z0, z1;
    load_z(c0, z0, z1);
    open_item(c0, z0, z1, cur);
    typename Pr::Raw r0 = Pr::load(cur.rs, cur.o, 0), r1 = Pr::load(cur.rs, cur.o, 1);
    typename Pr::Raw r2, r3;
    if constexpr (Pr::DEPTH == 4) {
        r2 = Pr::load(cur.rs, cur.o, 2);
        r3 = Pr::load(cur.rs, cur.o, 3);
    }
    float col[3 * SD_MAX_NV];
    bool invc[SD_MAX_NV];
    colours(cur, col, invc);

    // per-ray compositing state
    f32x16 dacc[NDT];
#pragma unroll
    for (int i = 0; i < NDT; ++i) dacc[i] = f32x16{};
    float Tc = 1.f, dpart = 0.f, wpart = 0.f;
    float cpart[3 * SD_MAX_NV];
#pragma unroll
    for (int i = 0; i < 3 * SD_MAX_NV; ++i) cpart[i] = 0.f;

    for (int i = 0; i < nitems; ++i) {
        float zn0, zn1;
        load_z(c1, zn0, zn1);  // in flight during this item's MLP

        const int lo = sd_opaque0();
        const uint8_t *lw = lds + lo;
        f32x16 acc[4];
        sd_init_bias(acc, lds_b + lo, h);
        {
            const PointGeo &geo = cur.geo;
            const __amdgpu_buffer_rsrc_t rs = cur.rs;
            const TapOff o = cur.o;
            if constexpr (Pr::DEPTH == 4) {
                int q = 0;
                for (; q + 4 < nq; q += 4) {
                    SD_STEP(r0, q, true);
                    SD_STEP(r1, q + 1, true);
                    SD_STEP(r2, q + 2, true);
                    SD_STEP(r3, q + 3, true);
                }
                SD_STEP(r0, q, false);
                SD_STEP(r1, q + 1, false);
                SD_STEP(r2, q + 2, false);
                SD_STEP(r3, q + 3, false);
            } else {
                int q = 0;
                for (; q + 2 < nq; q += 2) {
                    SD_STEP(r0, q, true);
                    SD_STEP(r1, q + 1, true);
                }
                SD_STEP(r0, q, false);
                SD_STEP(r1, q + 1, false);
            }
        }

        // open the next item and put its first tap loads in flight
        Item nxt;
        open_item(c1, zn0, zn1, nxt);
        c1 = sd_advance(c1, nsub, nwaves, R, rps);
        r0 = Pr::load(nxt.rs, nxt.o, 0);
        r1 = Pr::load(nxt.rs, nxt.o, 1);
        if constexpr (Pr::DEPTH == 4) {
            r2 = Pr::load(nxt.rs, nxt.o, 2);
            r3 = Pr::load(nxt.rs, nxt.o, 3);
        }

        if (m.b_empty_h) sd_empty_sub(acc, lds_ws + 128 + lo, h, cur.geo.inv_f);
        // positional-code chunks of this item
#pragma unroll
        for (int pc = 0; pc < SD_PE_CHUNKS; ++pc) {
            float f[8];
            sd_pe_chunk<Pr::FAST_PE>(cur.geo.v, pc, h, f);
            Pr::mma1(lw, nq + pc, lane, Pr::from_f(f), acc);
        }

        float s = sd_relu_sigma(acc, lds_ws + lo, h);
        s += __shfl_xor(s, 32);
        const float sigma = sd_softplus(s + m.b_sigma);

        // alpha compositing (nerf.py:376-389); transmittance = prefix product
        const int k = cur.sub * 32 + li;
        float alpha = 1.f - expf(-fabsf(cur.delta) * fmaxf(sigma, 0.f));
        if (a.hard_alpha_cap && k == K - 1) alpha = 1.f;
        const float tk = (1.f - alpha) + 1e-10f;
        float incl = tk;
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) {
            float v = __shfl_up(incl, d, 32);
            if (li >= d) incl *= v;
        }
        float excl = __shfl_up(incl, 1, 32);
        if (li == 0) excl = 1.f;
        const float w = alpha * (Tc * excl);
        Tc *= __shfl(incl, 31, 32);
        dpart += w * cur.zk;
        wpart += w;
#pragma unroll
        for (int v = 0; v < SD_MAX_NV; ++v)
            if (v < nv) {
                cpart[3 * v] += w * col[3 * v];
                cpart[3 * v + 1] += w * col[3 * v + 1];
                cpart[3 * v + 2] += w * col[3 * v + 2];
            }

        // DINO head folded into the compositing sum: dacc += (w h)^T W_out^T
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] *= w;
        const uint8_t *wo = wout_base + (WL ? lo : 0);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) Pr::mma2(wo, dt, acc, lane, dacc[dt]);

        // per-sample outputs, coalesced along the ray
        const int64_t o = (int64_t)cur.ray * K + k;
        if (h == 0) {
            if (a.weights) a.weights[o] = w;
            if (a.alphas) a.alphas[o] = alpha;
            if (a.invalid_f) a.invalid_f[o] = cur.geo.inv_f ? 1 : 0;
        } else {
#pragma unroll
            for (int v = 0; v < SD_MAX_NV; ++v)
                if (v < nv) {
                    if (a.invalid) a.invalid[o * nv + v] = (invc[v] | cur.geo.inv_f) ? 1.f : 0.f;
                    if (a.rgb_samps) {
                        float *rsp = a.rgb_samps + (o * nv + v) * 3;
                        rsp[0] = col[3 * v]; rsp[1] = col[3 * v + 1]; rsp[2] = col[3 * v + 2];
                    }
                }
        }

        if (cur.sub == nsub - 1) {
            // ray epilogue: reduce the per-lane partial sums over the 32 lanes of a half
#pragma unroll
            for (int d = 1; d < 32; d <<= 1) {
                dpart += __shfl_xor(dpart, d);
                wpart += __shfl_xor(wpart, d);
#pragma unroll
                for (int c = 0; c < 3 * SD_MAX_NV; ++c)
                    if (c < 3 * nv) cpart[c] += __shfl_xor(cpart[c], d);
            }
            // dino[dim] = sum over rows of dacc (+ other half) + wsum * b
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                float sacc = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) sacc += dacc[dt][r];
                sacc += __shfl_xor(sacc, 32);
                if ((dt & 1) == h) {
                    const int dim = dt * 32 + li;
                    a.dino[(int64_t)cur.ray * m.D + dim] = sacc + wpart * m.b_dino[dim];
                }
                dacc[dt] = f32x16{};
            }
            if (lane == 0) a.depth[cur.ray] = dpart;
            if (lane < 3 * nv) {
                float cv = 0.f;
#pragma unroll
                for (int c = 0; c < 3 * SD_MAX_NV; ++c)
                    if (c == lane) cv = cpart[c];
                a.rgb[(int64_t)cur.ray * 3 * nv + lane] = cv;
            }
            Tc = 1.f; dpart = 0.f; wpart = 0.f;
#pragma unroll
            for (int c = 0; c < 3 * SD_MAX_NV; ++c) cpart[c] = 0.f;
        }

        // colours of the next item (its loads were issued with its taps above)
        colours(nxt, col, invc);
        cur = nxt;
    }
}

// ---------------------------------------------------------------------------
// per-point field query (no compositing): 32 consecutive points per wave step,
// software-pipelined across tiles like k_render's items: the next tile's points are
// loaded during this tile's grid chunks, and once those chunks are accumulated the next
// tile's geometry is computed and its first DEPTH tap loads are issued, so this tile's code
// chunks, sigma, output layer and stores run under their latency (a tile at a time left
// every tap gather's L2 / Infinity-Cache round trip exposed: ~9x the tile's MFMA time)
// ---------------------------------------------------------------------------
#ifndef SD_FQ_ABL_ONETAP
#define SD_FQ_ABL_ONETAP 0
#endif
// diagnostic build only (SD_FQ_PROF=1): per-phase s_memtime cycles of k_field summed over all
// waves (tools/field_prof.py); the outputs are unchanged
#ifndef SD_FQ_PROF
#define SD_FQ_PROF 0
#endif
#if SD_FQ_PROF
__device__ unsigned long long fq_prof[8];
#define FQ_T(i)                                                  \
    {                                                            \
        const uint64_t _t = __builtin_amdgcn_s_memtime();        \
        pacc[i] += (uint32_t)(_t - tlast);                       \
        tlast = _t;                                              \
    }
extern "C" int sd_field_prof(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fq_prof), sizeof(fq_prof)) != hipSuccess) return -2;
    if (reset) {
        unsigned long long z[8] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(fq_prof), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define FQ_T(i)
#endif
#ifndef SD_FQ_ABL_NOSTORE
#define SD_FQ_ABL_NOSTORE 0
#endif
// WL: the W_out fragments staged in LDS (16-bit, when they fit beside W_in: D <= 128 at
// C = 256, any D <= 512 on the projected grid's 128 columns), else read from L2 (f32, and
// 16-bit 384-d heads over a 256-channel grid)
// DEF (bf16 dino, D <= 64: the SSCBench query feeding sd_seg_query): a tile's outputs leave
// in the NEXT tile's grid phase, once its tap loads are issued.  Stores count in vmcnt
// like loads and retire in order with them, so a tap load issued behind a tile's 32
// row stores waits for their acknowledgements too; issued behind the loads, the stores
// have a whole tile of MLP work to complete before the next wait that includes them.
template <int P, bool WL, bool DEF = false>
__global__ void __launch_bounds__(WG<P>::T, 1)
k_field(const sd_field_args a, const sd_mlp m, const LdsPlan pl) {
    typedef Prec<P> Pr;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    sd_stage(lds, m, pl);
    const uint8_t *wout_base = WL ? lds + pl.win_bytes : (const uint8_t *)m.w_out;
    const float *lds_b = (const float *)(lds + pl.win_bytes + (WL ? pl.wout_bytes : 0));
    const float *lds_ws = lds_b + 128;

    const int lane = threadIdx.x & 63, h = lane >> 5, li = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t NP = a.B * a.P;
    const int64_t ntiles = (NP + 31) / 32;
    const int C = m.C, nv = a.nv, nq = C >> 4;
    const int ndt = m.D >> 5;
    const uint32_t plane_bytes = (uint32_t)a.Hf * a.Wf * C * Prec<P>::ESZ;
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;
    // one descriptor over all batch planes (host checks B * plane < 4 GiB)
    const __amdgpu_buffer_rsrc_t rs = sd_rsrc(a.grid, (uint32_t)(a.B * (int64_t)plane_bytes));
    // the dino output (NP x D, f32 or bf16; < 4 GiB, checked by the host)
    const __amdgpu_buffer_rsrc_t rdino =
        sd_rsrc(a.dino, (uint32_t)(NP * m.D * (a.dino_dtype == SD_BF16 ? 2 : 4)));

    // XCD-aware tile ranges (workgroups b, b + 8, ... share an XCD: speed only): XCD x
    // visits tiles [x T / 8, (x + 1) T / 8) of the (optionally locality-sorted) order, its
    // workgroups interleaved, so a tile's grid taps are fetched into one XCD's L2
    const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
    const int xcd = blockIdx.x % nx, nwg = gridDim.x / nx;
    const int64_t tend = ntiles * (xcd + 1) / nx;
    const int64_t tstep = (int64_t)nwg * WG<P>::W;
    int64_t tt = ntiles * xcd / nx + (int64_t)(blockIdx.x / nx) * WG<P>::W + wave;
    if (tt >= tend) return;

    struct FTile {
        int64_t p, b;
        bool valid;
        float px, py, pz;
        PointGeo geo;
        TapOff o;
    };
    auto tile_of = [&](int64_t t) { return a.tile_order ? (int64_t)a.tile_order[t] : t; };
    auto load_pts = [&](int64_t t, float &x, float &y, float &z) {
        const int64_t pu = tile_of(t) * 32 + li;
        const int64_t p = pu < NP ? pu : NP - 1;
        x = a.xyz[p * 3];
        y = a.xyz[p * 3 + 1];
        z = a.xyz[p * 3 + 2];
    };
    auto open_tile = [&](int64_t t, float x, float y, float z, FTile &f) {
        const int64_t pu = tile_of(t) * 32 + li;
        f.valid = pu < NP;
        f.p = f.valid ? pu : NP - 1;
        f.b = f.p / a.P;
        f.px = x; f.py = y; f.pz = z;
        f.geo = sd_point_geo(a.cam_f + f.b * SD_CAM_WORDS, x, y, z, a.Wf, a.Hf);
        f.o = sd_tapoff(f.geo.t, C, Pr::ESZ, h, (uint32_t)(f.b * plane_bytes));
#if SD_FQ_ABL_ONETAP  // diagnostic (outputs wrong): every tap reads texel 00
        f.o.o01 = f.o.o10 = f.o.o11 = f.o.o00;
#endif
    };

    // the output biases of this lane's dims, loaded once: read in the output phase, the
    // load waited (in-order vmcnt) for the next tile's tap loads issued before it
    float bdino[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) bdino[dt] = dt < ndt ? m.b_dino[dt * 32 + li] : 0.f;
    // prologue: tile tt opened, its first DEPTH tap loads and the next tile's points in flight
    FTile cur;
    {
        float x, y, z;
        load_pts(tt, x, y, z);
        open_tile(tt, x, y, z, cur);
    }
    typename Pr::Raw r0 = Pr::load(rs, cur.o, 0), r1 = Pr::load(rs, cur.o, 1);
    typename Pr::Raw r2, r3;
    if constexpr (Pr::DEPTH == 4) {
        r2 = Pr::load(rs, cur.o, 2);
        r3 = Pr::load(rs, cur.o, 3);
    }
#if SD_FQ_PROF
    uint32_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tlast = __builtin_amdgcn_s_memtime();
#endif
    // DEF: the previous tile's outputs wait in this wave's 4-KiB LDS block (the tile's
    // 32 rows of D bf16, as in HBM: one contiguous 64 D-byte run), its sigma and frustum
    // flag in registers, until flush() copies the block out with 16-byte stores
    uint16_t *scr = (uint16_t *)(lds + pl.total - WG<P>::W * 4096 + wave * 4096);
    float pend_sig = 0.f;
    int64_t pend_tile = -1, pend_p = 0;
    bool pend_ok = false, pend_inv = false;
    auto flush = [&]() __attribute__((always_inline)) {
        if (pend_tile < 0) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t vo = (uint32_t)(pend_tile * 64 * m.D);
        for (int k = 0; k < (m.D >> 4); ++k) {  // 64 D bytes = D / 16 rounds of 64 x 16 B
            const uint32_t off = (uint32_t)(k * 64 + lane) * 16u;
            typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
            const u32x4v v = *(const u32x4v *)((const uint8_t *)scr + off);
            __builtin_amdgcn_raw_buffer_store_b128(v, rdino, vo + off, 0, 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (pend_ok && h == 0) {
            a.sigma[pend_p] = pend_sig;
            if (a.invalid_f) a.invalid_f[pend_p] = pend_inv ? 1 : 0;
        }
    };
    for (; tt < tend; tt += tstep) {
        const int64_t tn = tt + tstep;
        const bool more = tn < tend;
        float nx0 = 0.f, ny0 = 0.f, nz0 = 0.f;
        if (more) load_pts(tn, nx0, ny0, nz0);  // in flight during this tile's grid chunks
        FQ_T(5);

        const int lo = sd_opaque0();
        const uint8_t *lw = lds + lo;
        f32x16 acc[4];
        sd_init_bias(acc, lds_b + lo, h);
        {
            const PointGeo &geo = cur.geo;
            const TapOff o = cur.o;
            if constexpr (Pr::DEPTH == 4) {
                int q = 0;
                for (; q + 4 < nq; q += 4) {
                    SD_STEP(r0, q, true);
                    SD_STEP(r1, q + 1, true);
                    SD_STEP(r2, q + 2, true);
                    SD_STEP(r3, q + 3, true);
                }
                if (DEF) {  // every tap load of this tile issued: the previous tile's stores
                    flush();
                    pend_tile = -1;
                }
                SD_STEP(r0, q, false);
                SD_STEP(r1, q + 1, false);
                SD_STEP(r2, q + 2, false);
                SD_STEP(r3, q + 3, false);
            } else {
                int q = 0;
                for (; q + 2 < nq; q += 2) {
                    SD_STEP(r0, q, true);
                    SD_STEP(r1, q + 1, true);
                }
                SD_STEP(r0, q, false);
                SD_STEP(r1, q + 1, false);
            }
        }
        FQ_T(0);
        // open the next tile and put its first tap loads in flight
        FTile nxt;
        if (more) {
            open_tile(tn, nx0, ny0, nz0, nxt);
            r0 = Pr::load(rs, nxt.o, 0);
            r1 = Pr::load(rs, nxt.o, 1);
            if constexpr (Pr::DEPTH == 4) {
                r2 = Pr::load(rs, nxt.o, 2);
                r3 = Pr::load(rs, nxt.o, 3);
            }
        }

        FQ_T(1);
        if (m.b_empty_h) sd_empty_sub(acc, lds_ws + 128 + lo, h, cur.geo.inv_f);
#pragma unroll
        for (int pc = 0; pc < SD_PE_CHUNKS; ++pc) {
            float f[8];
            sd_pe_chunk<Pr::FAST_PE>(cur.geo.v, pc, h, f);
            Pr::mma1(lw, nq + pc, lane, Pr::from_f(f), acc);
        }
        float s = sd_relu_sigma(acc, lds_ws + lo, h);
        s += __shfl_xor(s, 32);
        const float sigma = sd_softplus(s + m.b_sigma);

        FQ_T(2);
        const uint8_t *wo = wout_base + (WL ? lo : 0);
        const int64_t tile = tile_of(tt);
        // one 32-dim tile of the DINO output: 8 (f32: 32) MFMAs + 16 row stores
        auto out_tile = [&](int dt, float bd) __attribute__((always_inline)) {
            f32x16 ov = {};
            Prec<P>::mma2(wo, dt, acc, lane, ov);
            // O layout: row = point (r&3)+8(r>>2)+4h of this tile, column = dim li
            const int dim = dt * 32 + li;
            if (DEF) {
                // the previous tile's block left in flush(), before this tile's grid chunks
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    scr[((r & 3) + 8 * (r >> 2) + 4 * h) * m.D + dim] =
                        __builtin_bit_cast(uint16_t, (__bf16)(ov[r] + bd));
            } else if (SD_FQ_ABL_NOSTORE) {
                if (ov[0] == 12345.f) a.dino[tile] = ov[1];  // keep the product alive
            } else {
                // buffer stores at per-lane byte offsets (row, column dim): rows past the
                // last point fall outside the descriptor's range (the range check covers the
                // vector + instruction offset, not the scalar one: the row goes in the
                // vector offset) and are dropped -- no bounds test per store
                const uint32_t esz = a.dino_dtype == SD_BF16 ? 2u : 4u;
                const uint32_t vo = (uint32_t)(((tile * 32 + 4 * h) * m.D + dim) * esz);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint32_t ro = vo + (uint32_t)(((r & 3) + 8 * (r >> 2)) * m.D) * esz;
                    if (a.dino_dtype == SD_BF16)
                        __builtin_amdgcn_raw_buffer_store_b16(
                            __builtin_bit_cast(uint16_t, (__bf16)(ov[r] + bd)), rdino, ro, 0, 0);
                    else
                        __builtin_amdgcn_raw_buffer_store_b32(
                            __builtin_bit_cast(uint32_t, ov[r] + bd), rdino, ro, 0, 0);
                }
            }
        };
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            if (dt >= ndt) break;
            out_tile(dt, bdino[dt]);
        }
        // wide heads (configs[3]: D = 384): the tiles past the 4 with register-cached biases
        if (!DEF)
            for (int dt = 4; dt < ndt; ++dt) out_tile(dt, m.b_dino[dt * 32 + li]);
        FQ_T(3);
        if (DEF) {
            pend_tile = tile;
            pend_p = cur.p;
            pend_ok = cur.valid;
            pend_sig = sigma;
            pend_inv = cur.geo.inv_f;
        } else if (cur.valid && h == 0) {
            a.sigma[cur.p] = sigma;
            if (a.invalid_f) a.invalid_f[cur.p] = cur.geo.inv_f ? 1 : 0;
        }
        if (cur.valid && h == 1 && nv > 0 && (a.rgb || a.invalid)) {
            for (int v = 0; v < nv; ++v) {
                float col[3];
                bool ic = sd_color_view(a.cam_c + (cur.b * nv + v) * SD_CAM_WORDS,
                                        a.img + (cur.b * nv + v) * cplane, a.Wc, a.Hc, cur.px,
                                        cur.py, cur.pz, col);
                if (a.rgb) {
                    a.rgb[(cur.p * nv + v) * 3] = col[0];
                    a.rgb[(cur.p * nv + v) * 3 + 1] = col[1];
                    a.rgb[(cur.p * nv + v) * 3 + 2] = col[2];
                }
                if (a.invalid) a.invalid[cur.p * nv + v] = (ic | cur.geo.inv_f) ? 1.f : 0.f;
            }
        }
        if (more) cur = nxt;
        FQ_T(4);
    }
    if (DEF) flush();  // the last tile's outputs
#if SD_FQ_PROF
    if (lane == 0)
        for (int i = 0; i < 8; ++i) atomicAdd(&fq_prof[i], (unsigned long long)pacc[i]);
#endif
}

// ---------------------------------------------------------------------------
// standalone compositor: one wave per ray, lane = feature column (sequential in k)
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
    if (K <= 32 && nf <= 1) {
        // every load first (lane k: z, sigma of sample k; the K feature / colour values of
        // the lane's column), the recurrence over k in registers (readlane broadcasts, the
        // same products in the same order), every store at the end: the loop used to store
        // the weights / alphas of sample k before loading sample k + 1, one memory round
        // trip per sample
        const float zl = lane < K ? zr[lane] : 0.f;
        const float zn = lane + 1 < K ? zr[lane + 1] : 0.f;
        const float sl = lane < K ? sr[lane] : 0.f;
        float fv[32], cv[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            fv[k] = (feat && k < K && lane < F) ? feat[(ray * K + k) * F + lane] : 0.f;
            cv[k] = (rgb && k < K && lane < Cc) ? rgb[(ray * K + k) * Cc + lane] : 0.f;
        }
        const float delta = (lane + 1 < K) ? zn - zl : 1e10f;
        float alpha = 1.f - expf(-fabsf(delta) * fmaxf(sl, 0.f));
        if (hard_cap && lane == K - 1) alpha = 1.f;
        float wl = 0.f;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if (k >= K) break;
            const float ak = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, alpha), k));
            const float zk = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, zl), k));
            const float w = ak * T;
            T = T * ((1.f - ak) + 1e-10f);
            dep += w * zk;
            if (lane == k) wl = w;
            if (feat) facc[0] += fv[k] * w;
            if (rgb) cacc += w * cv[k];
        }
        if (lane < K) {
            if (weights) weights[ray * K + lane] = wl;
            if (alphas) alphas[ray * K + lane] = alpha;
        }
        if (lane == 0 && depth) depth[ray] = dep;
        if (feat && feat_out && lane < F) feat_out[ray * F + lane] = facc[0];
        if (rgb && rgb_out && lane < Cc) rgb_out[ray * Cc + lane] = cacc;
        return;
    }
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
static int sd_plan(const sd_mlp *m, LdsPlan *pl) {
    if (!m || !m->w_in || !m->b_in_h || !m->w_sig_h || !m->w_out || !m->b_dino) {
        sd_set_error("sd_mlp: null parameter pointer");
        return -1;
    }
    if (m->d_hidden != SD_DH || m->C <= 0 || (m->C % 64) || m->D <= 0 || (m->D % 32) || m->D > 512 ||
        (m->dtype != SD_BF16 && m->dtype != SD_F32 && m->dtype != SD_F16)) {
        sd_set_error("sd_mlp: unsupported shape (need d_hidden=128, C%64==0, D%32==0, D<=512)");
        return -1;
    }
    int nq = m->C / 16 + SD_PE_CHUNKS;
    int esz = m->dtype == SD_F32 ? 4 : 2;
    pl->win_bytes = nq * 4 * SD_WAVE * 8 * esz;
    pl->wout_bytes = (m->D / 32) * 4 * SD_WAVE * (m->dtype == SD_F32 ? 64 : 32);
    int rest = 384 * 4;  // b_in, w_sigma, learn_empty rows
    // 16-bit W_out fragments in LDS when they fit beside W_in (always for D <= 128 at
    // C <= 256, sd_render_fused's range); otherwise k_field reads them from L2 like f32
    pl->wout_in_lds = m->dtype != SD_F32 && pl->win_bytes + pl->wout_bytes + rest <= 160 * 1024;
    pl->total = pl->win_bytes + (pl->wout_in_lds ? pl->wout_bytes : 0) + rest;
    if (pl->total > 160 * 1024) {
        sd_set_error("sd_mlp: MLP fragments exceed the 160 KiB LDS (C or D too large)");
        return -1;
    }
    return 0;
}

// Persistent grid: one workgroup per CU (fewer if there is less work); every wave
// strides over its work units.
template <int P, typename KernT, typename ArgT>
static int sd_launch(KernT kern, int64_t work_waves, const LdsPlan &pl, hipStream_t s,
                     const ArgT &a, const sd_mlp &m) {
    int64_t nblk = (work_waves + WG<P>::W - 1) / WG<P>::W;
    if (nblk > sd_num_cus()) nblk = sd_num_cus();
    sd_lds_attr((const void *)kern, 160 * 1024);
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(WG<P>::T), pl.total, s, a, m, pl);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        return -2;
    }
    return 0;
}

template <int P, int NV>
static int sd_render_ndt(const sd_render_args &a, const sd_mlp &m, const LdsPlan &pl,
                         hipStream_t s) {
    switch (m.D / 32) {
        case 1: return sd_launch<P>(k_render<P, NV, 1>, a.R, pl, s, a, m);
        case 2: return sd_launch<P>(k_render<P, NV, 2>, a.R, pl, s, a, m);
        case 4: return sd_launch<P>(k_render<P, NV, 4>, a.R, pl, s, a, m);
        default:
            sd_set_error("sd_render_fused: D must be 32, 64 or 128 (use sd_field_query + sd_composite)");
            return -1;
    }
}

template <int P>
static int sd_render_nv(const sd_render_args &a, const sd_mlp &m, const LdsPlan &pl,
                        hipStream_t s) {
    return a.nv == 1 ? sd_render_ndt<P, 1>(a, m, pl, s) : sd_render_ndt<P, 0>(a, m, pl, s);
}

extern "C" int sd_render_fused(const sd_render_args *args, const sd_mlp *mlp, void *stream) {
    LdsPlan pl;
    if (!args) {
        sd_set_error("sd_render_fused: null args");
        return -1;
    }
    if (sd_plan(mlp, &pl)) return -1;
    const sd_render_args &a = *args;
    if (a.grid_dtype != sd_field_dtype(mlp->dtype)) {
        sd_set_error("sd_render_fused: grid_dtype must be sd_field_dtype(mlp->dtype) (f16 for "
                     "both 16-bit modes)");
        return -1;
    }
    if (mlp->dtype != SD_F32 && !pl.wout_in_lds) {  // k_render stages 16-bit W_out in LDS
        sd_set_error("sd_render_fused: 16-bit MLP fragments exceed the 160 KiB LDS (C too large)");
        return -1;
    }
    if (a.ld_depth || a.ld_dino || a.ld_rgb) {
        sd_set_error("sd_render_fused: output row strides are not supported (must be 0)");
        return -1;
    }
    if (a.R < 0 || a.R >= (1LL << 31) || a.K <= 0 || (a.K % 32) || a.ray_dim < 6 ||
        a.rays_per_sb <= 0 || !a.rays ||
        !a.z || !a.grid || !a.cam_f || !a.depth || !a.dino || a.Hf <= 0 || a.Wf <= 0 ||
        a.nv < 0 || a.nv > SD_MAX_NV || mlp->D > 128 ||
        (int64_t)a.Hf * a.Wf * mlp->C * (mlp->dtype == SD_F32 ? 4 : 2) >= (1LL << 32) ||
        (a.nv > 0 && (!a.img || !a.cam_c || !a.rgb || a.Hc <= 0 || a.Wc <= 0))) {
        sd_set_error("sd_render_fused: invalid argument (K % 32 == 0, nv <= 4, D <= 128, "
                     "grid plane < 4 GiB)");
        return -1;
    }
    if (a.R == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (mlp->dtype == SD_F16) return sd_render_nv<SD_F16>(a, *mlp, pl, s);
    if (mlp->dtype == SD_BF16) return sd_render_nv<SD_BF16>(a, *mlp, pl, s);
    return sd_render_nv<SD_F32>(a, *mlp, pl, s);
}

extern "C" int sd_field_query(const sd_field_args *args, const sd_mlp *mlp, void *stream) {
    LdsPlan pl;
    if (!args) {
        sd_set_error("sd_field_query: null args");
        return -1;
    }
    if (sd_plan(mlp, &pl)) return -1;
    const sd_field_args &a = *args;
    if (a.grid_dtype != sd_field_dtype(mlp->dtype)) {
        sd_set_error("sd_field_query: grid_dtype must be sd_field_dtype(mlp->dtype) (f16 for "
                     "both 16-bit modes)");
        return -1;
    }
    if (a.B <= 0 || a.P < 0 || !a.xyz || !a.grid || !a.cam_f || !a.sigma || !a.dino ||
        a.Hf <= 0 || a.Wf <= 0 || a.nv < 0 || a.nv > SD_MAX_NV ||
        (a.dino_dtype != SD_F32 && a.dino_dtype != SD_BF16) ||
        // the dino rows of the last 32-point tile's padding lanes are dropped by the buffer
        // descriptor's range check: their offsets must not wrap, so the bound is on the padded count
        (a.B * a.P + 31) / 32 * 32 * (int64_t)mlp->D * (a.dino_dtype == SD_BF16 ? 2 : 4) >= (1LL << 32) ||
        a.B * (int64_t)a.Hf * a.Wf * mlp->C * (mlp->dtype == SD_F32 ? 4 : 2) >= (1LL << 32) ||
        (a.nv > 0 && (a.rgb || a.invalid) && (!a.img || !a.cam_c || a.Hc <= 0 || a.Wc <= 0))) {
        sd_set_error("sd_field_query: invalid argument (all grid planes < 4 GiB)");
        return -1;
    }
    if (a.P == 0) return 0;
    const int64_t ntiles = (a.B * a.P + 31) / 32;
    hipStream_t s = (hipStream_t)stream;
#ifndef SD_FQ_DEFER
#define SD_FQ_DEFER 1
#endif
    // (k_field DEF: + one 4-KiB output block per wave after the plan's LDS image)
    LdsPlan pd = pl;
    pd.total += WG<SD_F16>::W * 4096;
    if (SD_FQ_DEFER && mlp->dtype != SD_F32 && pl.wout_in_lds && a.dino_dtype == SD_BF16 &&
        mlp->D <= 64 && pd.total <= 160 * 1024)
        return mlp->dtype == SD_F16 ? sd_launch<SD_F16>(k_field<SD_F16, true, true>, ntiles, pd, s, a, *mlp)
                                    : sd_launch<SD_BF16>(k_field<SD_BF16, true, true>, ntiles, pd, s, a, *mlp);
    if (mlp->dtype == SD_F16)
        return pl.wout_in_lds ? sd_launch<SD_F16>(k_field<SD_F16, true>, ntiles, pl, s, a, *mlp)
                              : sd_launch<SD_F16>(k_field<SD_F16, false>, ntiles, pl, s, a, *mlp);
    if (mlp->dtype == SD_BF16)
        return pl.wout_in_lds ? sd_launch<SD_BF16>(k_field<SD_BF16, true>, ntiles, pl, s, a, *mlp)
                              : sd_launch<SD_BF16>(k_field<SD_BF16, false>, ntiles, pl, s, a, *mlp);
    return sd_launch<SD_F32>(k_field<SD_F32, false>, ntiles, pl, s, a, *mlp);
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
