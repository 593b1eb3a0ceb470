// sdhip_proj.hip -- projected-grid feature-field render (gfx950 / CDNA4, 16-bit modes).
//
// F.grid_sample (bilinear, border, align_corners=False; bts.py:299-309) is linear in
// the grid and its four weights sum to one, so the grid columns of ResnetFC's first
// layer (resnetfc.py:163) commute with the gather:
//     W_in[:, :C] . sample(G, xy) + b_in  ==  sample(P, xy),   P = W_in[:, :C] . G + b_in.
// k_project evaluates P once per grid pixel (B*Hf*Wf x 128 x C MFMA GEMM, HBM-bound on
// reading G); k_render_proj gathers 4 taps x 128 P channels per sample (half of the
// C = 256 grid channels) and needs only the 39 code columns per sample on the matrix
// cores: the per-sample first-layer contraction drops from K = 295 to K = 39.
//
// Render work unit: one wave = one ray at a time, in items of 16 consecutive samples
// (16x16x32 MFMA; lane l: sample j = l & 15, group g = l >> 4).  Per item:
//   hidden (16 x 16 tile t = rows 16t..16t+15, 8 tiles) =
//       I . blend(P taps)            one identity MFMA per tile (chunk q = t / 2)
//     + W_code . code                2 code chunks x 8 tiles
//   -> ReLU -> 16-bit X fragments (accumulator-as-operand: element e of fragment s of
//      group g is hidden 32 s + 16 (e >> 2) + 4 g + (e & 3))
//   sigma^T  = W_sigma . X^T         4 MFMAs, every row = sigma of sample j
//   dino^T   = W_dino  . X^T         4 MFMAs per 16 dims, weighted by w_j and summed
//                                    over the ray's samples in registers.
// Compositing (nerf.py:376-405): alpha, DPP prefix product of (1-alpha+1e-10) over the
// 16 samples of an item (+ carry across items), weights, depth, colour (group g
// samples render view g), DINO; the ray epilogue reduces over the 16 sample lanes.
// Pipelining: the z values of item i+2 and the P-tap loads of item i+1 are in flight
// while item i computes.
#include "sdhip_render.h"
#include <stdlib.h>
#include <type_traits>

// diagnostic ablation switches (timing experiments only; outputs are wrong when set)
#ifndef SD_ABL_NORAYPASS
#define SD_ABL_NORAYPASS 0
#endif
#ifndef SD_ABL_NOBLEND
#define SD_ABL_NOBLEND 0
#endif
#ifndef SD_ABL_NOPE
#define SD_ABL_NOPE 0
#endif
#ifndef SD_ABL_NODINO
#define SD_ABL_NODINO 0
#endif
#ifndef SD_PWG
#define SD_PWG 256  // threads per workgroup (4 waves); several workgroups per CU
#endif


// ---------------------------------------------------------------------------
// k_project: P[b][pix][n] = sum_c W_in[n][c] G[b][c][pix] + b_in[n]   (n < 128), stored
// plain (B, Hf, Wf, 128) in the 16-bit MLP dtype: 256 B per grid pixel, so the two
// horizontal bilinear taps of a sample (x0, x0 + 1) are 512 contiguous bytes.  One wave =
// 32 pixel columns x 128 hidden = 4 tiles of 32x32x16, K = C in chunks of 16.
// A = the sd_mlp layer-1 fragments of the grid columns (LDS); B = 8 channels of the
// lane's pixel read from NCHW (32 consecutive floats per channel across a half) or, NHWC
// (the native encoder's channels-last grid), as two 16-B loads of the pixel's row.
// ---------------------------------------------------------------------------
// waves per SIMD the channels-last k_project's register budget is cut for (1: the compiler's
// choice, 176 VGPRs = 2 waves per SIMD).  3 (167 VGPRs, no spill) measured the same time
// (C2 50-53 us either way, tools/proj_ab.sh): more resident waves do not move this kernel
#ifndef SD_PROJ_STAGE
#define SD_PROJ_STAGE 1  // output tile staged through LDS for whole-row 16-B stores (0: 8-B scatter)
#endif
#ifndef SD_PROJ_WPE
#define SD_PROJ_WPE 1
#endif
template <int P, bool NHWC, bool HILO>
__global__ void __launch_bounds__(SD_PWG) __attribute__((amdgpu_waves_per_eu(NHWC ? SD_PROJ_WPE : 1)))
k_project(const float *__restrict__ grid, int64_t B, int C, int64_t HW, int W, const sd_mlp m,
          uint32_t *__restrict__ out) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int nq = C >> 4;
    {
        const uint4 *src = (const uint4 *)m.w_in;
        uint4 *dst = (uint4 *)lds;
        for (int i = threadIdx.x; i < nq * 4 * SD_WAVE; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    const Frag *lw = (const Frag *)lds;
    const int lane = threadIdx.x & 63, h = lane >> 5, li = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t ntile = (HW + 31) / 32, total = B * ntile;
    for (int64_t task = (int64_t)blockIdx.x * (SD_PWG / 64) + wave; task < total;
         task += (int64_t)gridDim.x * (SD_PWG / 64)) {
        const int64_t b = task / ntile;
        const int64_t pix = (task - b * ntile) * 32 + li;
        const bool valid = pix < HW;
        const int64_t pc = pix < HW ? pix : HW - 1;
        // channel c of this lane's pixel: gp[c * cs]
        const int64_t cs = NHWC ? 1 : HW;
        const float *gp = NHWC ? grid + (b * HW + pc) * C + 8 * h : grid + b * C * HW + pc + (int64_t)(8 * h) * HW;
        f32x16 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const f32x4 *bb = (const f32x4 *)(m.b_in_h + (t * 2 + h) * 16);
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                f32x4 v = bb[q4];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[t][4 * q4 + i] = v[i];
            }
        }
        // two K steps of grid loads in flight (x0: step q, x1: step q + 1): the kernel
        // is HBM-bound and one step per wave does not cover the latency
        float x0[8], x1[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x0[e] = gp[e * cs];
        if (nq > 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) x1[e] = gp[16 * cs + e * cs];
        }
        auto kstep = [&](int q, float (&x)[8]) {
            // HILO: the f32 grid as a hi + lo pair of 16-bit operands (see k_project_lds)
            Frag f, fl;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                f[e] = (typename Tr::E)x[e];
                if (HILO) fl[e] = (typename Tr::E)(x[e] - (float)f[e]);
            }
            if (q + 2 < nq) {
                const float *gn = gp + (int64_t)(16 * (q + 2)) * cs;
#pragma unroll
                for (int e = 0; e < 8; ++e) x[e] = gn[e * cs];
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                acc[t] = Tr::mma32(lw[(q * 4 + t) * SD_WAVE + lane], f, acc[t]);
                if (HILO) acc[t] = Tr::mma32(lw[(q * 4 + t) * SD_WAVE + lane], fl, acc[t]);
            }
        };
        int q = 0;
        for (; q + 1 < nq; q += 2) {
            kstep(q, x0);
            kstep(q + 1, x1);
        }
        if (q < nq) kstep(q, x0);
        if (SD_PROJ_STAGE) {
            // the wave's 32 x 128 tile through LDS (68-dword pixel rows: 2-way conflicts at
            // most), then 16-B stores: 4 whole 256-B pixel rows per wave instruction
            uint32_t *so = (uint32_t *)(lds + nq * 4 * SD_WAVE * 16) + wave * (32 * 68);
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4)
                    // accumulator rows 4 r4 .. 4 r4 + 3 = hidden 32 t + 8 r4 + 4 h + 0..3
                    *(uint2 *)(so + li * 68 + (32 * t + 8 * r4 + 4 * h) / 2) =
                        uint2{sd_pack2<typename Tr::E>(acc[t][4 * r4], acc[t][4 * r4 + 1]),
                              sd_pack2<typename Tr::E>(acc[t][4 * r4 + 2], acc[t][4 * r4 + 3])};
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS writes
            const int64_t pix0 = (task - b * ntile) * 32;
            const int c = lane & 15;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int pp = 4 * k + (lane >> 4);
                if (pix0 + pp < HW) {
                    const uint4 v = *(const uint4 *)(so + pp * 68 + 4 * c);
                    *(uint4 *)(out + (b * HW + pix0 + pp) * (SD_DH / 2) + 4 * c) = v;
                }
            }
        } else if (valid) {
            uint2 *op = (uint2 *)(out + (b * HW + pix) * (SD_DH / 2));
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4)
                    // accumulator rows 4 r4 .. 4 r4 + 3 = hidden 32 t + 8 r4 + 4 h + 0..3
                    op[(32 * t + 8 * r4 + 4 * h) / 4] =
                        uint2{sd_pack2<typename Tr::E>(acc[t][4 * r4], acc[t][4 * r4 + 1]),
                              sd_pack2<typename Tr::E>(acc[t][4 * r4 + 2], acc[t][4 * r4 + 3])};
        }
    }
}

// ---------------------------------------------------------------------------
// k_project_lds: the channels-last projection (C = 256) as a streaming kernel.  k_project
// reads each lane's own pixel row 32 B at a time (32 pixel rows, 1 KiB apart, per wave
// instruction) and reached ~3.3 TB/s; here the grid is swept in order by LDS-DMA of whole
// pixel rows (1 KiB = one 64-lane DMA instruction) into a ring of PJ_NS slots of 16 rows,
// up to 6 slots (~96 KiB) in flight per CU.  Workgroup = 4 waves, one per CU; wave w owns
// hidden tile w (32 hidden): its 16 layer-1 A fragments (one per K step of 16 channels)
// stay in 64 VGPRs for the whole kernel, so the LDS holds only the grid rows.  Per
// 32-pixel chunk (slots 2k, 2k + 1) every wave reads the rows as the MFMA B operand
// (lane (pixel n, half h): 8 channels, 32 B), converts them to the 16-bit type and issues
// 16 32x32x16 MFMAs -- the same products in the same order as k_project, so P is
// bit-identical.  (PJ_FULLROW=0: the round-4 first version, half rows per slot.)  The 32 x 128 output tile goes
// through an LDS staging area and leaves as 16-B stores of whole 256-B pixel rows.
// ---------------------------------------------------------------------------
#ifndef PJ_FULLROW
#define PJ_FULLROW 1               // 1: slots of 16 whole pixel rows (1-KiB DMAs); 0: half rows
#endif
#define PJ_NS 8                    // ring slots
#ifndef PJ_WT
#define PJ_WT 1                    // P stored write-through
#endif
#define PJ_ROWB (PJ_FULLROW ? 1040 : 528)  // LDS bytes per staged row: data + 16 B pad (conflict-free reads)
#define PJ_SROWS (PJ_FULLROW ? 16 : 32)    // pixel rows per slot
#define PJ_SLOT (PJ_SROWS * PJ_ROWB)
#define PJ_OUTROW 272              // staging row stride (256 B of P + 16 pad)
#define PJ_LDS (PJ_NS * PJ_SLOT + 32 * PJ_OUTROW)

template <int P, bool FI, bool HILO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
k_project_lds(const float *__restrict__ grid, int64_t npix, const sd_mlp m, uint32_t *__restrict__ out,
              const sd_frame_args fa) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    typedef typename Tr::E E;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)lds;
    const int lane = threadIdx.x & 63, h = lane >> 5, li = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nch = (npix + 31) / 32;
    if (FI) {  // the frame's render inputs first (sd_project_grid_nhwc_inputs): grid-stride
        const int64_t nfi = sd_frame_items(fa);
        for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nfi; t += (int64_t)gridDim.x * 256)
            sd_frame_item(fa, t);
    }
    if ((int64_t)blockIdx.x >= nch) return;  // workgroup-uniform
    const int my = (int)((nch - 1 - blockIdx.x) / gridDim.x + 1);  // chunks of this workgroup

    // layer-1 A fragments of hidden tile `wave` (k_project's w_in: [q][ht][lane]) + bias rows
    Frag W[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) W[q] = ((const Frag *)m.w_in)[(q * 4 + wave) * SD_WAVE + lane];
    f32x16 bias;
    {
        const f32x4 *bb = (const f32x4 *)(m.b_in_h + (wave * 2 + h) * 16);
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            const f32x4 v = bb[q4];
#pragma unroll
            for (int i = 0; i < 4; ++i) bias[4 * q4 + i] = v[i];
        }
    }
    uint8_t *stg = lds + PJ_NS * PJ_SLOT;
    f32x16 acc = bias;
    // 32 x 128 accumulator tile of chunk k -> staging rows -> 16-B stores of whole pixel rows
    auto store_chunk = [&](int k) {
        // accumulator rows 4 r4 .. 4 r4 + 3 = hidden 32 wave + 8 r4 + 4 h + 0..3 of pixel li
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4)
            *(uint2 *)(stg + li * PJ_OUTROW + 2 * (32 * wave + 8 * r4 + 4 * h)) =
                uint2{sd_pack2<E>(acc[4 * r4], acc[4 * r4 + 1]),
                      sd_pack2<E>(acc[4 * r4 + 2], acc[4 * r4 + 3])};
        acc = bias;
        __syncthreads();  // the 32 x 128 tile is complete in the staging rows
        const int64_t pix0 = ((int64_t)blockIdx.x + (int64_t)k * gridDim.x) * 32;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int pp = 8 * wave + 4 * kk + (lane >> 4);
            const uint4 v = *(const uint4 *)(stg + pp * PJ_OUTROW + 16 * (lane & 15));
            if (pix0 + pp < npix) {
                if (PJ_WT) {  // write-through (sc1): P leaves L2 clean, no write-back at the boundary
                    typedef unsigned u4v __attribute__((ext_vector_type(4)));
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        (void *)(out + pix0 * (SD_DH / 2)), 0, 0x7fffffff, 0x00020000);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), rs,
                                                           (uint32_t)(pp * SD_DH * 2 + 16 * (lane & 15)), 0, 16);
                } else {
                    *(uint4 *)(out + (pix0 + pp) * (SD_DH / 2) + 4 * (lane & 15)) = v;
                }
            }
        }
    };
#if PJ_FULLROW
    // slot i = rows 16 (i & 1) .. + 15 of chunk i >> 1, whole 1-KiB pixel rows: this wave
    // DMAs rows 4 wave .. 4 wave + 3.  Slots past the workgroup's last chunk re-read the last
    // pixel (every chunk issues the same number of vector-memory operations).
    auto issue = [&](int i) {
        const int64_t c = (int64_t)blockIdx.x + (int64_t)(i >> 1) * gridDim.x;
        const uint32_t sb = lds0 + (uint32_t)(i % PJ_NS) * PJ_SLOT;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * wave + r;
            int64_t pix = c * 32 + 16 * (i & 1) + row;
            pix = pix < npix ? pix : npix - 1;
#ifndef PJ_NT
#define PJ_NT 1  // non-temporal grid stream (read once)
#endif
            if (PJ_NT)
                sd_dma16_nt(grid + pix * 256 + 4 * lane, sb + (uint32_t)row * PJ_ROWB);
            else
                sd_dma16(grid + pix * 256 + 4 * lane, sb + (uint32_t)row * PJ_ROWB);
        }
    };
#pragma unroll
    for (int i = 0; i < PJ_NS - 2; ++i) issue(i);
    for (int k = 0; k < my; ++k) {
        // slots 2k, 2k + 1 landed: this wave's DMAs of slots 2k + 2 .. 2k + PJ_NS - 3 (4 each,
        // + any stores) are younger
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        static_assert(4 * (PJ_NS - 4) == 16, "vmcnt immediate");
        __syncthreads();  // every wave's rows landed; chunk k - 1's slots are free
        issue(2 * k + PJ_NS - 2);
        issue(2 * k + PJ_NS - 1);
        // lane (pixel li, half h): slot 2k + (li >> 4), row li & 15, channels 16 q + 8 h ..
        const uint8_t *sl = lds + ((2 * k + (li >> 4)) % PJ_NS) * PJ_SLOT + (li & 15) * PJ_ROWB + 32 * h;
        // HILO (sd_mlp.proj_flags, round 6): the f32 grid enters the MFMA as a hi + lo pair
        // of 16-bit operands (hi = f16(g), lo = f16(g - hi), g - hi exact in f32): the one
        // rounding of G the projection makes otherwise costs up to 5.8e-3 m of composited
        // depth at configs[3]'s K = 128 (tools/lowp_depth_emul.py; W_in stays one f16
        // operand).  Twice the MFMAs and the conversions: C2 +8 us, C5 +48 us, so only the
        // renders that need it ask for it
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const f32x4 a = *(const f32x4 *)(sl + 64 * q), b = *(const f32x4 *)(sl + 64 * q + 16);
            Frag f, fl;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                f[e] = (E)a[e];
                f[4 + e] = (E)b[e];
                if (HILO) {
                    fl[e] = (E)(a[e] - (float)f[e]);
                    fl[4 + e] = (E)(b[e] - (float)f[4 + e]);
                }
            }
            acc = Tr::mma32(W[q], f, acc);
            if (HILO) acc = Tr::mma32(W[q], fl, acc);
        }
        store_chunk(k);
    }
#else
    // slot i = (chunk i >> 1, half i & 1): this wave DMAs rows 8 wave .. 8 wave + 7, 512 B each
    // (lanes 0..31)
    auto issue = [&](int i) {
        const int64_t c = (int64_t)blockIdx.x + (int64_t)(i >> 1) * gridDim.x;
        const uint32_t sb = lds0 + (uint32_t)(i % PJ_NS) * PJ_SLOT;
        if (lane < 32) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int row = 8 * wave + r;
                int64_t pix = c * 32 + row;
                pix = pix < npix ? pix : npix - 1;
                sd_dma16(grid + pix * 256 + (i & 1) * 128 + 4 * lane, sb + (uint32_t)row * PJ_ROWB);
            }
        }
    };
#pragma unroll
    for (int i = 0; i < PJ_NS - 1; ++i) issue(i);
    auto half_step = [&](int i, auto half_c) {
        constexpr int HALF = decltype(half_c)::value;
        asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
        static_assert(8 * (PJ_NS - 2) == 48, "vmcnt immediate");
        __syncthreads();
        issue(i + PJ_NS - 1);
        const uint8_t *sl = lds + (i % PJ_NS) * PJ_SLOT + li * PJ_ROWB + 32 * h;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f32x4 a = *(const f32x4 *)(sl + 64 * q), b = *(const f32x4 *)(sl + 64 * q + 16);
            Frag f, fl;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                f[e] = (E)a[e];
                f[4 + e] = (E)b[e];
                if (HILO) {
                    fl[e] = (E)(a[e] - (float)f[e]);
                    fl[4 + e] = (E)(b[e] - (float)f[4 + e]);
                }
            }
            acc = Tr::mma32(W[8 * HALF + q], f, acc);
            if (HILO) acc = Tr::mma32(W[8 * HALF + q], fl, acc);
        }
    };
    for (int k = 0; k < my; ++k) {
        half_step(2 * k, std::integral_constant<int, 0>());
        half_step(2 * k + 1, std::integral_constant<int, 1>());
        store_chunk(k);
    }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup
}

// ---------------------------------------------------------------------------
// render helpers
// ---------------------------------------------------------------------------

// Per-sample record written by the ray pass into wave-private LDS, quad-major
// ([q][k][4 words], q = 0 .. RS/4-1) so that both the ray pass (lane = sample) and the
// item reads (lane j = sample) are conflict-free 16-byte accesses:
//   q0: byte offsets pix * 256 of the taps (x0, y0) and (x0, y1) in the plain P
//       interleaved P (bit 0 of the first: outside the encoder frustum; bits 0..3 of
//       the second: outside render view 0..3), 2 spare words
//   q1: bilinear weights pre-packed in the blend's operand format (T16<P>::pack_w)
//   q2: x, y, z~ (positional-code inputs), z
//   q3: delta, colour of render view 0 (r, g, b); then views 1..3 (3 words each)
// SD_RECBUF = 1: one record buffer per wave, refilled for the wave's next ray just
// before that ray's first item is opened (the current ray's records are dead by then);
// 2: double-buffered, the next ray's pass one whole ray ahead (twice the LDS).
__host__ __device__ constexpr int sd_rec_words(int nv) { return (13 + 3 * nv + 3) & ~3; }

#ifndef SD_RECBUF
#define SD_RECBUF 2
#endif
#ifndef SD_RWG
#define SD_RWG 256  // render workgroup (4 waves; 2 waves per SIMD: VGPR-bound at ~215)
#endif
#ifndef SD_HC_MIN_D
#define SD_HC_MIN_D 16  // D >= this: hidden-space compositing + k_head_hc (measured faster
                        // than the folded head already at D = 64: 0.685 vs 0.706 ms, C2)
#endif
#define SD_HC_STRIDE 132  // floats per ray of the hidden-composite scratch: hsum[128], wsum
#define SD_MAX_D 512
static inline bool sd_head_hc(int D) {
    return D >= SD_HC_MIN_D || (D != 32 && D != 64 && D != 128);
}
#ifndef SD_RWAVES
#define SD_RWAVES 2  // waves per SIMD the register budget is cut for (2: <= 256 VGPRs)
#endif

struct PItem {
    int ray, sub, sbi, n, rr;  // rr: the real ray of the (virtual) ray index
    uint32_t o[2];  // tap (x0, y0) / (x0, y1) byte offsets (+ 16 g) inside the P plane
    uint4 wp;       // packed blend weights
    float v[3];
    float zk, delta;
    float col[3];   // colour of this lane's render view (group g; NV == 1: view 0)
    bool inv_f, invc;
    __amdgpu_buffer_rsrc_t rs;
};

struct PRaw { uint4 a, b, c, d; };

// chunk q (channels 32 q .. 32 q + 31; this lane's group: 8 of them = 32 bytes per row)
__device__ __forceinline__ PRaw sd_pload(const PItem &it, int q) {
    const uint32_t s = (uint32_t)q * 64u;
    PRaw r;
    r.a = sd_ld128(it.rs, it.o[0], s);
    r.b = sd_ld128(it.rs, it.o[0] + 256u, s);
    r.c = sd_ld128(it.rs, it.o[1], s);
    r.d = sd_ld128(it.rs, it.o[1] + 256u, s);
    return r;
}


// LDS image of the render kernel: [code 2][8][64] | [sigma 4][64] | [dino D/16][4][64]
// (16 B per lane entry), then per wave SD_RECBUF x K sample records.
#define SD_LDS_PE 0
#define SD_LDS_PE1 (SD_LDS_PE + 8 * SD_WAVE)   // 16x16x16 code fragments (8 B per lane entry)
#define SD_LDS_SIG (SD_LDS_PE + 12 * SD_WAVE)
#define SD_LDS_OUT (SD_LDS_SIG + 4 * SD_WAVE)

// wave-uniform cursor with the wave's ray ordinal n (selects the record buffer)
struct RCursor {
    int ray, sub, sbi, n, rr;
};

template <int P, int NV, int NDT>
__global__ void __launch_bounds__(SD_RWG) __attribute__((amdgpu_waves_per_eu(SD_RWAVES)))
k_render_proj(const sd_render_args a, const sd_head m, const int32_t *__restrict__ list) {
    typedef typename RMode<P>::F Tr;  // operands upstream of sigma (f16 in both modes)
    typedef typename RMode<P>::H Th;  // DINO head (bf16 in the bf16 mode)
    constexpr bool HEAD_CVT = !std::is_same<Tr, Th>::value;  // X re-rounded for the head
    typedef typename Tr::Frag Frag;
    typedef typename Tr::Frag4 Frag4;
    typedef typename Tr::E E;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    // list mode (fallback behind the tile kernel, launched with its grid): workgroup b
    // renders tile workgroup b's overflow list (sdhip_render.h), usually empty -- it leaves
    // before staging the weights
    const int nlist = list ? __builtin_amdgcn_readfirstlane(list[blockIdx.x]) : 0;
    if (list && nlist == 0) return;
    {
        uint4 *d = (uint4 *)lds;
        const uint4 *pe = (const uint4 *)m.w_pe, *sg = (const uint4 *)m.w_sig,
                    *wo = (const uint4 *)m.w_out;
        for (int i = threadIdx.x; i < 12 * SD_WAVE; i += blockDim.x) d[SD_LDS_PE + i] = pe[i];
        for (int i = threadIdx.x; i < 4 * SD_WAVE; i += blockDim.x) d[SD_LDS_SIG + i] = sg[i];
        for (int i = threadIdx.x; i < NDT * 4 * SD_WAVE; i += blockDim.x) d[SD_LDS_OUT + i] = wo[i];
        __syncthreads();
    }
    const Frag *lf = (const Frag *)lds;

    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // identity fragments live in registers (8 VGPRs): A[i][k] = [k == i] / [k == 16 + i]
    Frag id0, id1;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        id0[e] = (E)((8 * g + e == j) ? 1.f : 0.f);
        id1[e] = (E)((8 * g + e == j + 16) ? 1.f : 0.f);
    }
    const int K = a.K, nsub = K >> 4, nv = NV > 0 ? NV : a.nv;
    const int RQ = sd_rec_words(nv) / 4;  // 16-byte quads per record
    uint4 *recs = (uint4 *)(lds + (SD_LDS_OUT + NDT * 4 * SD_WAVE) * 16) + wave * SD_RECBUF * K * RQ;
    const uint32_t plane_bytes = (uint32_t)a.Hf * a.Wf * SD_DH * 2;
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;
    // XCD-aware ray ranges: workgroups b, b + 8, ... share one XCD (round-robin dispatch,
    // a speed assumption only), so XCD x gets the contiguous rays [x R/8, (x+1) R/8): the
    // P rows its rays' epipolar lines cross stay in that XCD's 4 MiB L2 instead of every
    // XCD streaming all of P.  R below is this range's end.
    // (list mode: one range -- the workgroup's own list)
    const int nx = (!list && gridDim.x % 8 == 0) ? 8 : 1;
    const int xcd = blockIdx.x % nx;
    const int nwaves = list ? SD_RWG / 64 : (gridDim.x / nx) * (SD_RWG / 64);
    const int rps = (int)a.rays_per_sb;
    // list != NULL: the rays of the blocks in list b (SD_LIST_BLK consecutive rays each)
    // form the virtual ray sequence of workgroup b
    const int Rreal = (int)a.R;
    const int64_t RA = list ? (int64_t)nlist * SD_LIST_BLK : a.R;
    const int32_t *lblk = list ? list + gridDim.x + (int64_t)blockIdx.x * sd_ovf_cap(a.R, gridDim.x) : nullptr;
    auto rmap = [&](int v) {
        return list ? min(lblk[v / SD_LIST_BLK] * SD_LIST_BLK + v % SD_LIST_BLK, Rreal - 1) : v;
    };
    const int R = (int)(RA * (xcd + 1) / nx);
    const int ray0 = (int)(RA * xcd / nx) + (list ? 0 : (blockIdx.x / nx) * (SD_RWG / 64)) + wave;
    if (ray0 >= R) return;
    const int nitems = ((R - ray0 + nwaves - 1) / nwaves) * nsub;
    // in-kernel z (a.z == NULL): sd_sample_z's arithmetic, jitter from the counter RNG
    const float zstep = (float)(1.0 / (double)K), zend = (float)(1.0 - 1.0 / (double)K);

    auto advance = [&](RCursor c) {
        if (c.sub + 1 < nsub) {
            c.sub++;
        } else if (c.ray + nwaves < R) {
            c.ray += nwaves;
            c.sub = 0;
            c.n++;
            c.rr = rmap(c.ray);
            c.sbi = __builtin_amdgcn_readfirstlane((int)((unsigned)c.rr / (unsigned)rps));
        }
        return c;
    };

    // ---- ray pass: per-sample geometry and colours of one ray, lane = sample ----------
    // zq[2p], zq[2p+1]: z[k], z[k+1] of this lane's sample k = 64 p + lane (prefetched)
    constexpr int MAXP = 2;  // K <= 128
    auto load_ray_z = [&](int ray, float zq[2 * MAXP]) {
        float zo[MAXP];
        if (a.z) {
            const float *zr = a.z + (int64_t)ray * K;
#pragma unroll
            for (int p = 0; p < MAXP; ++p) zo[p] = zr[min(64 * p + lane, K - 1)];
        } else {
            sd_cfloat *rr = (sd_cfloat *)(a.rays + (int64_t)ray * a.ray_dim);
            const float near = rr[6], far = rr[7];
            const uint64_t base = a.z_offset + (uint64_t)ray * (uint64_t)K;
#pragma unroll
            for (int p = 0; p < MAXP; ++p) {
                const int k = min(64 * p + lane, K - 1);
                zo[p] = sd_z_sample_rng(near, far, K, k, sd_uniform(a.z_seed, base + k), zstep, zend,
                                    a.z_lindisp);
            }
        }
        // z[k + 1] from the next lane (lane 63: lane 0 of the next 64-sample block)
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            // every lane takes part in the exchange (no shuffle under a lane condition)
            float nx = __shfl_down(zo[p], 1, 64);
            const float first_next = p + 1 < MAXP
                ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                      __builtin_bit_cast(int, zo[p + 1 < MAXP ? p + 1 : p]), 0))
                : zo[p];
            if (lane == 63) nx = (p + 1 < MAXP && 64 * (p + 1) < K) ? first_next : zo[p];
            zq[2 * p] = zo[p];
            zq[2 * p + 1] = nx;
        }
    };
    // NV == 1: the colour texel loads of sample 64 p + lane, p = 0, are left in flight
    // (ColPend) and the colour words written by ray_col at the end of the item
    constexpr bool DEFER = NV == 1;
    ColPend cpend;
    auto ray_pass = [&](int ray, int sbi, int buf, const float zq[2 * MAXP]) {
        sd_cfloat *rr = (sd_cfloat *)(a.rays + (int64_t)ray * a.ray_dim);
        const float ox = rr[0], oy = rr[1], oz = rr[2], dx = rr[3], dy = rr[4], dz = rr[5];
        uint4 *rb = recs + buf * K * RQ;
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
            const int k = 64 * p + lane;
            if (64 * p < K && k < K) {
                const float z0 = zq[2 * p], z1 = zq[2 * p + 1];
                const float px = ox + z0 * dx, py = oy + z0 * dy, pz = oz + z0 * dz;  // nerf.py:252
                PointGeo geo = sd_point_geo_fast((sd_cfloat *)(a.cam_f + sbi * SD_CAM_WORDS), px, py, pz, a.Wf, a.Hf);
                float col[3 * SD_MAX_NV];
                uint32_t invc = 0;
                const float delta = (k + 1 < K) ? (z1 - z0) : 1e10f;
                if (DEFER && p == 0) {
                    bool ic;
                    const Taps tc = sd_color_taps_fast((sd_cfloat *)(a.cam_c + sbi * SD_CAM_WORDS), a.Wc, a.Hc,
                                                  px, py, pz, ic);
                    sd_color_issue(a.img + (int64_t)sbi * cplane, tc, cpend);
                    cpend.delta = delta;
                    invc = ic ? 1u : 0u;
                }
#pragma unroll
                for (int v = 0; v < SD_MAX_NV; ++v) {
                    col[3 * v] = col[3 * v + 1] = col[3 * v + 2] = 0.f;
                    if (v < nv && !(DEFER && p == 0)) {
                        const bool ic = NV == 1
                            ? sd_color_view((sd_cfloat *)(a.cam_c + sbi * SD_CAM_WORDS), a.img + (int64_t)sbi * cplane,
                                            a.Wc, a.Hc, px, py, pz, col)
                            : sd_color_view((sd_cfloat *)(a.cam_c + (sbi * nv + v) * SD_CAM_WORDS),
                                            a.img + (int64_t)(sbi * nv + v) * cplane, a.Wc, a.Hc,
                                            px, py, pz, col + 3 * v);
                        invc |= (ic ? 1u : 0u) << v;
                    }
                }
                rb[0 * K + k] = uint4{(uint32_t)geo.t.i00 * 256u | (geo.inv_f ? 1u : 0u),
                                      (uint32_t)geo.t.i10 * 256u | invc, 0u, 0u};
                rb[1 * K + k] = sd_pack_w<SD_F16>(geo.t.w00, geo.t.w01, geo.t.w10, geo.t.w11);
                rb[2 * K + k] = __builtin_bit_cast(uint4, f32x4{geo.v[0], geo.v[1], geo.v[2], z0});
                if (!(DEFER && p == 0))
                    rb[3 * K + k] = __builtin_bit_cast(uint4, f32x4{delta, col[0], col[1], col[2]});
#pragma unroll
                for (int q = 4; q < sd_rec_words(SD_MAX_NV) / 4; ++q)
                    if (q < RQ) {
                        float e[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const int c = 4 * q + t - 16 + 3;  // colour word index
                            e[t] = c < 3 * SD_MAX_NV ? col[c] : 0.f;
                        }
                        rb[q * K + k] = __builtin_bit_cast(uint4, f32x4{e[0], e[1], e[2], e[3]});
                    }
            }
        }
        __builtin_amdgcn_wave_barrier();
    };
    // deferred colour words of the last ray pass (sample k = lane)
    auto ray_col = [&](int buf) {
        if (DEFER && lane < K) {
            float col[3];
            sd_color_finish(cpend, col);
            recs[buf * K * RQ + 3 * K + lane] =
                __builtin_bit_cast(uint4, f32x4{cpend.delta, col[0], col[1], col[2]});
        }
        __builtin_amdgcn_wave_barrier();
    };
    // ---- item open: this lane's sample record from LDS -------------------------------
    auto open_item = [&](const RCursor &c, PItem &it) {
        it.ray = c.ray;
        it.rr = c.rr;
        it.sub = c.sub;
        it.sbi = c.sbi;
        it.n = c.n;
        const uint4 *rb = recs + (SD_RECBUF == 2 ? (c.n & 1) : 0) * K * RQ;
        const int k = c.sub * 16 + j;
        const uint4 q0 = rb[k];
        const uint4 q1 = rb[K + k];
        const f32x4 q2 = __builtin_bit_cast(f32x4, rb[2 * K + k]);
        const f32x4 q3 = __builtin_bit_cast(f32x4, rb[3 * K + k]);
        const uint32_t lo = 16u * (uint32_t)g;
        it.o[0] = (q0.x & ~255u) + lo;
        it.o[1] = (q0.y & ~255u) + lo;
        it.inv_f = q0.x & 1u;
        const int vv = NV == 1 ? 0 : g;
        it.invc = (q0.y >> vv) & 1u;
        it.wp = q1;
        it.v[0] = q2[0]; it.v[1] = q2[1]; it.v[2] = q2[2];
        it.zk = q2[3];
        it.delta = q3[0];
        if (NV == 1 || g == 0) {
            it.col[0] = q3[1]; it.col[1] = q3[2]; it.col[2] = q3[3];
        } else {
            // view g's colour: words 13 + 3 g .. 15 + 3 g of the record
            const float *fb = (const float *)rb;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int wd = 13 + 3 * g + c;
                it.col[c] = g < nv ? fb[((wd >> 2) * K + k) * 4 + (wd & 3)] : 0.f;
            }
        }
        it.rs = sd_rsrc((const uint8_t *)a.grid + (int64_t)it.sbi * plane_bytes, plane_bytes);
    };

    // prologue: records of the first ray, item 0 open with its taps in flight
    const int rr0 = rmap(ray0);
    RCursor c0 = {ray0, 0, (int)((unsigned)rr0 / (unsigned)rps), 0, rr0};
    float zq[2 * MAXP];
    load_ray_z(c0.rr, zq);
    ray_pass(c0.rr, c0.sbi, 0, zq);
    ray_col(0);
    const bool more = ray0 + nwaves < R;
    if (more) load_ray_z(rmap(ray0 + nwaves), zq);  // z of the wave's second ray in flight
    PItem cur;
    open_item(c0, cur);
    RCursor c1 = advance(c0);
    PRaw r0 = sd_pload(cur, 0), r1 = sd_pload(cur, 1), r2 = sd_pload(cur, 2), r3 = sd_pload(cur, 3);

    // NDT > 0: DINO head folded into the compositing sum (dacc, D = 16 NDT);
    // NDT == 0: hidden-space compositing, hacc = sum_j w_j relu(h_j) (rows 16 t + 4 g + r),
    // the head applied per ray afterwards (k_head_hc: W_dino . hsum + b_dino wsum)
    constexpr bool HC = NDT == 0;
    f32x4 dacc[HC ? 1 : NDT], hacc[HC ? 8 : 1];
#pragma unroll
    for (int i = 0; i < (HC ? 1 : NDT); ++i) dacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < (HC ? 8 : 1); ++i) hacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float Tc = 1.f, dpart = 0.f, wpart = 0.f, cpart[3] = {0.f, 0.f, 0.f};
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

    // one item: `cur` computes, `nxt` is opened (unrolled by two below so the item
    // state ping-pongs between two register sets instead of being copied)
    auto step = [&](PItem &cur, PItem &nxt) {
        bool passed = false;  // wave-uniform: a ray pass left colour loads in flight
#if !SD_ABL_NORAYPASS
        if (SD_RECBUF == 2) {
            // first item of a ray: records of the wave's next ray into the other buffer
            if (cur.sub == 0 && cur.ray + nwaves < R) {
                const int nr = cur.ray + nwaves, nrr = rmap(nr);
                ray_pass(nrr, (int)((unsigned)nrr / (unsigned)rps), (cur.n + 1) & 1, zq);
                passed = true;
                if (nr + nwaves < R) load_ray_z(rmap(nr + nwaves), zq);
            }
        } else if (c1.n != cur.n) {
            // the next item starts the wave's next ray: its records replace this ray's
            // (every record of this ray was read when `cur` was opened)
            ray_pass(c1.rr, c1.sbi, 0, zq);
            ray_col(0);
            if (c1.ray + nwaves < R) load_ray_z(rmap(c1.ray + nwaves), zq);
        }
#endif
        open_item(c1, nxt);
        c1 = advance(c1);

        const int lo = sd_opaque0();
        const Frag *lw = lf + lo;
        // grid part: identity MFMAs on the blended P chunks; refill with item i+1's taps
        f32x4 acc[8];
#define SD_PCHUNK(r, q)                                                        \
        {                                                                      \
            Frag f_ = SD_ABL_NOBLEND ? __builtin_bit_cast(Frag, r.a ^ r.b ^ r.c ^ r.d) \
                                     : sd_blend_plain<SD_F16>(r.a, r.b, r.c, r.d, cur.wp); \
            r = sd_pload(nxt, q);                                              \
            acc[2 * q] = Tr::mma(id0, f_, zero4);                              \
            acc[2 * q + 1] = Tr::mma(id1, f_, zero4);                          \
        }
        SD_PCHUNK(r0, 0)
        SD_PCHUNK(r1, 1)
        SD_PCHUNK(r2, 2)
        SD_PCHUNK(r3, 3)
#undef SD_PCHUNK
        // positional-code columns
        {
            Frag f0;
            Frag4 f1;
#if SD_ABL_NOPE
            for (int e = 0; e < 8; ++e) f0[e] = (E)cur.v[e % 3];
            f1 = __builtin_bit_cast(Frag4, uint2{__builtin_bit_cast(uint32_t, cur.v[0]), 0u});
#else
            sd_code_frags<Frag, Frag4, E>(cur.v, g, f0, f1);
#endif
            const Frag4 *lw1 = (const Frag4 *)(lds + SD_LDS_PE1 * 16) + lo;
            // all 16x16x32 steps first, then the 16x16x16 ones (see sdhip_tile.hip)
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = Tr::mma(lw[SD_LDS_PE + t * SD_WAVE + lane], f0, acc[t]);
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = Tr::mma16(lw1[t * SD_WAVE + lane], f1, acc[t]);
        }
        // 16-bit operand fragments (accumulator-as-operand), ReLU on the packed values
        Frag X[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint4 u = {sd_relu2(sd_pack2<E>(acc[2 * s][0], acc[2 * s][1])),
                             sd_relu2(sd_pack2<E>(acc[2 * s][2], acc[2 * s][3])),
                             sd_relu2(sd_pack2<E>(acc[2 * s + 1][0], acc[2 * s + 1][1])),
                             sd_relu2(sd_pack2<E>(acc[2 * s + 1][2], acc[2 * s + 1][3]))};
            X[s] = __builtin_bit_cast(Frag, u);
        }
        // sigma (bts.py:516-541): every accumulator row holds w_sigma . h of sample j
        f32x4 sg = zero4;
#pragma unroll
        for (int s = 0; s < 4; ++s) sg = Tr::mma(lw[SD_LDS_SIG + s * SD_WAVE + lane], X[s], sg);
        const float sv = sg[0] + m.b_sigma;
        const float sigma = sd_softplus_fast(sv);

        // alpha compositing (nerf.py:376-389)
        const int k = cur.sub * 16 + j;
        float alpha = 1.f - __expf(-fabsf(cur.delta) * fmaxf(sigma, 0.f));
        if (a.hard_alpha_cap && k == K - 1) alpha = 1.f;
        const float incl = sd_scan_mul16((1.f - alpha) + 1e-10f);
        const float excl = SD_DPP1(incl, 0x111);
        const float w = alpha * (Tc * excl);
        Tc *= __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 15));
        dpart += w * cur.zk;
        wpart += w;
        cpart[0] += w * cur.col[0];
        cpart[1] += w * cur.col[1];
        cpart[2] += w * cur.col[2];
        if (HC) {
            // from the ReLU'd 16-bit operands (the f32 accumulators are dead by now)
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 u = __builtin_bit_cast(uint4, X[s2]);
                const uint32_t d4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int t = 2 * s2 + (q >> 1), r = 2 * (q & 1);
                    hacc[t][r] = fmaf(w, sd_unpack_lo<SD_F16>(d4[q]), hacc[t][r]);
                    hacc[t][r + 1] = fmaf(w, sd_unpack_hi<SD_F16>(d4[q]), hacc[t][r + 1]);
                }
            }
        }
        // DINO head folded into the compositing sum: dacc += w_j (W_dino h_j); in the bf16
        // mode relu(h) re-rounded to the head's bf16 operands
        typename Th::Frag XH[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if constexpr (HEAD_CVT) {
                if (NDT > 0) {
                    const uint4 u = __builtin_bit_cast(uint4, X[s]);
                    const uint32_t d4[4] = {u.x, u.y, u.z, u.w};
                    uint32_t o4[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        o4[q] = sd_pack2<typename Th::E>(sd_unpack_lo<SD_F16>(d4[q]), sd_unpack_hi<SD_F16>(d4[q]));
                    XH[s] = __builtin_bit_cast(typename Th::Frag, uint4{o4[0], o4[1], o4[2], o4[3]});
                }
            } else {
                XH[s] = __builtin_bit_cast(typename Th::Frag, X[s]);
            }
        }
        const typename Th::Frag *lwh = (const typename Th::Frag *)lds + lo;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
            f32x4 o = zero4;
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if (!SD_ABL_NODINO || s == 0) o = Th::mma(lwh[SD_LDS_OUT + (dt * 4 + s) * SD_WAVE + lane], XH[s], o);
#pragma unroll
            for (int r = 0; r < 4; ++r) dacc[dt][r] = fmaf(w, o[r], dacc[dt][r]);
        }

        // per-sample outputs: wave-uniform ray base + 32-bit lane offset
        const int64_t rk = (int64_t)cur.rr * K;
        if (g == 0) {
            if (a.weights) (a.weights + rk)[k] = w;
            if (a.alphas) (a.alphas + rk)[k] = alpha;
            if (a.invalid_f) (a.invalid_f + rk)[k] = cur.inv_f ? 1 : 0;
        }
        if (g < nv) {
            if (a.invalid) (a.invalid + rk * nv)[k * nv + g] = (cur.invc | cur.inv_f) ? 1.f : 0.f;
            if (a.rgb_samps) {
                float *rsp = a.rgb_samps + rk * nv * 3 + (k * nv + g) * 3;
                rsp[0] = cur.col[0]; rsp[1] = cur.col[1]; rsp[2] = cur.col[2];
            }
        }

        if (cur.sub == nsub - 1) {
            // ray epilogue: sums over the 16 sample lanes of every row
            const float dsum = sd_rowsum16(dpart), wsum = sd_rowsum16(wpart);
            const float c0s = sd_rowsum16(cpart[0]), c1s = sd_rowsum16(cpart[1]),
                        c2s = sd_rowsum16(cpart[2]);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = sd_rowsum16(dacc[dt][r]);
                if (j == 0) {
                    // rows 4 g + r of dino tile dt = dims 16 dt + 4 g + r
                    const int dim = 16 * dt + 4 * g;
                    const f32x4 bd = *(const f32x4 *)(m.b_dino + dim);
                    f32x4 res;
#pragma unroll
                    for (int r = 0; r < 4; ++r) res[r] = v[r] + wsum * bd[r];
                    *(f32x4 *)(a.dino + (int64_t)cur.rr * a.ld_dino + dim) = res;
                }
                dacc[dt] = zero4;
            }
            if (HC) {
                float *hs = a.work + (int64_t)cur.rr * SD_HC_STRIDE;
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = sd_rowsum16(hacc[t][r]);
                    if (j == 0) *(f32x4 *)(hs + 16 * t + 4 * g) = v;
                    hacc[t] = zero4;
                }
                if (lane == 0) hs[SD_DH] = wsum;
            }
            if (lane == 0) a.depth[(int64_t)cur.rr * a.ld_depth] = dsum;
            if (j == 0 && g < nv) {
                float *rp = a.rgb + (int64_t)cur.rr * a.ld_rgb + 3 * g;
                rp[0] = c0s; rp[1] = c1s; rp[2] = c2s;
            }
            Tc = 1.f; dpart = 0.f; wpart = 0.f;
            cpart[0] = cpart[1] = cpart[2] = 0.f;
        }
        if (SD_RECBUF == 2 && passed) ray_col((cur.n + 1) & 1);
    };
    PItem alt;
    for (int i = 0; i < nitems; i += 2) {
        step(cur, alt);
        if (i + 1 < nitems) step(alt, cur);
    }
}

// ---------------------------------------------------------------------------
// k_head_hc: dino[r] = W_dino . hsum[r] + b_dino * wsum[r] for the hidden-space
// composited rays (render kernel with NDT == 0).  One wave = 16 rays x all D dims:
// A = the W_dino fragments of sd_head (LDS), B = hsum^T in the same hidden-index
// permutation hid(s, g, e) = 32 s + 16 (e >> 2) + 4 g + (e & 3), 16x16x32 MFMA.
// ---------------------------------------------------------------------------
template <int P>
__global__ void __launch_bounds__(SD_PWG)
k_head_hc(const float *__restrict__ work, int64_t R, const sd_head m, float *__restrict__ dino,
          int64_t ld_dino, const int32_t *__restrict__ list) {
    typedef typename RMode<P>::H Tr;  // the DINO head's operand type
    typedef typename Tr::Frag Frag;
    typedef typename Tr::E E;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int ndt = m.D >> 4;
    {
        const uint4 *src = (const uint4 *)m.w_out;
        uint4 *dst = (uint4 *)lds;
        for (int i = threadIdx.x; i < ndt * 4 * SD_WAVE; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    const Frag *lw = (const Frag *)lds;
    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // list != NULL: workgroup b takes tile workgroup b's overflow list (see k_render_proj;
    // launched with the tile grid)
    const int64_t RA = list ? (int64_t)__builtin_amdgcn_readfirstlane(list[blockIdx.x]) * SD_LIST_BLK : R;
    const int32_t *lblk = list ? list + gridDim.x + (int64_t)blockIdx.x * sd_ovf_cap(R, gridDim.x) : nullptr;
    const int64_t ntile = (RA + 15) / 16;
    const int64_t t0 = list ? wave : (int64_t)blockIdx.x * (SD_PWG / 64) + wave;
    const int64_t tstep = list ? SD_PWG / 64 : (int64_t)gridDim.x * (SD_PWG / 64);
    for (int64_t tile = t0; tile < ntile; tile += tstep) {
        const int64_t v = min(tile * 16 + j, RA - 1);
        const int64_t ray = list ? min((int64_t)lblk[v / SD_LIST_BLK] * SD_LIST_BLK + v % SD_LIST_BLK, R - 1)
                                 : tile * 16 + j;
        const float *hs = work + (ray < R ? ray : R - 1) * SD_HC_STRIDE;
        Frag B[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const f32x4 lo = *(const f32x4 *)(hs + 32 * s + 4 * g);
            const f32x4 hi = *(const f32x4 *)(hs + 32 * s + 16 + 4 * g);
            const uint4 u = {sd_pack2<E>(lo[0], lo[1]), sd_pack2<E>(lo[2], lo[3]),
                             sd_pack2<E>(hi[0], hi[1]), sd_pack2<E>(hi[2], hi[3])};
            B[s] = __builtin_bit_cast(Frag, u);
        }
        const float ws = hs[SD_DH];
        for (int dt = 0; dt < ndt; ++dt) {
            f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) o = Tr::mma(lw[(dt * 4 + s) * SD_WAVE + lane], B[s], o);
            // rows 4 g + r of tile dt = dims 16 dt + 4 g + r, column j = ray
            const int dim = 16 * dt + 4 * g;
            const f32x4 bd = *(const f32x4 *)(m.b_dino + dim);
            f32x4 res;
#pragma unroll
            for (int r = 0; r < 4; ++r) res[r] = o[r] + ws * bd[r];
            if (ray < R) *(f32x4 *)(dino + ray * ld_dino + dim) = res;
        }
    }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
template <typename KernT>
static int sd_launch_proj(KernT kern, int64_t work_waves, int lds_bytes, hipStream_t s,
                          int64_t &nblk, int wg = SD_PWG) {
    sd_lds_attr((const void *)kern, lds_bytes);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, wg, lds_bytes) !=
            hipSuccess || per_cu <= 0)
        per_cu = 1;
    nblk = (work_waves + wg / 64 - 1) / (wg / 64);
    const int64_t cap = (int64_t)sd_num_cus() * per_cu;
    if (nblk > cap) nblk = cap;
    return 0;
}

static int sd_check_err() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        return -2;
    }
    return 0;
}

extern "C" int sd_frame_inputs(const float *img_nchw, int64_t N, int64_t H, int64_t W, float *out_nhwc4,
                               const float *w2c, int64_t s_w, const float *Ks, int64_t s_k, int64_t n,
                               float *out_cam, void *stream);

static int sd_project_any(const float *grid, int64_t B, int64_t Hf, int64_t Wf, const sd_mlp *m,
                          void *out, void *stream, bool nhwc, const sd_frame_args *fa = nullptr) {
    if (!grid || !m || !out || !m->w_in || !m->b_in_h || B <= 0 || Hf <= 0 || Wf <= 0 ||
        m->d_hidden != SD_DH || m->C <= 0 || (m->C % 64) ||
        (m->dtype != SD_BF16 && m->dtype != SD_F16)) {
        sd_set_error("sd_project_grid: invalid argument (16-bit dtype, C % 64 == 0, d_hidden 128)");
        return -1;
    }
    const int64_t HW = Hf * Wf;
    const int lds_bytes = m->C / 16 * 4 * SD_WAVE * 16 + (SD_PROJ_STAGE ? SD_PWG / 64 * 32 * 68 * 4 : 0);
    if (lds_bytes > 160 * 1024) {
        sd_set_error("sd_project_grid: C too large for the LDS-staged weights");
        return -1;
    }
    hipStream_t s = (hipStream_t)stream;
    int64_t nblk;
    const int64_t work = B * ((HW + 31) / 32);
    static const bool old_proj = getenv("SDHIP_PROJ_OLD") != nullptr;  // diagnostic A/B switch
    if (nhwc && m->C == 256 && !old_proj) {  // the streaming LDS-DMA kernel
        const int64_t nch = work;
        nblk = sd_num_cus();
        if (nblk > nch) nblk = nch;
        const sd_frame_args none = {};
        auto go = [&](auto kern) {
            sd_lds_attr((const void *)kern, PJ_LDS);
            hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(256), PJ_LDS, s, grid, B * HW, *m,
                               (uint32_t *)out, fa ? *fa : none);
        };
        // both 16-bit modes: P in f16 (RMode, sdhip_render.h)
        const bool hl = (m->proj_flags & SD_PROJ_EXACT_GRID) != 0;
        if (fa) {
            if (hl) go(k_project_lds<SD_F16, true, true>); else go(k_project_lds<SD_F16, true, false>);
        } else {
            if (hl) go(k_project_lds<SD_F16, false, true>); else go(k_project_lds<SD_F16, false, false>);
        }
        return sd_check_err();
    }
    if (fa) {  // other grids: the frame inputs by their own launch
        int rc = sd_frame_inputs(fa->img_nchw, fa->N, fa->H, fa->W, fa->out_nhwc4, fa->w2c, fa->s_w,
                                 fa->Ks, fa->s_k, fa->n, fa->out_cam, stream);
        if (rc) return rc;
    }
#define SD_PROJ_LAUNCH(PP, NH, HL)                                                                \
    do {                                                                                          \
        sd_launch_proj(k_project<PP, NH, HL>, work, lds_bytes, s, nblk);                          \
        hipLaunchKernelGGL((k_project<PP, NH, HL>), dim3((unsigned)nblk), dim3(SD_PWG), lds_bytes, s, \
                           grid, B, m->C, HW, (int)Wf, *m, (uint32_t *)out);                      \
    } while (0)
    const bool hl = (m->proj_flags & SD_PROJ_EXACT_GRID) != 0;
    if (nhwc) {
        if (hl) SD_PROJ_LAUNCH(SD_F16, true, true); else SD_PROJ_LAUNCH(SD_F16, true, false);
    } else {
        if (hl) SD_PROJ_LAUNCH(SD_F16, false, true); else SD_PROJ_LAUNCH(SD_F16, false, false);
    }
#undef SD_PROJ_LAUNCH
    return sd_check_err();
}

extern "C" int sd_project_grid(const float *grid, int64_t B, int64_t Hf, int64_t Wf,
                               const sd_mlp *m, void *out, void *stream) {
    return sd_project_any(grid, B, Hf, Wf, m, out, stream, false);
}

extern "C" int sd_project_grid_nhwc_inputs(const float *grid, int64_t B, int64_t Hf, int64_t Wf,
                                           const sd_mlp *m, void *out, const sd_frame_args *fa,
                                           void *stream) {
    if (!fa || !fa->img_nchw || !fa->out_nhwc4 || fa->N <= 0 || fa->H <= 0 || fa->W <= 0 || !fa->w2c ||
        !fa->Ks || !fa->out_cam || fa->n <= 0 || fa->s_w < 16 || fa->s_k < 9) {
        sd_set_error("sd_project_grid_nhwc_inputs: invalid frame arguments");
        return -1;
    }
    if (((uintptr_t)grid & 15) || ((uintptr_t)fa->out_nhwc4 & 15)) {
        sd_set_error("sd_project_grid_nhwc_inputs: grid and packed image must be 16-byte aligned");
        return -1;
    }
    return sd_project_any(grid, B, Hf, Wf, m, out, stream, true, fa);
}

extern "C" int sd_project_grid_nhwc(const float *grid, int64_t B, int64_t Hf, int64_t Wf,
                                    const sd_mlp *m, void *out, void *stream) {
    if (((uintptr_t)grid & 15)) {
        sd_set_error("sd_project_grid_nhwc: grid must be 16-byte aligned");
        return -1;
    }
    return sd_project_any(grid, B, Hf, Wf, m, out, stream, true);
}

template <int P, int NV, int NDT>
static int sd_rp_launch(const sd_render_args &a, const sd_head &m, hipStream_t s,
                        const int32_t *list) {
    const int lds_bytes = (SD_LDS_OUT + NDT * 4 * SD_WAVE) * 16 +
                          (SD_RWG / 64) * SD_RECBUF * a.K * sd_rec_words(a.nv) * 4;
    if (lds_bytes > 160 * 1024) {
        sd_set_error("sd_render_proj: LDS image exceeds 160 KiB (K or D too large)");
        return -1;
    }
    int64_t nblk;
    sd_launch_proj(k_render_proj<P, NV, NDT>, a.R, lds_bytes, s, nblk, SD_RWG);
    if (list) nblk = sd_num_cus();  // list mode: the tile grid (workgroup b = list b)
    hipLaunchKernelGGL((k_render_proj<P, NV, NDT>), dim3((unsigned)nblk), dim3(SD_RWG), lds_bytes,
                       s, a, m, list);
    return sd_check_err();
}

template <int P, int NV>
static int sd_rp_ndt(const sd_render_args &a, const sd_head &m, hipStream_t s,
                     const int32_t *list = nullptr) {
    // list mode (overflow fallback, usually empty): the folded head where it exists, so
    // no second launch
    if (!sd_head_hc(m.D) || (list && (m.D == 32 || m.D == 64 || m.D == 128))) {
        switch (m.D / 16) {
            case 2: return sd_rp_launch<P, NV, 2>(a, m, s, list);
            case 4: return sd_rp_launch<P, NV, 4>(a, m, s, list);
            case 8: return sd_rp_launch<P, NV, 8>(a, m, s, list);
        }
    }
    int rc = sd_rp_launch<P, NV, 0>(a, m, s, list);
    if (rc) return rc;
    const int lds_bytes = (m.D >> 4) * 4 * SD_WAVE * 16;
    int64_t nblk;
    sd_launch_proj(k_head_hc<P>, (a.R + 15) / 16, lds_bytes, s, nblk);
    if (list) nblk = sd_num_cus();
    hipLaunchKernelGGL(k_head_hc<P>, dim3((unsigned)nblk), dim3(SD_PWG), lds_bytes, s, a.work, a.R,
                       m, a.dino, a.ld_dino, list);
    return sd_check_err();
}

template <int P>
static int sd_rp_nv(const sd_render_args &a, const sd_head &m, hipStream_t s) {
    return a.nv == 1 ? sd_rp_ndt<P, 1>(a, m, s) : sd_rp_ndt<P, 0>(a, m, s);
}

// work = [hidden-composite scratch of the per-ray kernel][overflow list of the tile kernel]
static int64_t sd_hc_bytes(int64_t R, int32_t D) {
    return sd_head_hc(D) ? R * SD_HC_STRIDE * (int64_t)sizeof(float) : 0;
}
extern "C" int64_t sd_render_proj_work_bytes(int64_t R, int32_t D) {
    return sd_hc_bytes(R, D) + ((4 * sd_ovf_words(R, sd_num_cus()) + 15) / 16) * 16;
}

extern "C" int sd_render_tile_ok(const sd_render_args *a, const sd_head *m);
extern "C" int sd_render_tile_launch(const sd_render_args *a, const sd_head *m, int32_t *ovf,
                                     void *stream);

extern "C" int sd_render_proj(const sd_render_args *args, const sd_head *m, void *stream) {
    if (!args || !m || !m->w_pe || !m->w_sig || !m->w_out || !m->b_dino ||
        (m->dtype != SD_BF16 && m->dtype != SD_F16) || m->D <= 0 || (m->D % 16) ||
        m->D > SD_MAX_D) {
        sd_set_error("sd_render_proj: invalid head (16-bit dtype, D % 16 == 0, D <= 512)");
        return -1;
    }
    if (args->grid_dtype != SD_F16) {
        sd_set_error("sd_render_proj: grid_dtype must be SD_F16 (the projected grid of both "
                     "16-bit modes, sd_field_dtype)");
        return -1;
    }
    if (!args->work) {
        sd_set_error("sd_render_proj: args->work is required (sd_render_proj_work_bytes)");
        return -1;
    }
    sd_render_args a = *args;  // output strides normalised below (0 = dense)
    if (a.R < 0 || a.R >= (1LL << 31) || a.K <= 0 || (a.K % 16) || a.K > 128 || a.ray_dim < 6 ||
        a.rays_per_sb <= 0 || !a.rays || (!a.z && a.ray_dim < 8) ||
        !a.grid || !a.cam_f || !a.depth || !a.dino || a.Hf <= 0 || a.Wf <= 0 ||
        a.nv < 0 || a.nv > SD_MAX_NV || (int64_t)a.Hf * a.Wf * SD_DH * 2 >= (1LL << 32) ||
        (a.nv > 0 && (!a.img || !a.cam_c || !a.rgb || a.Hc <= 0 || a.Wc <= 0))) {
        sd_set_error("sd_render_proj: invalid argument (K % 16 == 0, K <= 128, nv <= 4, "
                     "P plane < 4 GiB)");
        return -1;
    }
    if (a.ld_depth < 0 || a.ld_dino < 0 || a.ld_rgb < 0 ||
        (a.ld_dino && a.ld_dino < m->D) || (a.ld_rgb && a.ld_rgb < 3 * a.nv)) {
        sd_set_error("sd_render_proj: output row strides must be 0 (dense) or >= the row width");
        return -1;
    }
    // the dino rows are written as 16-B vectors: the base and the row stride must keep every
    // row 16-B aligned (packed rows put dino first: [dino | depth | rgb])
    if (((uintptr_t)a.dino & 15) || (a.ld_dino % 4)) {
        sd_set_error("sd_render_proj: dino must be 16-B aligned with ld_dino % 4 == 0");
        return -1;
    }
    if (!a.ld_depth) a.ld_depth = 1;
    if (!a.ld_dino) a.ld_dino = m->D;
    if (!a.ld_rgb) a.ld_rgb = 3 * a.nv;
    if (a.R == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    static const bool no_tile = getenv("SDHIP_NO_TILE") != nullptr;  // diagnostic A/B switch
    if (!no_tile && sd_render_tile_ok(&a, m)) {
        // LDS-staged tile kernel (sdhip_tile.hip); groups whose tap box does not fit a tile
        // buffer are listed and rendered by the per-ray kernel behind it
        int32_t *ovf = (int32_t *)((uint8_t *)a.work + sd_hc_bytes(a.R, m->D));
        int rc = sd_render_tile_launch(&a, m, ovf, stream);
        if (rc) return rc;
        if (m->dtype == SD_F16) return sd_rp_ndt<SD_F16, 1>(a, *m, s, ovf);
        return sd_rp_ndt<SD_BF16, 1>(a, *m, s, ovf);
    }
    if (m->dtype == SD_F16) return sd_rp_nv<SD_F16>(a, *m, s);
    return sd_rp_nv<SD_BF16>(a, *m, s);
}
