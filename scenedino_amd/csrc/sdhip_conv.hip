// sdhip_conv.hip -- the DPT head's full-chip convolutions on gfx950 (CDNA4) MFMA.
//
// The reference runs them as torch Conv2d / ConvTranspose2d (scenedino/models/backbones/dino/
// dpt_head.py:160-176, 226-236: the residual conv units at 48x160, DPTHead.project and the
// output head at 96x320 and 192x640, 256 channels, for a 192x640 frame).  Same implicit GEMM
// as k_gemm's CONV form (rows m = output pixels, k = (ky, kx, ci), out-of-image taps read as
// zeros through the buffer bounds), re-tiled for launches whose tiles cover the CUs:
//   * one 512-thread workgroup per CU, 8 waves as 2 (M) x 4 (N), a BM x BN output tile
//     (256 x 256: wave tile 128 x 64; 256 x 128; 128 x 128; 128 x 64: 64 x 16) on
//     v_mfma_f32_16x16x32_bf16;
//   * 64-deep K steps, A (im2col rows) and W tiles moved global -> LDS by LDS-DMA
//     (buffer_load ... lds, 8 rows of 128 B per wave instruction) into a ring of RS stages,
//     16-B chunks XOR-swizzled per row on the SOURCE side (conflict-free ds_read_b128 of
//     the fragments, MI355X guide rule 21); the loads of RS - 1 steps stay in flight across
//     the per-step barrier (counted vmcnt, raw s_barrier: never a vmcnt(0) in the loop);
//   * the residual units' pre-activation ReLU on the A fragments (v_pk_max_i16 on the bf16
//     bit patterns: sign set -> +0);
//   * epilogue: bias (+ the bf16 residuals), bf16 or f32 NHWC rows or the sub-pixel scatter
//     of a ConvTranspose2d(k, stride k), staged per wave through LDS for 16-B stores.
// 2 x 128 x 64 MFMA work per wave per barrier at 256 x 256 instead of k_gemm<128,128>'s
// 64 x 64 with two barriers: the 128-row tiles' structure tops out near 0.75 PFLOP/s here.
#include <cstdlib>

#include "sdhip_common.h"
#include "sdhip_point.h"

#define CV_BK 64
#define CV_LDS_MAX (144 * 1024)

typedef __attribute__((ext_vector_type(4))) float cvf4;
typedef __attribute__((ext_vector_type(2))) short cvs2;

// LDS-DMA of 16 B per lane: source = buffer + voff (per lane) + soff (wave-uniform), LDS
// destination = lds_addr + 16 lane (M0 set in the same asm, the DMA right behind it)
__device__ __forceinline__ void cv_dma16s(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                 :: "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff) : "memory");
}
// 16-B chunk slot of logical chunk kc in a 128-B tile row (an involution): the 16 rows a
// ds_read_b128 lane group reads land on 16 distinct 16-B bank slots
__device__ __forceinline__ int cv_swz(int row, int kc) { return kc ^ ((row >> 1) & 7); }

// ReLU of 8 bf16 values: as int16 a bf16 with the sign bit set is negative (-0 included)
__device__ __forceinline__ bf16x8 cv_relu8(bf16x8 v) {
    uint4 u = __builtin_bit_cast(uint4, v);
    const cvs2 z = {0, 0};
    u.x = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(cvs2, u.x), z));
    u.y = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(cvs2, u.y), z));
    u.z = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(cvs2, u.z), z));
    u.w = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(cvs2, u.w), z));
    return __builtin_bit_cast(bf16x8, u);
}

template <int BM, int BN>
__host__ __device__ constexpr int cv_stage_bytes() { return (BM + BN) * CV_BK * 2; }
// CV_RELU_LDS = 1: rectify the A chunks once in LDS (one step ahead) instead of on every
// fragment read; measured slower on the 48x160 residual units (30.5 vs 25.1 us, one step
// less in flight and the extra LDS pass on the critical path), so off
#ifndef CV_RELU_LDS
#define CV_RELU_LDS 0
#endif
#ifndef CV_SPLIT_ISSUE
#define CV_SPLIT_ISSUE 1
#endif
#ifndef CV_CHUNK_MAJOR
#define CV_CHUNK_MAJOR 1
#endif
#ifndef CV_MAX_STAGES
#define CV_MAX_STAGES 6
#endif
// as many ring stages as fit (at most CV_MAX_STAGES): the loop is bound by the bytes each CU
// keeps in flight (L2 / Infinity Cache latency), not by the MFMA
template <int BM, int BN>
__host__ __device__ constexpr int cv_stages() {
    return CV_LDS_MAX / cv_stage_bytes<BM, BN>() >= CV_MAX_STAGES ? CV_MAX_STAGES : CV_LDS_MAX / cv_stage_bytes<BM, BN>();
}
// s_waitcnt vmcnt(A * PER) for a runtime A in [0, RS - 2] (the immediate must be a constant)
template <int PER, int RS>
__device__ __forceinline__ void cv_wait_ahead(int ahead) {
    if (RS >= 6 && ahead >= 4) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(4 * PER) : "memory");
    else if (RS >= 5 && ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(3 * PER) : "memory");
    else if (RS >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(2 * PER) : "memory");
    else if (RS >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "i"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// epilogue staging: f32 when the output is f32 or residuals are added before the bf16
// rounding, else bf16; per wave ER rows of WN values + 16 B
// waves along M of the 8-wave grid (the rest along N): 4 x 2 for the 128 x 64 tiles (wave
// tile 32 x 32: 64 KiB of fragment reads per K step instead of 80 with 64 x 16), else 2 x 4
#ifndef CV_WGM4
#define CV_WGM4 1
#endif
template <int BM, int BN>
__host__ __device__ constexpr int cv_wgm() { return CV_WGM4 && BM == 128 && BN == 64 ? 4 : 2; }
template <int BM, int BN, bool STF32>
__host__ __device__ constexpr int cv_epi_pitch() { return (BN / (8 / cv_wgm<BM, BN>())) * (STF32 ? 4 : 2) + 16; }
template <int BM, int BN, bool STF32>
__host__ __device__ constexpr int cv_epi_rows() {
    return 8 * (BM / cv_wgm<BM, BN>()) * cv_epi_pitch<BM, BN, STF32>() <= CV_LDS_MAX ? BM / cv_wgm<BM, BN>()
                                                                                   : BM / cv_wgm<BM, BN>() / 2;
}
template <int BM, int BN, bool STF32>
__host__ __device__ constexpr int cv_lds_bytes() {
    return cv_stages<BM, BN>() * cv_stage_bytes<BM, BN>() > 8 * cv_epi_rows<BM, BN, STF32>() * cv_epi_pitch<BM, BN, STF32>()
               ? cv_stages<BM, BN>() * cv_stage_bytes<BM, BN>()
               : 8 * cv_epi_rows<BM, BN, STF32>() * cv_epi_pitch<BM, BN, STF32>();
}

// XCD-aware tile order (MI355X guide §5 T1, the bijective form): the hardware deals
// workgroups round-robin over the 8 XCDs (linear id % 8); this maps XCD x's workgroups to
// one contiguous range of (row tile, column tile) pairs, column tiles of a row tile
// adjacent, so the row tiles an XCD runs at once share their input rows (3x3 halos) and
// weights in that XCD's L2 instead of every XCD streaming every row.  CV_XCD_REMAP=0: off.
#ifndef CV_XCD_REMAP
#define CV_XCD_REMAP 1
#endif
__device__ __forceinline__ void cv_tile_of(int &mt, int &nt) {
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy;
    const int lin = blockIdx.x + gx * blockIdx.y;
    int w = lin;
    if (CV_XCD_REMAP && nwg > 8) {
        const int xcd = lin & 7, q = nwg >> 3, r = nwg & 7;
        w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (lin >> 3);
    }
    mt = w / gy;
    nt = w - mt * gy;
}

// EPI: SD_EPI_BF16 / SD_EPI_F32 (out (M, ldo) = acc + bias [+ res + res2 when RES]) or
// SD_EPI_SHUF (the ConvTranspose2d(k, stride k) sub-pixel scatter, bf16); CONV: implicit
// 3x3 im2col A rows (else dense A rows of stride lda: 1x1 / transposed convolutions);
// RELU: ReLU on the A operand (the pre-activation of the residual conv units)
// Output rows stored write-through (sc1, CV_WT): a full-chip layer's tens of MB of output
// would otherwise sit partly dirty in L2 when the kernel ends, and the next launch writes
// them back before it starts (MI355X_MICROARCH.md: boundary + dirty bytes / 6 TB/s).  Inline
// asm with its own s_nop 1 (the data registers must not be rewritten before the store
// reads them).
#ifndef CV_WT
#define CV_WT 1
#endif
__device__ __forceinline__ void cv_store16(uint8_t *p, uint4 v) {
    if (CV_WT)
    {
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        const u4v w = __builtin_bit_cast(u4v, v);
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(w) : "memory");
    }
    else
        *(uint4 *)p = v;
}

template <int BM, int BN, int EPI, bool CONV, bool RELU, bool RES>
__global__ void __launch_bounds__(512) k_conv_big(sd_gemm_args g) {
    constexpr bool OUTF32 = EPI == SD_EPI_F32, STF32 = OUTF32 || RES;
    constexpr int BK = CV_BK, RS = cv_stages<BM, BN>(), STB = cv_stage_bytes<BM, BN>();
    constexpr int WGM = cv_wgm<BM, BN>(), WGN = 8 / WGM;
    constexpr int WM = BM / WGM, WN = BN / WGN, TI = WM / 16, TJ = WN / 16;  // wave tile, 16x16 MFMA tiles
    constexpr int CA = BM * 8 / 512, CB = BN * 8 / 512;  // 16-B DMA chunks per thread per stage
    constexpr int PER = CA + CB;
    static_assert(CB >= 1 && TJ >= 1 && RS >= 2 && RS <= 6 && (RS - 2) * PER <= 63, "tile shape");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WGN, wn = wave % WGN;
    int mt, nt;
    cv_tile_of(mt, nt);
    const int64_t m0 = (int64_t)mt * BM, n0 = (int64_t)nt * BN;
    const int nk = (int)(g.K / BK);
    const int64_t a_bytes = CONV ? (g.M / ((int64_t)g.OH * g.OW)) * g.H * g.W * g.Cin * 2 : g.M * g.lda * 2;
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(g.a), 0, (uint32_t)a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void *>(g.w), 0, (uint32_t)(g.N * g.K * 2), 0x00020000);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)smem;

    // this thread's DMA chunks: wave instruction q = 8 c + wave fills LDS bytes
    // [1024 q, 1024 q + 1024) = tile rows 8 q .. 8 q + 7; lane -> row 8 q + lane / 8, slot
    // lane % 8, which holds source chunk cv_swz(row, slot)
    int cpix[CA], ciy[CA], cix[CA];
    uint32_t kcA[CA], voB[CB];
#pragma unroll
    for (int c = 0; c < CA; ++c) {
        const int row = 8 * (8 * c + wave) + (lane >> 3);
        kcA[c] = (uint32_t)cv_swz(row, lane & 7) * 16u;
        const int64_t m = min(m0 + row, g.M - 1);
        if (!CONV) {  // dense rows: the whole fixed part of the source offset
            kcA[c] += (uint32_t)(m * g.lda * 2);
            continue;
        }
        const int ohw = g.OH * g.OW;
        const int b = (int)((uint32_t)m / (uint32_t)ohw);
        const int p = (int)(m - (int64_t)b * ohw);
        const int oy = p / g.OW, ox = p - oy * g.OW;
        cpix[c] = b * g.H * g.W;
        ciy[c] = oy * g.stride - 1;
        cix[c] = ox * g.stride - 1;
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int row = 8 * (8 * c + wave) + (lane >> 3);
        voB[c] = (uint32_t)((min(n0 + row, g.N - 1) * g.K) * 2) + (uint32_t)cv_swz(row, lane & 7) * 16u;
    }
    // conv K order: channel-chunk major, tap minor -- step kt = (chunk kt / 9, tap kt % 9),
    // the matching W columns tap Cin + 64 chunk .. + 63 (any order of the K steps gives the
    // same sum up to fp32 rounding).  The 9 taps of a chunk read the same input pixels
    // (shifted by one pixel or row) in 9 consecutive steps, so the tile's input rows are
    // re-read from L2 instead of from beyond it (tap-major order re-read each row 3 rows'
    // worth of steps later, after the XCD's tiles had streamed ~3x its L2 through).
    // The chunk's channel offset goes in the DMA's scalar offset.
    auto issue = [&](int kt, int parts = 3) {  // parts: 1 = the A tile, 2 = the W tile
        const uint32_t st = lds0 + (uint32_t)(kt % RS) * STB;
        int tap = 0, ci0 = kt * BK;
        if (CONV && CV_CHUNK_MAJOR) {
            const int chunk = kt / 9;
            tap = kt - 9 * chunk;
            ci0 = chunk * BK;
        } else if (CONV) {  // tap-major (the weight layout's own order; A/B runs)
            tap = ci0 / g.Cin;
            ci0 -= tap * g.Cin;
        }
        const int ky = tap / 3, kx = tap - 3 * ky;
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            if (!(parts & 1)) break;
            uint32_t vo = kcA[c];
            if (CONV) {
                const int iy = ciy[c] + ky, ix = cix[c] + kx;
                const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
                // past the buffer (also with the channel offset added): the DMA writes zeros
                vo = ok ? (uint32_t)((cpix[c] + iy * g.W + ix) * g.Cin * 2) + kcA[c] : 0x80000000u;
            }
            cv_dma16s(rsA, vo, (uint32_t)ci0 * 2u, st + (uint32_t)(8 * c + wave) * 1024u);
        }
        const uint32_t kb = (uint32_t)(CONV ? tap * g.Cin + ci0 : ci0) * 2u;  // W column offset
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            if (!(parts & 2)) break;
            cv_dma16s(rsB, voB[c], kb, st + (uint32_t)(BM * BK * 2) + (uint32_t)(8 * c + wave) * 1024u);
        }
    };
    // ReLU of the A chunks this thread DMA'd into stage kt, in place (after its own vmcnt
    // covers them; the next barrier publishes them): once per element, not once per
    // fragment read by each of the 4 column waves.  Needs RS >= 3 (stage kt + 1 is waited
    // for one step early); RS = 2 tiles apply it to the fragments instead.
    constexpr bool RELU_LDS = RELU && RS >= 3 && CV_RELU_LDS, RELU_FRAG = RELU && !RELU_LDS;
    auto relu_own = [&](int kt) {
        uint8_t *st = smem + (kt % RS) * STB;
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            bf16x8 *p = (bf16x8 *)(st + (8 * c + wave) * 1024 + lane * 16);
            *p = cv_relu8(*p);
        }
    };

    cvf4 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = cvf4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fk = lane >> 4;  // fragment row / 8-deep k group of the lane
#pragma unroll
    for (int i = 0; i < RS - 1; ++i)
        if (i < nk) issue(i);
    if (RELU_LDS) {  // stage 0
        cv_wait_ahead<PER, RS>(min(RS - 2, nk - 1));
        relu_own(0);
    }
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed: this thread's DMAs of the issued stages kt + 1 .. kt + RS - 2 may
        // be younger (fewer near the end: no stage is issued past nk - 1).  RELU_LDS: stage
        // kt + 1 landed (stage kt was waited for and rectified one step earlier)
        if (RELU_LDS) {
            if (kt + 1 < nk) {
                cv_wait_ahead<PER, RS>(min(RS - 3, nk - 2 - kt));
                relu_own(kt + 1);
            }
        } else {
            cv_wait_ahead<PER, RS>(min(RS - 2, nk - 1 - kt));
        }
        // every wave's DMAs of stage kt landed, every wave's fragment reads of step kt - 1
        // retired: slot (kt - 1) % RS is free
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // CV_SPLIT_ISSUE: the A tile's DMAs now, the W tile's between the two 32-deep halves
        // of the step's MFMAs (each DMA costs its wave ~60-185 issue cycles; spread between
        // MFMA clusters, MI355X guide "LDS-DMA piece issue cost")
        // (256 x 256 tiles only: 147 -> 143.5 us at 192x640; the 128 x 64 tiles measured
        // 0.5 us slower with it, profiles/r4_dpt_ops.txt)
        constexpr bool SPLIT_ISSUE = CV_SPLIT_ISSUE && BM == 256 && BN == 256;
        const bool nxt = kt + RS - 1 < nk;
        if (nxt) issue(kt + RS - 1, SPLIT_ISSUE ? 1 : 3);
        const uint8_t *sa = smem + (kt % RS) * STB;
        const uint8_t *sb = sa + BM * BK * 2;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if (SPLIT_ISSUE && s == 1 && nxt) issue(kt + RS - 1, 2);
            const int kc = 4 * s + fk;
            bf16x8 af[TI], bfr[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const int row = wm * WM + 16 * i + fr;
                af[i] = *(const bf16x8 *)(sa + row * 128 + 16 * cv_swz(row, kc));
                if (RELU_FRAG) af[i] = cv_relu8(af[i]);
            }
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int row = wn * WN + 16 * j + fr;
                bfr[j] = *(const bf16x8 *)(sb + row * 128 + 16 * cv_swz(row, kc));
            }
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    // every wave is done with the ring (no DMA outstanding: the last steps issued none)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- epilogue: + bias, the wave's tile through its own LDS region, 16-B row stores ----
    // D layout (16x16 tile): lane holds rows 4 (lane >> 4) + e, column lane & 15
    float bias[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int64_t n = min(n0 + wn * WN + 16 * j + fr, g.N - 1);
        bias[j] = g.bias ? g.bias[n] : 0.f;
    }
    constexpr int ER = cv_epi_rows<BM, BN, STF32>(), PITCH = cv_epi_pitch<BM, BN, STF32>();
    constexpr int CC = OUTF32 ? 4 : 8;  // columns per 16-B output store
    constexpr int CPRW = WN / CC;       // store chunks per wave row
    static_assert((ER * CPRW) % 64 == 0, "epilogue chunking");
    uint8_t *reg = smem + wave * ER * PITCH;
#pragma unroll
    for (int part = 0; part < WM / ER; ++part) {
        if (part) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int i = part * (ER / 16); i < (part + 1) * (ER / 16); ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 16 * i + 4 * fk + e - part * ER;
                    const float v = acc[i][j][e] + bias[j];
                    if (STF32)
                        *(float *)(reg + r * PITCH + (16 * j + fr) * 4) = v;
                    else
                        *(__bf16 *)(reg + r * PITCH + (16 * j + fr) * 2) = (__bf16)v;
                }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // the wave stores its own ER x WN block: lane -> (row, chunk of CC columns); the
        // lane's chunk (so its columns) is the same in every iteration, its row advances by
        // 64 / CPRW
        // SHUF: the lane's (image, y, x) of its first row by two divides, then stepped; its
        // sub-pixel and channel once (per-chunk 64-bit divides made the epilogue VALU-bound)
        uint32_t sb = 0, sy = 0, sx = 0, soff = 0;
        if (EPI == SD_EPI_SHUF) {
            const uint32_t kk = (uint32_t)g.shuf_k, iw = (uint32_t)g.in_w, ih = (uint32_t)g.in_h;
            const uint32_t cout = (uint32_t)(g.N / (kk * kk));
            const uint32_t m_first = (uint32_t)(m0 + wm * WM + part * ER + lane / CPRW);
            sb = m_first / (ih * iw);
            const uint32_t pix = m_first - sb * ih * iw;
            sy = pix / iw;
            sx = pix - sy * iw;
            const uint32_t n = (uint32_t)(n0 + wn * WN + (lane % CPRW) * CC);
            const uint32_t sub = n / cout, co = n - sub * cout, dy = sub / kk, dx = sub - dy * kk;
            soff = dy * iw * kk * cout + dx * cout + co;  // offset of (dy, dx, co) from pixel (y kk, x kk)
        }
        // the residual rows of every iteration loaded before the first store (loads after
        // a store to possibly-aliasing memory wait for it: one round trip per iteration)
        constexpr int NIT = ER * CPRW / 64;
        bf16x8 rpre[RES ? NIT : 1][2];
        if constexpr (RES && STF32 && !OUTF32) {
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int idx = it * 64 + lane, r = idx / CPRW, ch = idx - r * CPRW;
                const int64_t m = m0 + wm * WM + part * ER + r;
                const int64_t n = n0 + wn * WN + ch * CC;
                const bool ok = m < g.M && n < g.N;
#pragma unroll
                for (int u = 0; u < 8; ++u) rpre[it][0][u] = rpre[it][1][u] = (__bf16)0.f;
                if (ok && g.res) rpre[it][0] = *(const bf16x8 *)((const __bf16 *)g.res + m * g.ldo + n);
                if (ok && g.res2) rpre[it][1] = *(const bf16x8 *)((const __bf16 *)g.res2 + m * g.ldo + n);
            }
        }
#pragma unroll
        for (int it = 0; it < ER * CPRW / 64; ++it) {
            const int idx = it * 64 + lane, r = idx / CPRW, ch = idx - r * CPRW;
            const int64_t m = m0 + wm * WM + part * ER + r;
            const int64_t n = n0 + wn * WN + ch * CC;
            int64_t sbase = 0;
            if (EPI == SD_EPI_SHUF) {
                if (it) {  // advance the row by 64 / CPRW pixels
                    sx += 64 / CPRW;
                    while (sx >= (uint32_t)g.in_w) {
                        sx -= (uint32_t)g.in_w;
                        if (++sy == (uint32_t)g.in_h) sy = 0, ++sb;
                    }
                }
                const int64_t kk = g.shuf_k;
                sbase = (((int64_t)sb * g.in_h + sy) * kk * g.in_w + sx) * kk * (g.N / (kk * kk)) + soff;
            }
            if (m >= g.M || n >= g.N) continue;
            uint4 v;
            if (STF32 && !OUTF32) {  // f32 staging, residuals added before the bf16 rounding
                const cvf4 lo = *(const cvf4 *)(reg + r * PITCH + ch * 32);
                const cvf4 hi = *(const cvf4 *)(reg + r * PITCH + ch * 32 + 16);
                float f[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                if constexpr (RES) {
                    if (g.res) {
#pragma unroll
                        for (int u = 0; u < 8; ++u) f[u] += (float)rpre[it][0][u];
                    }
                    if (g.res2) {
#pragma unroll
                        for (int u = 0; u < 8; ++u) f[u] += (float)rpre[it][1][u];
                    }
                }
                bf16x8 o;
#pragma unroll
                for (int u = 0; u < 8; ++u) o[u] = (__bf16)f[u];
                v = __builtin_bit_cast(uint4, o);
            } else {
                v = *(const uint4 *)(reg + r * PITCH + ch * 16);
            }
            // element index of (m, n); SHUF: 8 columns inside one sub-pixel (cout % 8 == 0)
            const int64_t base = EPI == SD_EPI_SHUF ? sbase : m * g.ldo + n;
            cv_store16((uint8_t *)g.out + base * (OUTF32 ? 4 : 2), v);
        }
    }
}

// ---------------------------------------------------------------------------
// Halo tiles: 2-D output tiles of 8 rows x TW pixels for the 3x3 convolutions.  k_conv_big
// streams the im2col rows, so every input pixel crosses L2 -> LDS 9 times per column tile
// (once per tap; PMC: the DPT's 3x3 layers run at ~35 GB/s per CU, bound by the bytes each
// CU keeps in flight, not by the MFMA).  Here each 64-channel chunk of the tile's input
// halo ((8 + 2) x (TW + 2) pixels) is DMA'd into LDS once and the 9 taps read it shifted;
// only the weight tile is streamed per tap (a ring of RSB stages).  K order: chunk major,
// tap minor.  Per-thread halo offsets are fixed for the tile (the chunk's channel offset
// goes in the DMA's scalar offset).  Same 8-wave 2 x 4 MFMA layout, ReLU (on the halo, in
// LDS, once per chunk) and epilogues as k_conv_big.
#define CVH_TH 8
#ifndef CV_HALO
#define CV_HALO 1
#endif
template <int TW>
__host__ __device__ constexpr int cvh_hpix() { return (CVH_TH + 2) * (TW + 2); }
template <int TW>
__host__ __device__ constexpr int cvh_ha() { return (cvh_hpix<TW>() * 8 + 511) / 512; }  // halo DMAs / thread
template <int TW>
__host__ __device__ constexpr int cvh_halo_bytes() { return cvh_ha<TW>() * 512 * 16; }
// (the 256-column tiles take the whole 160 KiB: two weight stages beside the two halos)
template <int BN>
__host__ __device__ constexpr int cvh_lds_max() { return BN == 256 ? 160 * 1024 : CV_LDS_MAX; }
template <int TW, int BN>
__host__ __device__ constexpr int cvh_rsb() {
    return (cvh_lds_max<BN>() - 2 * cvh_halo_bytes<TW>()) / (BN * 128) >= 6 ? 6 : (cvh_lds_max<BN>() - 2 * cvh_halo_bytes<TW>()) / (BN * 128);
}
template <int TW, int BN, bool STF32>
__host__ __device__ constexpr int cvh_lds_bytes() {
    return 2 * cvh_halo_bytes<TW>() + cvh_rsb<TW, BN>() * BN * 128 > 8 * cv_epi_rows<CVH_TH * TW, BN, STF32>() * cv_epi_pitch<CVH_TH * TW, BN, STF32>()
               ? 2 * cvh_halo_bytes<TW>() + cvh_rsb<TW, BN>() * BN * 128
               : 8 * cv_epi_rows<CVH_TH * TW, BN, STF32>() * cv_epi_pitch<CVH_TH * TW, BN, STF32>();
}
// s_waitcnt vmcnt(n) for a runtime n (the count of this thread's younger DMAs)
__device__ __forceinline__ void cv_vmcnt(int n) {
#define CVW(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    switch (n) {
        CVW(1) CVW(2) CVW(3) CVW(4) CVW(5) CVW(6) CVW(7) CVW(8) CVW(9) CVW(10) CVW(11) CVW(12)
        CVW(13) CVW(14) CVW(15) CVW(16)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef CVW
}

template <int TW, int BN, int EPI, bool RELU, bool RES>
__global__ void __launch_bounds__(512) k_conv_halo(sd_gemm_args g) {
    constexpr bool OUTF32 = EPI == SD_EPI_F32, STF32 = OUTF32 || RES;
    constexpr int TH = CVH_TH, BM = TH * TW, HW2 = TW + 2;
    constexpr int HP = cvh_hpix<TW>(), HA = cvh_ha<TW>(), HB = cvh_halo_bytes<TW>();
    constexpr int RSB = cvh_rsb<TW, BN>(), SBB = BN * 128;
    constexpr int WM = BM / 2, WN = BN / 4, TI = WM / 16, TJ = WN / 16;
    constexpr int CB = BN * 8 / 512;
    static_assert(CB >= 1 && TJ >= 1 && RSB >= 2 && TW % 16 == 0 && (RSB - 2) * CB + HA <= 16, "halo tile shape");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int txn = (g.OW + TW - 1) / TW, tyn = (g.OH + TH - 1) / TH;
    int tile, ntile;
    cv_tile_of(tile, ntile);
    const int b = tile / (txn * tyn), trem = tile - b * txn * tyn;
    const int ty = trem / txn, tx = trem - ty * txn;
    const int y0 = ty * TH, x0 = tx * TW;
    const int64_t n0 = (int64_t)ntile * BN;
    const int nch = g.Cin / CV_BK, nk = 9 * nch;
    const int64_t a_bytes = (g.M / ((int64_t)g.OH * g.OW)) * g.H * g.W * g.Cin * 2;
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(g.a), 0, (uint32_t)a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<void *>(g.w), 0, (uint32_t)(g.N * g.K * 2), 0x00020000);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)smem;
    const uint32_t ldsB = lds0 + 2 * HB;

    // halo DMA chunks: wave instruction q = 8 h + wave fills LDS bytes [1024 q, + 1024) of
    // the halo buffer = halo pixels 8 q .. 8 q + 7; lane -> pixel 8 q + lane / 8, slot
    // lane % 8 (holding source chunk cv_swz(pixel, slot)); pixels past the halo and outside
    // the image read as zeros
    uint32_t voH[HA];
#pragma unroll
    for (int q = 0; q < HA; ++q) {
        const int hp = 8 * (8 * q + wave) + (lane >> 3);
        const int hr = hp / HW2, hc = hp - hr * HW2;
        const int y = y0 - 1 + hr, x = x0 - 1 + hc;
        const bool ok = hp < HP && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
        voH[q] = ok ? (uint32_t)((((int64_t)b * g.H + y) * g.W + x) * g.Cin * 2) + (uint32_t)cv_swz(hp, lane & 7) * 16u
                    : 0x80000000u;
    }
    uint32_t voB[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int row = 8 * (8 * c + wave) + (lane >> 3);
        voB[c] = (uint32_t)((min(n0 + row, g.N - 1) * g.K) * 2) + (uint32_t)cv_swz(row, lane & 7) * 16u;
    }
    // group s: the weight tile of step s (+ the halo of chunk s / 9 when s starts a chunk)
    auto issue = [&](int s) {
        const int chunk = s / 9, tap = s - 9 * chunk, ci0 = chunk * CV_BK;
        const uint32_t kb = (uint32_t)(tap * g.Cin + ci0) * 2u;
#pragma unroll
        for (int c = 0; c < CB; ++c)
            cv_dma16s(rsB, voB[c], kb, ldsB + (uint32_t)(s % RSB) * SBB + (uint32_t)(8 * c + wave) * 1024u);
        if (tap == 0) {
#pragma unroll
            for (int q = 0; q < HA; ++q)
                cv_dma16s(rsA, voH[q], (uint32_t)ci0 * 2u, lds0 + (uint32_t)(chunk & 1) * HB + (uint32_t)(8 * q + wave) * 1024u);
        }
    };
    auto group_size = [&](int s) { return CB + (s % 9 == 0 ? HA : 0); };

    cvf4 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = cvf4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fk = lane >> 4;
    // the lane's fragment pixels: tile row / column of pixel wm WM + 16 i + fr
    int prow[TI], pcol[TI];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
        const int q = wm * WM + 16 * i + fr;
        prow[i] = q / TW;
        pcol[i] = q - prow[i] * TW;
    }

#pragma unroll
    for (int i = 0; i < RSB - 1; ++i)
        if (i < nk) issue(i);
    for (int s = 0; s < nk; ++s) {
        int younger = 0;  // this thread's DMAs issued after group s
        for (int u = s + 1; u <= min(s + RSB - 2, nk - 1); ++u) younger += group_size(u);
        cv_vmcnt(younger);
        const int chunk = s / 9, tap = s - 9 * chunk;
        const uint8_t *hb = smem + (chunk & 1) * HB;
        if (RELU && tap == 0) {  // rectify this thread's halo chunks once (the barrier publishes)
#pragma unroll
            for (int q = 0; q < HA; ++q) {
                bf16x8 *p = (bf16x8 *)(smem + (chunk & 1) * HB + (8 * q + wave) * 1024 + lane * 16);
                *p = cv_relu8(*p);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (s + RSB - 1 < nk) issue(s + RSB - 1);
        const int ky = tap / 3, kx = tap - 3 * ky;
        const uint8_t *sb = smem + 2 * HB + (s % RSB) * SBB;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int kc = 4 * h2 + fk;
            bf16x8 af[TI], bfr[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const int hp = (prow[i] + ky) * HW2 + pcol[i] + kx;
                af[i] = *(const bf16x8 *)(hb + hp * 128 + 16 * cv_swz(hp, kc));
            }
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int row = wn * WN + 16 * j + fr;
                bfr[j] = *(const bf16x8 *)(sb + row * 128 + 16 * cv_swz(row, kc));
            }
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- epilogue (k_conv_big's, with the 2-D tile's pixel -> row map) ----
    float bias[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int64_t n = min(n0 + wn * WN + 16 * j + fr, g.N - 1);
        bias[j] = g.bias ? g.bias[n] : 0.f;
    }
    constexpr int ER = cv_epi_rows<BM, BN, STF32>(), PITCH = cv_epi_pitch<BM, BN, STF32>();
    constexpr int CC = OUTF32 ? 4 : 8;
    constexpr int CPRW = WN / CC;
    static_assert((ER * CPRW) % 64 == 0, "epilogue chunking");
    uint8_t *reg = smem + wave * ER * PITCH;
#pragma unroll
    for (int part = 0; part < WM / ER; ++part) {
        if (part) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int i = part * (ER / 16); i < (part + 1) * (ER / 16); ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 16 * i + 4 * fk + e - part * ER;
                    const float v = acc[i][j][e] + bias[j];
                    if (STF32)
                        *(float *)(reg + r * PITCH + (16 * j + fr) * 4) = v;
                    else
                        *(__bf16 *)(reg + r * PITCH + (16 * j + fr) * 2) = (__bf16)v;
                }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int it = 0; it < ER * CPRW / 64; ++it) {
            const int idx = it * 64 + lane, r = idx / CPRW, ch = idx - r * CPRW;
            const int q = wm * WM + part * ER + r;  // tile pixel
            const int y = y0 + q / TW, x = x0 + q % TW;
            const int64_t n = n0 + wn * WN + ch * CC;
            if (y >= g.OH || x >= g.OW || n >= g.N) continue;
            const int64_t m = ((int64_t)b * g.OH + y) * g.OW + x;
            uint4 v;
            if (STF32 && !OUTF32) {
                const cvf4 lo = *(const cvf4 *)(reg + r * PITCH + ch * 32);
                const cvf4 hi = *(const cvf4 *)(reg + r * PITCH + ch * 32 + 16);
                float f[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                if (RES) {
                    if (g.res) {
                        const bf16x8 a = *(const bf16x8 *)((const __bf16 *)g.res + m * g.ldo + n);
#pragma unroll
                        for (int u = 0; u < 8; ++u) f[u] += (float)a[u];
                    }
                    if (g.res2) {
                        const bf16x8 a = *(const bf16x8 *)((const __bf16 *)g.res2 + m * g.ldo + n);
#pragma unroll
                        for (int u = 0; u < 8; ++u) f[u] += (float)a[u];
                    }
                }
                bf16x8 o;
#pragma unroll
                for (int u = 0; u < 8; ++u) o[u] = (__bf16)f[u];
                v = __builtin_bit_cast(uint4, o);
            } else {
                v = *(const uint4 *)(reg + r * PITCH + ch * 16);
            }
            cv_store16((uint8_t *)g.out + (m * g.ldo + n) * (OUTF32 ? 4 : 2), v);
        }
    }
}

// The shapes this kernel takes (else sd_gemm's k_gemm path), with enough output tiles to
// give every CU one: a 3x3 stride-1 convolution with Cin % 64 == 0 (pre-activation ReLU and
// bf16 residuals allowed) and a bf16 / f32 epilogue, or a dense GEMM with K % 64 == 0 and a
// plain bf16 or the transposed-convolution (SHUF) epilogue; N % 64 == 0.  Tile: 256 x 256
// when those cover the CUs about twice (192x640: 480 tiles), else the first of 256 x 128,
// 128 x 128, 128 x 64 with at least 7/8 of a tile per CU (96x320: 240 of 256 x 128; 48x160:
// 240 of 128 x 64).  Returns 1 when launched, 0 when the shape is not one of these (the
// caller runs k_gemm), -2 on a launch error.  SD_CONV_BIG=0 in the environment (read per
// call) disables it (tests, A/B runs).
int sd_conv_big_try(const sd_gemm_args *args, void *stream) {
    const char *e = getenv("SD_CONV_BIG");
    if (e && e[0] == '0') return 0;
    const sd_gemm_args &g = *args;
    if (g.N % 64 || g.K % CV_BK) return 0;
    const bool res = g.res || g.res2;
    if (g.conv) {
        if (g.stride != 1 || g.Cin % 64 || g.K != 9LL * g.Cin || g.ldo % 8 || g.ldo < g.N ||
            (g.epi != SD_EPI_BF16 && g.epi != SD_EPI_F32) || (res && g.epi != SD_EPI_BF16))
            return 0;
    } else {
        if (g.lda % 8 || g.lda < g.K || res || g.relu_in) return 0;
        if (g.epi == SD_EPI_SHUF) {
            if (g.shuf_k <= 0 || (g.N / (g.shuf_k * g.shuf_k)) % 8) return 0;
        } else if (g.epi != SD_EPI_BF16 || g.ldo % 8 || g.ldo < g.N) {
            return 0;
        }
    }
    const int64_t a_bytes = g.conv ? (g.M / ((int64_t)g.OH * g.OW)) * g.H * g.W * g.Cin * 2 : g.M * g.lda * 2;
    if (a_bytes >= ((int64_t)1 << 31) || g.N * g.K * 2 >= ((int64_t)1 << 31)) return 0;
    const int64_t ncu = sd_num_cus();
    hipStream_t s = (hipStream_t)stream;
    if (g.conv && CV_HALO && !(e && e[0] == 'b')) {  // SD_CONV_BIG=b: the im2col tiles only
        const int64_t nb = g.M / ((int64_t)g.OH * g.OW);
        auto htiles = [&](int tw, int bn) {
            return g.N % bn ? 0 : nb * ((g.OH + CVH_TH - 1) / CVH_TH) * ((g.OW + tw - 1) / tw) * (g.N / bn);
        };
        // 8 x 32 halo tiles where the im2col tiles would be 256 x 128 (96x320: 43.5 vs 47.8
        // us); the 192x640 layer keeps the 256 x 256 im2col tiles (143 vs 161 us with 128-
        // column halo tiles) and the 48x160 residual units the 128 x 64 ones (25 vs 34 us with
        // 8 x 16 halo tiles; tools/dpt_ops_bench.py, profiles/r4_dpt_ops.txt)
        int tw = 0, hbn = 0;
        const int64_t t256 = ((g.M + 255) / 256) * (g.N % 256 ? 0 : g.N / 256);
        if (t256 < ncu * 15 / 8 && g.OW >= 32 && htiles(32, 128) >= ncu * 7 / 8) tw = 32, hbn = 128;
        // 8 x 32 halo tiles of all 256 output channels where the im2col tiles would be
        // 256 x 256 (the 192x640 output conv): 143 -> 132 us, bit-equal (the same K order;
        // tools/conv_halo256_ab.py, profiles/r6_dpt/conv_halo256_ab.txt).  SD_CONV_HALO256=0:
        // the im2col tiles
        const char *h256 = getenv("SD_CONV_HALO256");
        if (!tw && !(h256 && h256[0] == '0') && g.N % 256 == 0 && g.OW >= 32 && t256 >= ncu * 15 / 8)
            tw = 32, hbn = 256;
        if (tw) {
            auto hgo = [&](auto kern, int lds) {
                sd_lds_attr((const void *)kern, lds);
                hipLaunchKernelGGL(kern, dim3((unsigned)(htiles(tw, hbn) / (g.N / hbn)), (unsigned)(g.N / hbn)),
                                   dim3(512), lds, s, g);
            };
#define CVH_K(TW_, BN_, E, R, RS_) hgo(k_conv_halo<TW_, BN_, E, R, RS_>, cvh_lds_bytes<TW_, BN_, E == SD_EPI_F32 || RS_>())
#define CVH_TILE(TW_, BN_)                                                                           \
            if (tw == TW_) {                                                                         \
                if (g.epi == SD_EPI_F32) {                                                           \
                    if (g.relu_in) CVH_K(TW_, BN_, SD_EPI_F32, true, false);                         \
                    else CVH_K(TW_, BN_, SD_EPI_F32, false, false);                                  \
                } else if (res) {                                                                    \
                    if (g.relu_in) CVH_K(TW_, BN_, SD_EPI_BF16, true, true);                         \
                    else CVH_K(TW_, BN_, SD_EPI_BF16, false, true);                                  \
                } else {                                                                             \
                    if (g.relu_in) CVH_K(TW_, BN_, SD_EPI_BF16, true, false);                        \
                    else CVH_K(TW_, BN_, SD_EPI_BF16, false, false);                                 \
                }                                                                                    \
            }
            if (hbn == 128) {
                CVH_TILE(32, 128)
            } else {
                CVH_TILE(32, 256)
            }
#undef CVH_TILE
#undef CVH_K
            return hipGetLastError() == hipSuccess ? 1 : -2;
        }
    }
    auto tiles = [&](int bm, int bn) { return g.N % bn ? 0 : ((g.M + bm - 1) / bm) * (g.N / bn); };
    int bm, bn;
    if (tiles(256, 256) >= ncu * 15 / 8) bm = 256, bn = 256;
    else if (tiles(256, 128) >= ncu * 7 / 8) bm = 256, bn = 128;
    else if (tiles(128, 128) >= ncu * 7 / 8) bm = 128, bn = 128;
    else if (tiles(128, 64) >= ncu * 7 / 8) bm = 128, bn = 64;
    else return 0;
    auto go = [&](auto kern, int lds) {
        sd_lds_attr((const void *)kern, lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)((g.M + bm - 1) / bm), (unsigned)(g.N / bn)), dim3(512), lds, s, g);
    };
#define CV_K(BM_, BN_, E, C, R, RS_) go(k_conv_big<BM_, BN_, E, C, R, RS_>, cv_lds_bytes<BM_, BN_, E == SD_EPI_F32 || RS_>())
#define CV_TILE(BM_, BN_)                                                                            \
    if (bm == BM_ && bn == BN_) {                                                                    \
        if (!g.conv) {                                                                               \
            if (g.epi == SD_EPI_SHUF) CV_K(BM_, BN_, SD_EPI_SHUF, false, false, false);              \
            else CV_K(BM_, BN_, SD_EPI_BF16, false, false, false);                                   \
        } else if (g.epi == SD_EPI_F32) {                                                            \
            if (g.relu_in) CV_K(BM_, BN_, SD_EPI_F32, true, true, false);                            \
            else CV_K(BM_, BN_, SD_EPI_F32, true, false, false);                                     \
        } else if (res) {                                                                            \
            if (g.relu_in) CV_K(BM_, BN_, SD_EPI_BF16, true, true, true);                            \
            else CV_K(BM_, BN_, SD_EPI_BF16, true, false, true);                                     \
        } else {                                                                                     \
            if (g.relu_in) CV_K(BM_, BN_, SD_EPI_BF16, true, true, false);                           \
            else CV_K(BM_, BN_, SD_EPI_BF16, true, false, false);                                    \
        }                                                                                            \
    }
    CV_TILE(256, 256) else CV_TILE(256, 128) else CV_TILE(128, 128) else CV_TILE(128, 64)
#undef CV_TILE
#undef CV_K
    return hipGetLastError() == hipSuccess ? 1 : -2;
}
