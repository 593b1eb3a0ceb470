// sdhip_conv.hip -- the DPT head's large 3x3 convolutions on gfx950 (CDNA4) MFMA.
//
// The reference runs them as torch Conv2d (scenedino/models/backbones/dino/dpt_head.py:
// 160-176, 226-236: DPTHead.project and the output head's two 3x3 convolutions, 256 -> 256
// channels at 96x320 and 192x640 for a 192x640 frame).  Same implicit GEMM as k_gemm's CONV
// form (rows m = output pixels, k = (ky, kx, ci), out-of-image taps read as zeros through
// the buffer bounds), re-tiled for a chip-filling launch with long K (K = 2304):
//   * one 512-thread workgroup per CU, 8 waves as 2 (M) x 4 (N), a 256 x BN output tile
//     (BN = 256: wave tile 128 x 64; BN = 128: 128 x 32) on v_mfma_f32_16x16x32_bf16;
//   * 64-deep K steps, A (im2col rows) and W tiles moved global -> LDS by LDS-DMA
//     (buffer_load ... lds, 8 rows of 128 B per wave instruction) into a ring of RS stages,
//     16-B chunks XOR-swizzled per row on the SOURCE side (conflict-free ds_read_b128 of
//     the fragments, MI355X guide rule 21); the loads of RS - 1 steps stay in flight across
//     the per-step barrier (counted vmcnt, raw s_barrier: never a vmcnt(0) in the loop);
//   * epilogue: bias, bf16 or f32 NHWC rows staged through LDS for 16-B stores.
// 2 x 128 x 64 (or 32) MFMA work per wave per barrier instead of k_gemm<128,128>'s 64 x 64
// with two barriers: the 128-row tiles' structure tops out near 0.75 PFLOP/s on these shapes.
#include <cstdlib>

#include "sdhip_common.h"
#include "sdhip_point.h"

#define CV_BM 256
#define CV_BK 64

typedef __attribute__((ext_vector_type(4))) float cvf4;

__device__ __forceinline__ void cv_dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :: "v"(voff), "s"(rs), "s"(lds_addr) : "memory");
}
// 16-B chunk slot of logical chunk kc in a 128-B tile row (an involution): the 16 rows a
// ds_read_b128 lane group reads land on 16 distinct 16-B bank slots
__device__ __forceinline__ int cv_swz(int row, int kc) { return kc ^ ((row >> 1) & 7); }

template <int BN>
__host__ __device__ constexpr int cv_stages() { return BN >= 256 ? 2 : 3; }
template <int BN>
__host__ __device__ constexpr int cv_ring_bytes() { return cv_stages<BN>() * (CV_BM + BN) * CV_BK * 2; }
// epilogue staging: per wave ER rows x WN values (+16 B pad per row)
template <int BN, bool F32>
__host__ __device__ constexpr int cv_epi_rows() { return F32 && BN >= 256 ? 64 : 128; }
template <int BN, bool F32>
__host__ __device__ constexpr int cv_epi_pitch() { return (BN / 4) * (F32 ? 4 : 2) + 16; }
template <int BN, bool F32>
__host__ __device__ constexpr int cv_lds_bytes() {
    return cv_ring_bytes<BN>() > 8 * cv_epi_rows<BN, F32>() * cv_epi_pitch<BN, F32>()
               ? cv_ring_bytes<BN>() : 8 * cv_epi_rows<BN, F32>() * cv_epi_pitch<BN, F32>();
}

// EPI: SD_EPI_BF16 / SD_EPI_F32 (out (M, ldo) = acc + bias) or SD_EPI_SHUF (the
// ConvTranspose2d(k, stride k) sub-pixel scatter, bf16); CONV: implicit 3x3 im2col A rows
// (else dense A rows of stride lda: the 1x1 convolutions / transposed convolutions)
template <int BN, int EPI, bool CONV>
__global__ void __launch_bounds__(512) k_conv_big(sd_gemm_args g) {
    constexpr bool F32 = EPI == SD_EPI_F32;
    constexpr int BM = CV_BM, BK = CV_BK, RS = cv_stages<BN>();
    constexpr int WN = BN / 4, TJ = WN / 16;       // wave columns, 16-col MFMA tiles per wave
    constexpr int STB = (BM + BN) * BK * 2;        // bytes per ring stage: A rows, then W rows
    constexpr int CA = BM * 8 / 512, CB = BN * 8 / 512;  // 16-B chunks per thread per stage
    constexpr int PER = CA + CB;                   // LDS-DMAs per thread per stage
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
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
    auto issue = [&](int kt) {
        const uint32_t st = lds0 + (uint32_t)(kt % RS) * STB;
        const int k0 = kt * BK;
        const int tap = CONV ? k0 / g.Cin : 0, ci0 = k0 - tap * g.Cin;
        const int ky = tap / 3, kx = tap - 3 * ky;
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            if (!CONV) {
                cv_dma16(rsA, kcA[c] + (uint32_t)k0 * 2u, st + (uint32_t)(8 * c + wave) * 1024u);
                continue;
            }
            const int iy = ciy[c] + ky, ix = cix[c] + kx;
            const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
            const uint32_t off = ok ? (uint32_t)(((cpix[c] + iy * g.W + ix) * g.Cin + ci0) * 2) + kcA[c]
                                    : 0x80000000u;  // past the buffer: the DMA writes zeros (padding)
            cv_dma16(rsA, off, st + (uint32_t)(8 * c + wave) * 1024u);
        }
#pragma unroll
        for (int c = 0; c < CB; ++c)
            cv_dma16(rsB, voB[c] + (uint32_t)k0 * 2u, st + (uint32_t)(BM * BK * 2) + (uint32_t)(8 * c + wave) * 1024u);
    };

    cvf4 acc[8][TJ];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = cvf4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fk = lane >> 4;  // fragment row / 8-deep k group of the lane
#pragma unroll
    for (int i = 0; i < RS - 1; ++i)
        if (i < nk) issue(i);
    for (int kt = 0; kt < nk; ++kt) {
        // stage kt landed: of this thread's DMAs only those of stages kt + 1 .. kt + RS - 2
        // (the ones issued) may be younger
        if (RS >= 3 && kt + RS - 2 < nk)
            asm volatile("s_waitcnt vmcnt(%0)" :: "i"((RS >= 3 ? RS - 2 : 0) * PER) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // every wave's DMAs of stage kt landed, every wave's fragment reads of step kt - 1
        // retired: slot (kt - 1) % RS is free
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (kt + RS - 1 < nk) issue(kt + RS - 1);
        const uint8_t *sa = smem + (kt % RS) * STB;
        const uint8_t *sb = sa + BM * BK * 2;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int kc = 4 * s + fk;
            bf16x8 af[8], bfr[TJ];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = wm * 128 + 16 * i + fr;
                af[i] = *(const bf16x8 *)(sa + row * 128 + 16 * cv_swz(row, kc));
            }
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int row = wn * WN + 16 * j + fr;
                bfr[j] = *(const bf16x8 *)(sb + row * 128 + 16 * cv_swz(row, kc));
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
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
    constexpr int ER = cv_epi_rows<BN, F32>(), PITCH = cv_epi_pitch<BN, F32>();
    constexpr int ES = F32 ? 4 : 2;
    constexpr int CPRW = WN * ES / 16;  // 16-B chunks per wave row
    uint8_t *reg = smem + wave * ER * PITCH;
#pragma unroll
    for (int half = 0; half < 128 / ER; ++half) {
        if (half) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
        for (int i = half * (ER / 16); i < (half + 1) * (ER / 16); ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int r = 16 * i + 4 * fk + e - half * ER;
                    const float v = acc[i][j][e] + bias[j];
                    if (F32)
                        *(float *)(reg + r * PITCH + (16 * j + fr) * 4) = v;
                    else
                        *(__bf16 *)(reg + r * PITCH + (16 * j + fr) * 2) = (__bf16)v;
                }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // the wave stores its own ER x WN block: lane -> (row, 16-B chunk)
#pragma unroll
        for (int it = 0; it < ER * CPRW / 64; ++it) {
            const int idx = it * 64 + lane, r = idx / CPRW, ch = idx - r * CPRW;
            const int64_t m = m0 + wm * 128 + half * ER + r;
            const int64_t n = n0 + wn * WN + ch * (16 / ES);
            if (m < g.M && n < g.N) {
                const uint4 v = *(const uint4 *)(reg + r * PITCH + ch * 16);
                int64_t base = m * g.ldo + n;  // element index of (m, n)
                if (EPI == SD_EPI_SHUF) {  // 8 columns inside one sub-pixel (cout % 8 == 0)
                    const int kk = g.shuf_k, hw = g.in_h * g.in_w, cout = (int)(g.N / (kk * kk));
                    const int b = (int)((uint32_t)m / (uint32_t)hw);
                    const int pix = (int)(m - (int64_t)b * hw);
                    const int y = pix / g.in_w, x = pix - y * g.in_w;
                    const int sub = (int)(n / cout), co = (int)(n - (int64_t)sub * cout);
                    const int dy = sub / kk, dx = sub - dy * kk;
                    base = (((int64_t)b * g.in_h * kk + y * kk + dy) * (g.in_w * kk) + x * kk + dx) * cout + co;
                }
                *(uint4 *)((uint8_t *)g.out + base * ES) = v;
            }
        }
    }
}

// The shapes this kernel takes (else sd_gemm's k_gemm path), with enough output tiles to
// give every CU a 256-row tile: a 3x3 stride-1 convolution with Cin % 64 == 0 and a plain
// bf16 / f32 epilogue (bias only), or a dense GEMM with K % 64 == 0 and a plain bf16 or the
// transposed-convolution (SHUF) epilogue; N % 128 == 0.  BN = 256 when the 256 x 256 tiles
// cover the CUs about twice (192x640: 480 tiles), else 256 x 128 tiles (96x320: 240).
// Returns 1 when launched, 0 when the shape is not one of these (the caller runs k_gemm),
// -2 on a launch error.  SD_CONV_BIG=0 in the environment (read per call) disables it
// (tests, A/B runs).
int sd_conv_big_try(const sd_gemm_args *args, void *stream) {
    const char *e = getenv("SD_CONV_BIG");
    if (e && e[0] == '0') return 0;
    const sd_gemm_args &g = *args;
    if (g.res || g.res2 || g.N % 128 || g.K % CV_BK) return 0;
    if (g.conv) {
        if (g.stride != 1 || g.relu_in || g.Cin % 64 || g.K != 9LL * g.Cin ||
            (g.epi != SD_EPI_BF16 && g.epi != SD_EPI_F32) || g.ldo % 8 || g.ldo < g.N)
            return 0;
    } else {
        if (g.lda % 8 || g.lda < g.K) return 0;
        if (g.epi == SD_EPI_SHUF) {
            if (g.shuf_k <= 0 || (g.N / (g.shuf_k * g.shuf_k)) % 8) return 0;
        } else if (g.epi != SD_EPI_BF16 || g.ldo % 8 || g.ldo < g.N) {
            return 0;
        }
    }
    const int ncu = sd_num_cus();
    const int64_t t256 = (g.M + CV_BM - 1) / CV_BM;
    if (t256 * (g.N / 128) < (int64_t)ncu * 7 / 8) return 0;  // too few tiles: k_gemm's split forms
    const int64_t a_bytes = g.conv ? (g.M / ((int64_t)g.OH * g.OW)) * g.H * g.W * g.Cin * 2 : g.M * g.lda * 2;
    if (a_bytes >= ((int64_t)1 << 31) || g.N * g.K * 2 >= ((int64_t)1 << 31)) return 0;
    const bool wide = g.N % 256 == 0 && t256 * (g.N / 256) >= (int64_t)ncu * 15 / 8;
    hipStream_t s = (hipStream_t)stream;
    auto go = [&](auto kern, int bn, int lds) {
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)t256, (unsigned)(g.N / bn)), dim3(512), lds, s, g);
    };
#define CV_GO(BNV, E, C) go(k_conv_big<BNV, E, C>, BNV, cv_lds_bytes<BNV, E == SD_EPI_F32>())
    if (g.conv) {
        if (wide) {
            if (g.epi == SD_EPI_F32) CV_GO(256, SD_EPI_F32, true); else CV_GO(256, SD_EPI_BF16, true);
        } else {
            if (g.epi == SD_EPI_F32) CV_GO(128, SD_EPI_F32, true); else CV_GO(128, SD_EPI_BF16, true);
        }
    } else {
        if (wide) {
            if (g.epi == SD_EPI_SHUF) CV_GO(256, SD_EPI_SHUF, false); else CV_GO(256, SD_EPI_BF16, false);
        } else {
            if (g.epi == SD_EPI_SHUF) CV_GO(128, SD_EPI_SHUF, false); else CV_GO(128, SD_EPI_BF16, false);
        }
    }
#undef CV_GO
    return hipGetLastError() == hipSuccess ? 1 : -2;
}
