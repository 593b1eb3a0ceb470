// sdhip_vit.hip -- DINO / DINOv2 ViT encoder blocks on gfx950 (CDNA4) MFMA.
//
// The reference runs timm's VisionTransformer (scenedino/models/backbones/dino/vit.py:48-62,
// 112-189, wrapped by DINOv2Encoder, dinov2_module.py:230-288): patch-embed convolution,
// + class token + position embedding, depth x pre-LN Block
//     x = x + ls1 * proj(attn(norm1(x)))        (qkv with bias, softmax(q k^T / sqrt(hd)) v)
//     x = x + ls2 * fc2(gelu(fc1(norm2(x))))    (exact-erf GELU; LayerNorm eps 1e-6)
// then the final norm.  Kernels here:
//   k_gemm<BM,BN,EPI>  bf16 x bf16 -> fp32 MFMA (v_mfma_f32_32x32x16_bf16) "NT" GEMM
//                      out = A (M,K) . W (N,K)^T + bias with fused epilogues: bf16 store,
//                      GELU, fp32 residual update with layer scale, qkv scatter into the
//                      attention layouts, patch-embed scatter (+ position embedding).
//   k_attn             flash attention, head_dim 64, any token count: S^T = K Q^T per
//                      64-key block with the query on the MFMA lane (softmax row reductions
//                      stay in the lane), online softmax in fp32, O^T = V^T P with P taken
//                      straight from the S^T accumulator as the B operand (no LDS trip).
//   k_layernorm        one wave per token, fp32 in, bf16 out (the next GEMM's A operand).
//   k_patchify         input normalisation ((x/2+0.5-mean)/std, dinov2_module.py:225-227)
//                      + im2col of the patch-embed convolution, + class-token rows.
//   k_tokens_to_grid   drop prefix tokens, (B,T,C) -> (B,C,h,w), optional L2 normalise
//                      (vit.py:188, dinov2_module.py:270-287).
// Residual stream x is fp32 (B*T, C); GEMM operands bf16; all accumulation fp32.
#include <cstdlib>
#include <cstring>

#include "sdhip_common.h"
#include "sdhip_point.h"

extern "C" void sd_set_error(const char *msg);
int sd_conv_big_try(const sd_gemm_args *args, void *stream);  // sdhip_conv.hip

typedef __attribute__((ext_vector_type(4))) float vf4;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;

#define VT_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ f32x16 vt_zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

// ---------------------------------------------------------------------------
// GEMM
// ---------------------------------------------------------------------------
#ifndef VT_NS_BIG
#define VT_NS_BIG 2    // staging-ring depth of the 128 x 128 tiles
#endif
#ifndef VT_NS_SMALL
#define VT_NS_SMALL 2  // staging-ring depth of the 64 x 64 and 32 x 32 split-K tiles (4, 6: slower)
#endif
// VT_MF16 = 1: the GEMM's 32 x 32 accumulator blocks computed as 2 x 2
// v_mfma_f32_16x16x32_bf16 tiles instead of one v_mfma_f32_32x32x16_bf16 (register q of block
// (i, j) is element q & 3 of sub-tile q >> 2 = 2 a + b: row 16 a + 4 (lane >> 4) + (q & 3),
// column 16 b + (lane & 15)).  Measured 4-13 % slower on every encoder shape
// (tools/gemm_bench.py: 16 more VGPRs on the 128 x 128 tile, twice the fragment reads per
// MFMA cycle), so off.
#ifndef VT_MF16
#define VT_MF16 0
#endif
// VT_RING = 1: the K loop's A / W tiles go global -> LDS by LDS-DMA (buffer_load ... lds,
// per-lane source offsets) into a ring of vt_ring_stages() stages, so several K steps are in
// flight at once and a step waits for its own tile only (the register-staging loop of
// round 3 hid at most one step of load latency: the small ViT / DPT GEMMs of a 481-token
// or 12x40..48x160 frame are latency-bound).  The tiles sit unpadded in LDS with their
// 16-B chunks XOR-swizzled per row (vt_swz), which keeps the fragment reads conflict-free.
#ifndef VT_RING
#define VT_RING 1  // round 4 A/B (graph-replayed passes, 2 reps): ViT-S/16 0.615 -> 0.599 ms, encode 1.30 -> 1.276
#endif
#ifndef VT_RS_SK
#define VT_RS_SK 4  // ring stages of the 32 x 32 split-K tiles (16 KiB each at BK = 128)
#endif
__host__ __device__ constexpr int vt_ring_stages(int BM, int BN) { return BM >= 128 || BN >= 128 ? 3 : BM == 32 ? VT_RS_SK : 4; }
// which tiles take the ring: the 32 x 32 split-K tiles of the small-M GEMMs (ViT-S/16 and
// DINOv2-B/14 at 481 tokens, the DPT's 12x40 / 24x80 convolutions).  VT_RING_ALL = 1 puts
// every tile on it (the 64 x 64 and 128 x 128 tiles measured slower: one 96-KiB ring per CU
// halves their occupancy -- ViT-B/8 + DPT 3.46 -> 4.13 ms)
#ifndef VT_RING_ALL
#define VT_RING_ALL 0
#endif
__host__ __device__ constexpr bool vt_ring_tile(int BM) { return VT_RING && !VT_MF16 && (BM == 32 || VT_RING_ALL); }
template <int BM, int BN, int BK>
__host__ __device__ constexpr int vt_ring_bytes() { return vt_ring_stages(BM, BN) * (BM + BN) * BK * 2; }
// chunk slot of 16-B chunk kc of tile row `row` (CPR chunks per row): rows sharing 256 B of
// LDS use disjoint chunk sets, 16 consecutive rows cover the 64 banks once
template <int CPR>
__device__ __forceinline__ int vt_swz(int row, int kc) {
    if constexpr (CPR >= 16) return kc ^ (row & 15);  // rows of >= 256 B: one row per bank sweep
    else return kc ^ ((row / (16 / CPR)) & (CPR - 1));
}
__device__ __forceinline__ void vt_dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff,
                                         uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                 :: "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff) : "memory");
}

__device__ __forceinline__ int vt_row(int q, int lane) {
    return VT_MF16 ? 16 * (q >> 3) + 4 * ((lane >> 4) & 3) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ int vt_col(int q, int lane) {
    return VT_MF16 ? 16 * ((q >> 2) & 1) + (lane & 15) : (lane & 31);
}
#define GK 32       // K granularity of sd_gemm (the K loop runs in steps of BK = 64 or 32)

__device__ __forceinline__ float vt_gelu(float x) {
    // nn.GELU() default (approximate='none'): 0.5 x (1 + erf(x / sqrt(2))).  erf by
    // Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 rounding of the
    // output): ~12 instructions against libm erff's ~30 in a GEMM epilogue that evaluates
    // it 64 times per lane.
    const float z = fabsf(x) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
    float poly = fmaf(1.061405429f, t, -1.453152027f);
    poly = fmaf(poly, t, 1.421413741f);
    poly = fmaf(poly, t, -0.284496736f);
    poly = fmaf(poly, t, 0.254829592f);
    poly *= t;
    const float e = 1.f - poly * __expf(-z * z);   // erf(|x| / sqrt 2)
    return 0.5f * x * (1.f + copysignf(e, x));
}

__device__ __forceinline__ uint32_t vt_bytes(int64_t elems) {
    const int64_t b = elems * 2;
    return b > 0xffffffffLL ? 0xffffffffu : (uint32_t)b;
}

// bf16 ReLU on 8 packed values (sign bit set -> +0), integer ops only
__device__ __forceinline__ bf16x8 vt_relu8(bf16x8 v) {
    uint4 u = __builtin_bit_cast(uint4, v);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] &= ~(((w[i] >> 15) & 0x00010001u) * 0xffffu);
    return __builtin_bit_cast(bf16x8, uint4{w[0], w[1], w[2], w[3]});
}

// BM = BN = 32 is the split-K form for GEMMs too small to fill the chip with 64x64 tiles
// (ViT-S/16: 481 tokens): the 4 waves share one 32x32 output tile and split every BK step
// between them (wave w runs the 16-deep MFMA sub-steps w, w + 4, ...), then their
// accumulators are summed through LDS in a fixed order (deterministic) and wave 0 runs the
// epilogue.  Four times the workgroups of the 64x64 tiling, a quarter of the MFMA chain per
// wave.
// LayerNorm of the residual stream in the tail of the residual GEMM (sd_gemm_resid_ln): the
// residual update's f32 rows go out as write-through (sc1) stores, every workgroup of a
// BM-row band takes a ticket, and the band's last arriver reads the band's rows back (sc1
// loads) and writes LN(x) as the next GEMM's bf16 A operand -- k_layernorm's per-row
// arithmetic in its order (bit-equal), without its launch.  The ticket self-resets.
#define VT_EPI_RESID_LN 100  // internal epilogue: SD_EPI_RESID + the LayerNorm tail (its own kernel)
struct VtLnTail {
    const float *w, *b;
    float eps;
    __bf16 *out;    // (M, N) bf16, or nullptr: no tail
    uint32_t *cnt;  // one zeroed ticket per row band
};

__device__ __forceinline__ float vt_wave_sum(float x);

template <int BM>
__device__ __forceinline__ void vt_ln_tail(const sd_gemm_args &g, const VtLnTail &lt, int64_t m0,
                                           uint8_t *smem, int tid) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's write-through stores
    __syncthreads();
    uint32_t *flag = (uint32_t *)smem;
    if (tid == 0)
        *flag = __hip_atomic_fetch_add(lt.cnt + m0 / BM, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                gridDim.x - 1;
    __syncthreads();
    if (!*flag) return;  // workgroup-uniform
    if (tid == 0) __hip_atomic_store(lt.cnt + m0 / BM, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int lane = tid & 63, wave = tid >> 6;
    const int C = (int)g.N;
    const int nch = C <= 512 ? 2 : C <= 768 ? 3 : 4;  // sd_layernorm's PER
    const float inv_c = 1.f / (float)C;
    const int64_t mend = min(m0 + BM, g.M);
    constexpr int RB = BM / 4 < 8 ? BM / 4 : 8;  // rows per wave whose loads go out together
    for (int64_t r0 = m0 + wave; r0 < mend; r0 += 4 * RB) {
        vf4 v[RB][4];
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int64_t row = r0 + 4 * k;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 4 * lane + 256 * i;
                v[k][i] = vf4{0.f, 0.f, 0.f, 0.f};
                if (i < nch && row < mend && c < C) {
                    const float *p = (const float *)g.out + row * g.ldo + c;
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        v[k][i][u] = __hip_atomic_load(p + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int64_t row = r0 + 4 * k;
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (i < nch) s += (v[k][i][0] + v[k][i][1]) + (v[k][i][2] + v[k][i][3]);
            const float mean = vt_wave_sum(s) * inv_c;
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 4 * lane + 256 * i;
                if (i < nch && c < C) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float d = v[k][i][u] - mean;
                        q = fmaf(d, d, q);
                    }
                }
            }
            const float rstd = __builtin_amdgcn_rsqf(vt_wave_sum(q) * inv_c + lt.eps);
            if (row >= mend) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 4 * lane + 256 * i;
                if (i < nch && c < C) {
                    const vf4 wv = *(const vf4 *)(lt.w + c), bv = *(const vf4 *)(lt.b + c);
                    bf16x4 o;
#pragma unroll
                    for (int u = 0; u < 4; ++u) o[u] = (__bf16)((v[k][i][u] - mean) * rstd * wv[u] + bv[u]);
                    *(bf16x4 *)(lt.out + row * C + c) = o;
                }
            }
        }
    }
}

// GEMM output rows (the staged epilogue's 16-B stores) write-through (sc1, VT_WT): the next
// launch then does not first write back this one's dirty L2 lines (MI355X_MICROARCH.md:
// boundary + dirty bytes / 6 TB/s; the DPT convolutions gained the same way, sdhip_conv.hip)
#ifndef VT_WT
#define VT_WT 1
#endif
template <typename T, typename V>
__device__ __forceinline__ void vt_store16(T *p, const V &v) {
    static_assert(sizeof(V) == 16, "16-B store");
    if (VT_WT) {
        typedef unsigned u4v __attribute__((ext_vector_type(4)));
        const u4v w = __builtin_bit_cast(u4v, v);
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(w) : "memory");
    } else {
        *(V *)p = v;
    }
}

#ifndef VT_XCD_MAP
#define VT_XCD_MAP 0  // measured no faster on the encoder (profiles/r6_vit/gemm_tile_order_splitk_ab.txt)
#endif
#ifndef VT_XCD_GM
#define VT_XCD_GM 4
#endif
template <int BM, int BN, int BK, int EPI, bool CONV>
__global__ void __launch_bounds__(256) k_gemm(sd_gemm_args g, float *__restrict__ sk_slab, uint32_t *__restrict__ sk_cnt,
                                              VtLnTail lt) {
    constexpr bool SK = BM == 32;
    static_assert(!SK || (BN == 32 && BK % 64 == 0), "split-K tile: 32x32, BK multiple of 64");
    constexpr int WM = SK ? 32 : BM / 2, WN = SK ? 32 : BN / 2;  // per-wave tile (2 x 2 waves)
    constexpr int TM = WM / 32, TN = WN / 32; // 32x32 MFMA tiles per wave
    constexpr int CPR = BK / 8;               // 16-B chunks per tile row
    constexpr int CA = BM * CPR / 256;        // 16-B chunks of the A tile per thread
    constexpr int CB = BN * CPR / 256;
    // LDS rows padded by 16 B: row stride (BK + 8) * 2 B puts the 16 rows a ds_read_b128
    // lane group touches on 16 distinct 4-bank groups
    constexpr int GLDS = BK + 8;
    // Output-staged epilogues: the fp32 tile goes through LDS (reusing the operand
    // buffers) so that global stores are 16-B vectors along the output's contiguous axis
    // (pixels for NCHW, channels otherwise) instead of 2-B lane scatters.
    constexpr bool STAGED = EPI == SD_EPI_BF16 || EPI == SD_EPI_GELU || EPI == SD_EPI_SHUF ||
                            EPI == SD_EPI_F32 || EPI == SD_EPI_NCHW || EPI == SD_EPI_QKV;
    constexpr int OST = EPI == SD_EPI_NCHW ? BN + 1 : BN + 8;  // fp32 words per staged row
    constexpr int KL_BYTES = 2 * (BM + BN) * GLDS * 2;
    constexpr int EP_BYTES = STAGED ? BM * OST * 4 : 0;
    constexpr bool RING = vt_ring_tile(BM);
    // the ring kernels take their LDS dynamically (vt_launch_gemm sizes it), the others a
    // static operand double buffer
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dyn[];
    __shared__ __attribute__((aligned(16))) uint8_t smem_st[RING ? 16 : (KL_BYTES > EP_BYTES ? KL_BYTES : EP_BYTES)];
    uint8_t *const smem = RING ? smem_dyn : smem_st;
#define SA(buf) ((__bf16 *)smem + (buf) * (BM * GLDS))
#define SB(buf) ((__bf16 *)smem + 2 * BM * GLDS + (buf) * (BN * GLDS))

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = SK ? 0 : wave >> 1, wn = SK ? 0 : wave & 1;
    const int r = lane & 31, h = lane >> 5;
    // XCD-aware tile order (VT_XCD_MAP): workgroups are dealt to the 8 XCDs round-robin by
    // linear id, so the tiles of XCD x are taken as the x-th contiguous eighth of a grouped
    // order (VT_XCD_GM row tiles per group, column-major inside it): each XCD works on a
    // compact block of row x column tiles and re-reads its A rows / B columns from its own L2
    // instead of every XCD fetching nearly all of A and B.  Tiles only move between
    // workgroups: the arithmetic is unchanged.
    int bx = (int)blockIdx.x, by = (int)blockIdx.y;
    if (VT_XCD_MAP) {
        const int nx = (int)gridDim.x, ny = (int)gridDim.y, T = nx * ny;
        if ((T & 7) == 0 && T >= 16 && ny > 1 && nx > 1) {
            const int lin = by * nx + bx;
            const int t = (lin & 7) * (T >> 3) + (lin >> 3);
            const int gsz = VT_XCD_GM * nx, grp = t / gsz, loc = t - grp * gsz;
            const int rows = min(VT_XCD_GM, ny - grp * VT_XCD_GM);
            by = grp * VT_XCD_GM + loc % rows;
            bx = loc / rows;
        }
    }
    const int64_t m0 = (int64_t)by * BM, n0 = (int64_t)bx * BN;
    const __bf16 *A = (const __bf16 *)g.a;
    const __bf16 *Wt = (const __bf16 *)g.w;
    // cross-workgroup split-K (32 x 32 ring tiles, gridDim.z > 1): this workgroup's K steps
    // [kbeg, kbeg + nk) of the K / BK
    const int nk_all = (int)(g.K / BK), nzs = (int)gridDim.z, zs = (int)blockIdx.z;
    const int kbeg = (int)((int64_t)nk_all * zs / nzs);
    const int nk = (int)((int64_t)nk_all * (zs + 1) / nzs) - kbeg;

    // NS register staging sets (a ring): step k's compute runs while the tiles of steps
    // k + 1 .. k + NS - 1 are in flight; step k + 1's tile goes to LDS after step k's
    // MFMAs and its set is re-filled with step k + 1 + NS -- global latency gets NS - 1
    // steps of MFMA work to hide under, at one LDS double buffer.  The small tiles (32 x 32
    // split-K, 64 x 64) have little MFMA work per step and the VGPRs for a deep ring.
    constexpr int NS = BM >= 128 ? VT_NS_BIG : VT_NS_SMALL;
    bf16x8 ra[NS][CA], rb[NS][CB];
    // Rows past M (N) are clamped to the last row instead of predicated: they only feed
    // output rows (columns) that are never stored, and unpredicated loads keep the
    // compiler's vmcnt accounting exact (a masked load forces vmcnt(0) waits).
    // Buffer loads: the per-thread byte offset (voffset) is fixed for the whole K loop and
    // the K step is the scalar offset, so no address VGPR is rewritten per step (a rewrite
    // of a load's own destination/address registers costs a vmcnt drain).
    // conv: A = NHWC input of B = M / (OH OW) images; an out-of-image tap gets an offset
    // past the buffer's end, which the buffer load returns as zeros (the padding)
    const int64_t a_elems = CONV ? (g.M / ((int64_t)g.OH * g.OW)) * g.H * g.W * g.Cin
                                 : g.M * g.lda;
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16 *>(A), 0, vt_bytes(a_elems), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16 *>(Wt), 0, vt_bytes(g.N * g.K), 0x00020000);
    uint32_t voA[CA], voB[CB];
    int cpix[CA], ciy[CA], cix[CA];  // conv: image base pixel, top-left tap row / column
#pragma unroll
    for (int c = 0; c < CA; ++c) {
        const int ch = tid + 256 * c, row = ch / CPR, col = (ch % CPR) * 8;
        const int64_t m = min(m0 + row, g.M - 1);
        if (CONV) {
            const int ohw = g.OH * g.OW;
            const int b = (int)((uint32_t)m / (uint32_t)ohw);
            const int p = (int)(m - (int64_t)b * ohw);
            const int oy = p / g.OW, ox = p - oy * g.OW;
            cpix[c] = b * g.H * g.W;
            ciy[c] = oy * g.stride - 1;
            cix[c] = ox * g.stride - 1;
            voA[c] = (uint32_t)col;
        } else {
            voA[c] = (uint32_t)((m * g.lda + col) * 2);
        }
    }
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int ch = tid + 256 * c, row = ch / CPR, col = (ch % CPR) * 8;
        voB[c] = (uint32_t)((min(n0 + row, g.N - 1) * g.K + col) * 2);
    }
    auto gload = [&](int kt, bf16x8 (&ra)[CA], bf16x8 (&rb)[CB]) {
        const uint32_t so = (uint32_t)kt * BK * 2;
        if (CONV) {
            const int k0 = kt * BK;
            const int tap = k0 / g.Cin, ci0 = k0 - tap * g.Cin;
            const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
            for (int c = 0; c < CA; ++c) {
                const int iy = ciy[c] + ky, ix = cix[c] + kx;
                const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
                const uint32_t off =
                    ok ? (uint32_t)(((cpix[c] + iy * g.W + ix) * g.Cin + ci0) * 2) + voA[c] * 2
                       : 0x80000000u;
                ra[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsA, off, 0, 0));
            }
        } else {
#pragma unroll
            for (int c = 0; c < CA; ++c)
                ra[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsA, voA[c], so, 0));
        }
#pragma unroll
        for (int c = 0; c < CB; ++c)
            rb[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsB, voB[c], so, 0));
    };
    auto lstore = [&](int buf, bf16x8 (&ra)[CA], bf16x8 (&rb)[CB]) {
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            const int ch = tid + 256 * c, row = ch / CPR, col = (ch % CPR) * 8;
            *(bf16x8 *)&SA(buf)[row * GLDS + col] = (CONV && g.relu_in) ? vt_relu8(ra[c]) : ra[c];
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            const int ch = tid + 256 * c, row = ch / CPR, col = (ch % CPR) * 8;
            *(bf16x8 *)&SB(buf)[row * GLDS + col] = rb[c];
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = vt_zero16();

    auto compute = [&](int kt) {
        const int buf = kt & 1;
        if (VT_MF16) {
            // 32-deep k-steps: lane (row l & 15, group l >> 4) holds k = 8 (l >> 4) .. + 7
            const int rr = lane & 15, kg = lane >> 4;
#pragma unroll
            for (int s0 = 0; s0 < (SK ? BK / 128 : BK / 32); ++s0) {
                const int s = SK ? 4 * s0 + wave : s0;
                bf16x8 af[TM][2], bfr[TN][2];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int a = 0; a < 2; ++a)
                        af[i][a] = *(const bf16x8 *)&SA(buf)[(wm * WM + i * 32 + 16 * a + rr) * GLDS + 32 * s + 8 * kg];
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        bfr[j][b] = *(const bf16x8 *)&SB(buf)[(wn * WN + j * 32 + 16 * b + rr) * GLDS + 32 * s + 8 * kg];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int b = 0; b < 2; ++b) {
                                const int o = 4 * (2 * a + b);
                                f32x4 c = {acc[i][j][o], acc[i][j][o + 1], acc[i][j][o + 2], acc[i][j][o + 3]};
                                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][a], bfr[j][b], c, 0, 0, 0);
                                acc[i][j][o] = c[0];
                                acc[i][j][o + 1] = c[1];
                                acc[i][j][o + 2] = c[2];
                                acc[i][j][o + 3] = c[3];
                            }
            }
            return;
        }
#pragma unroll
        for (int s0 = 0; s0 < (SK ? BK / 64 : BK / 16); ++s0) {
            const int s = SK ? 4 * s0 + wave : s0;
            bf16x8 af[TM], bfr[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                af[i] = *(const bf16x8 *)&SA(buf)[(wm * WM + i * 32 + r) * GLDS + 16 * s + 8 * h];
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bfr[j] = *(const bf16x8 *)&SB(buf)[(wn * WN + j * 32 + r) * GLDS + 16 * s + 8 * h];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = VT_MFMA(af[i], bfr[j], acc[i][j]);
        }
    };

    if constexpr (RING) {
        // ---- LDS-DMA ring: stage kt of the K loop in slot kt % RS ----------------------
        constexpr int RS = vt_ring_stages(BM, BN);
        constexpr int STB = (BM + BN) * BK * 2;  // bytes per stage: A tile, then W tile
        const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)smem;
        // this thread's chunks: DMA instruction i of the wave (64 consecutive 16-B slots);
        // slot -> (row, swizzled chunk) -> source chunk
        uint32_t dA[CA], dB[CB];
#pragma unroll
        for (int c = 0; c < CA; ++c) {
            const int slot = (c * 4 + wave) * 64 + lane, row = slot / CPR;
            const int kc = vt_swz<CPR>(row, slot % CPR);  // the source chunk this slot holds
            if (CONV) voA[c] = (uint32_t)(kc * 8);
            else voA[c] = (uint32_t)(((int64_t)min(m0 + row, g.M - 1) * g.lda + kc * 8) * 2);
            if (CONV) {
                const int64_t m = min(m0 + row, g.M - 1);
                const int ohw = g.OH * g.OW;
                const int b = (int)((uint32_t)m / (uint32_t)ohw);
                const int p = (int)(m - (int64_t)b * ohw);
                const int oy = p / g.OW, ox = p - oy * g.OW;
                cpix[c] = b * g.H * g.W;
                ciy[c] = oy * g.stride - 1;
                cix[c] = ox * g.stride - 1;
            }
            dA[c] = (uint32_t)(c * 4 + wave) * 1024u;
        }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            const int slot = (c * 4 + wave) * 64 + lane, row = slot / CPR;
            const int kc = vt_swz<CPR>(row, slot % CPR);
            voB[c] = (uint32_t)((min(n0 + row, g.N - 1) * g.K + kc * 8) * 2);
            dB[c] = (uint32_t)(BM * BK * 2) + (uint32_t)(c * 4 + wave) * 1024u;
        }
        // issue stage kt (steps past the last re-load step nk - 1 into their free slot, so
        // that every step issues CA + CB DMAs and the vmcnt count below is exact)
        auto issue = [&](int kt) {
            const int k = kbeg + min(kt, nk - 1);
            const uint32_t st = lds0 + (uint32_t)(kt % RS) * STB;
            if (CONV) {
                const int k0 = k * BK;
                const int tap = k0 / g.Cin, ci0 = k0 - tap * g.Cin;
                const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
                for (int c = 0; c < CA; ++c) {
                    const int iy = ciy[c] + ky, ix = cix[c] + kx;
                    const bool ok = (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
                    const uint32_t off =
                        ok ? (uint32_t)(((cpix[c] + iy * g.W + ix) * g.Cin + ci0) * 2) + voA[c] * 2
                           : 0x80000000u;  // past the buffer: the DMA writes zeros (padding)
                    vt_dma16(rsA, off, 0u, __builtin_amdgcn_readfirstlane(st + dA[c]));
                }
            } else {
#pragma unroll
                for (int c = 0; c < CA; ++c)
                    vt_dma16(rsA, voA[c], (uint32_t)k * BK * 2, __builtin_amdgcn_readfirstlane(st + dA[c]));
            }
#pragma unroll
            for (int c = 0; c < CB; ++c)
                vt_dma16(rsB, voB[c], (uint32_t)k * BK * 2, __builtin_amdgcn_readfirstlane(st + dB[c]));
        };
#pragma unroll
        for (int i = 0; i < RS - 1; ++i) issue(i);
        for (int kt = 0; kt < nk; ++kt) {
            // stage kt landed: this thread's DMAs of stages kt + 1 .. kt + RS - 2 are younger
            static_assert((RS - 2) * (CA + CB) <= 63, "vmcnt range");
            asm volatile("s_waitcnt vmcnt(%0)" :: "i"((RS - 2) * (CA + CB)) : "memory");
            __syncthreads();  // every thread's chunks of stage kt landed; slot (kt - 1) % RS free
            issue(kt + RS - 1);
            const __bf16 *sa = (const __bf16 *)(smem + (kt % RS) * STB);
            const __bf16 *sb = sa + BM * BK;
#pragma unroll
            for (int s0 = 0; s0 < (SK ? BK / 64 : BK / 16); ++s0) {
                const int s = SK ? 4 * s0 + wave : s0;
                const int kc = 2 * s + h;  // 16-B chunk of the lane's k-range
                bf16x8 af[TM], bfr[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm * WM + i * 32 + r;
                    af[i] = *(const bf16x8 *)&sa[row * BK + 8 * vt_swz<CPR>(row, kc)];
                    if (CONV && g.relu_in) af[i] = vt_relu8(af[i]);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int row = wn * WN + j * 32 + r;
                    bfr[j] = *(const bf16x8 *)&sb[row * BK + 8 * vt_swz<CPR>(row, kc)];
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = VT_MFMA(af[i], bfr[j], acc[i][j]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy stages' DMAs
        __syncthreads();  // every wave is done with the ring: the epilogue reuses the LDS
    } else {
    // prologue: set i <- step i (i < NS), step 0 to LDS, set 0 <- step NS.  Loads past the
    // last step re-load step nk - 1 (unconditional: a load issued on one path only makes the
    // compiler's vmcnt model wait for the newest loads as well)
#pragma unroll
    for (int i = 0; i < NS; ++i) gload(min(i, nk - 1), ra[i], rb[i]);
    lstore(0, ra[0], rb[0]);
    gload(min(NS, nk - 1), ra[0], rb[0]);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += NS) {
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const int k = kt + i;
            if (k < nk) {  // workgroup-uniform
                compute(k);
                const int nx = (i + 1) % NS;  // the set holding step k + 1 (constant once unrolled)
                if (k + 1 < nk) lstore((k + 1) & 1, ra[nx], rb[nx]);
                gload(min(k + 1 + NS, nk - 1), ra[nx], rb[nx]);
                __syncthreads();
            }
        }
    }
    }

    if constexpr (SK) {
        // split-K reduction: waves 1..3 park their partial tiles past the staging area,
        // wave 0 adds them in wave order (the K loop ended on a barrier)
        float *part = (float *)(smem + 16384);
        if (wave > 0) {
#pragma unroll
            for (int q = 0; q < 16; ++q) part[((wave - 1) * 16 + q) * 64 + lane] = acc[0][0][q];
        }
        __syncthreads();
        if (wave == 0) {
#pragma unroll
            for (int w = 0; w < 3; ++w)
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[0][0][q] += part[(w * 16 + q) * 64 + lane];
        }
        if (RING && nzs > 1) {
            // cross-workgroup combine, deterministic: every K slice writes its 32 x 32 partial
            // (write-through sc1 stores: no release fence), takes a ticket; the last arriver
            // sums the slices in slice order (sc1 loads), resets the ticket for the next
            // launch and runs the epilogue (MI355X guide §5, split-K reduction recipe)
            const int tile = blockIdx.y * gridDim.x + blockIdx.x;
            float *slab = sk_slab + (int64_t)tile * nzs * 1024;
            if (wave == 0) {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    __hip_atomic_store(slab + zs * 1024 + q * 64 + lane, acc[0][0][q], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
            uint32_t *flag = (uint32_t *)smem;
            if (tid == 0)
                *flag = __hip_atomic_fetch_add(sk_cnt + tile, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                        (uint32_t)(nzs - 1);
            __syncthreads();
            if (!*flag) return;  // workgroup-uniform
            if (wave == 0) {
                // one slice per round trip: its 16 loads issued together, summed in slice order
#pragma unroll
                for (int q = 0; q < 16; ++q) acc[0][0][q] = 0.f;
                for (int z = 0; z < nzs; ++z) {
                    float v[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                        v[q] = __hip_atomic_load(slab + z * 1024 + q * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                    for (int q = 0; q < 16; ++q) acc[0][0][q] += v[q];
                }
            }
            if (tid == 0) __hip_atomic_store(sk_cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();  // the flag word is part of the epilogue's LDS
        }
        if constexpr (!STAGED) {
            if (wave != 0 && EPI != VT_EPI_RESID_LN) return;  // (the LN tail needs all waves)
        }
    }
    // epilogue: accumulator register q of tile (i, j): row (q&3)+8(q>>2)+4h, column r
    if constexpr (STAGED) {
        // phase 1: v = acc + bias (GELU) -> fp32 tile [m][n] in LDS (the K loop ended on a
        // barrier, every wave is done with the operand tiles)
        float *sT = (float *)smem;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (SK && wave != 0) break;
            float bias2[2];  // the lane's (at most two) columns of block column j
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int nl = wn * WN + j * 32 + vt_col(4 * b, lane);
                bias2[b] = (g.bias && n0 + nl < g.N) ? g.bias[n0 + nl] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int ml = wm * WM + i * 32 + vt_row(q, lane);
                    const int nl = wn * WN + j * 32 + vt_col(q, lane);
                    float v = acc[i][j][q] + bias2[VT_MF16 ? (q >> 2) & 1 : 0];
                    if (EPI == SD_EPI_GELU) v = vt_gelu(v);
                    sT[ml * OST + nl] = v;
                }
        }
        __syncthreads();
        if constexpr (EPI == SD_EPI_QKV) {
            // phase 2.  q / k columns: thread = 8 consecutive head-dim columns of one token
            // -> one 16-B store along head_dim (head_dim % 8 == 0: a chunk never straddles
            // the q / k / v thirds).  V^T columns: thread = 8 consecutive tokens of one
            // head-dim row -> one 16-B store along the token axis (consecutive threads take
            // consecutive token runs of the same row: 128-B segments).
            const int C = g.heads * g.head_dim;
            if (n0 < 2 * (int64_t)C) {
#pragma unroll 4
                for (int t = tid; t < BM * (BN / 8); t += 256) {
                    const int ml = t / (BN / 8), nl = (t - ml * (BN / 8)) * 8;
                    const int64_t m = m0 + ml, n = n0 + nl;
                    if (m >= g.M || n >= g.N) continue;
                    const int which = (int)(n / C);
                    if (which == 2) continue;
                    __bf16 *dst0 = (__bf16 *)(which == 0 ? g.q : g.k);
                    const int64_t tstride = which == 0 ? g.tokens : g.tokens_pad;
                    const int rem = (int)(n - (int64_t)which * C);
                    const int head = rem / g.head_dim, e = rem - head * g.head_dim;
                    const uint32_t b = (uint32_t)m / (uint32_t)g.tokens;
                    const int64_t tok = m - (int64_t)b * g.tokens;
                    const vf4 lo = *(const vf4 *)&sT[ml * OST + nl];
                    const vf4 hi = *(const vf4 *)&sT[ml * OST + nl + 4];
                    bf16x8 o;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        o[u] = (__bf16)lo[u];
                        o[4 + u] = (__bf16)hi[u];
                    }
                    *(bf16x8 *)(dst0 + (((int64_t)b * g.heads + head) * tstride + tok) * g.head_dim + e) = o;
                }
            }
            if (n0 + BN > 2 * (int64_t)C) {
#pragma unroll 4
                for (int t = tid; t < BN * (BM / 8); t += 256) {
                    const int nl = t / (BM / 8), ml = (t - nl * (BM / 8)) * 8;
                    const int64_t m = m0 + ml, n = n0 + nl;
                    if (m >= g.M || n >= g.N || n < 2 * (int64_t)C) continue;
                    const int rem = (int)(n - 2 * (int64_t)C);
                    const int head = rem / g.head_dim, e = rem - head * g.head_dim;
                    const uint32_t b = (uint32_t)m / (uint32_t)g.tokens;
                    const int64_t tok = m - (int64_t)b * g.tokens;
                    __bf16 *row = (__bf16 *)g.vt + (((int64_t)b * g.heads + head) * g.head_dim + e) * g.tokens_pad;
                    if ((tok & 7) == 0 && tok + 8 <= g.tokens && m + 8 <= g.M) {
                        bf16x8 o;
#pragma unroll
                        for (int u = 0; u < 8; ++u) o[u] = (__bf16)sT[(ml + u) * OST + nl];
                        *(bf16x8 *)(row + tok) = o;
                    } else {
                        for (int u = 0; u < 8 && m + u < g.M; ++u) {
                            const uint32_t bu = (uint32_t)(m + u) / (uint32_t)g.tokens;
                            const int64_t tu = m + u - (int64_t)bu * g.tokens;
                            ((__bf16 *)g.vt)[(((int64_t)bu * g.heads + head) * g.head_dim + e) * g.tokens_pad + tu] =
                                (__bf16)sT[(ml + u) * OST + nl];
                        }
                    }
                }
            }
        } else if constexpr (EPI == SD_EPI_NCHW) {
            // phase 2: thread = 4 consecutive pixels of one channel -> one 16-B store
            const int plane = g.tokens;
            const bool vec = (plane & 3) == 0;
#pragma unroll 4
            for (int t = tid; t < BN * (BM / 4); t += 256) {
                const int nl = t / (BM / 4), ml = (t - nl * (BM / 4)) * 4;
                const int64_t n = n0 + nl, m = m0 + ml;
                if (n >= g.N || m >= g.M) continue;
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = sT[(ml + u) * OST + nl];
                const uint32_t b = (uint32_t)m / (uint32_t)plane;
                const int64_t pix = m - (int64_t)b * plane;
                float *dst = (float *)g.out + ((int64_t)b * g.N + n) * plane + pix;
                if (vec && m + 3 < g.M) {
                    *(vf4 *)dst = vf4{v[0], v[1], v[2], v[3]};
                } else {
                    for (int u = 0; u < 4 && m + u < g.M; ++u) {
                        const uint32_t bu = (uint32_t)(m + u) / (uint32_t)plane;
                        const int64_t pu = m + u - (int64_t)bu * plane;
                        ((float *)g.out)[((int64_t)bu * g.N + n) * plane + pu] = v[u];
                    }
                }
            }
        } else {
            // phase 2: thread = 8 consecutive columns of one row -> one 16-B bf16 store
            // (f32 output: two)
            const int cout = EPI == SD_EPI_SHUF ? (int)(g.N / (g.shuf_k * g.shuf_k)) : 0;
            const bool vec = EPI == SD_EPI_SHUF ? (cout & 7) == 0 : (g.ldo & 7) == 0;
#pragma unroll 4
            for (int t = tid; t < BM * (BN / 8); t += 256) {
                const int ml = t / (BN / 8), nl = (t - ml * (BN / 8)) * 8;
                const int64_t m = m0 + ml, n = n0 + nl;
                if (m >= g.M || n >= g.N) continue;
                const vf4 lo = *(const vf4 *)&sT[ml * OST + nl];
                const vf4 hi = *(const vf4 *)&sT[ml * OST + nl + 4];
                float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                const bool full = vec && n + 8 <= g.N;
                if (EPI == SD_EPI_BF16 && full) {
                    if (g.res) {
                        const bf16x8 a = *(const bf16x8 *)((const __bf16 *)g.res + m * g.ldo + n);
#pragma unroll
                        for (int u = 0; u < 8; ++u) v[u] += (float)a[u];
                    }
                    if (g.res2) {
                        const bf16x8 a = *(const bf16x8 *)((const __bf16 *)g.res2 + m * g.ldo + n);
#pragma unroll
                        for (int u = 0; u < 8; ++u) v[u] += (float)a[u];
                    }
                } else if (EPI == SD_EPI_BF16 && (g.res || g.res2)) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        if (n + u >= g.N) break;
                        if (g.res) v[u] += (float)((const __bf16 *)g.res)[m * g.ldo + n + u];
                        if (g.res2) v[u] += (float)((const __bf16 *)g.res2)[m * g.ldo + n + u];
                    }
                }
                int64_t base;  // element index of column n of row m
                if (EPI == SD_EPI_SHUF) {
                    const int kk = g.shuf_k, hw = g.in_h * g.in_w;
                    const int b = (int)((uint32_t)m / (uint32_t)hw);
                    const int pix = (int)(m - (int64_t)b * hw);
                    const int y = pix / g.in_w, x = pix - y * g.in_w;
                    if (full) {
                        const int sub = (int)(n / cout), co = (int)(n - (int64_t)sub * cout);
                        const int dy = sub / kk, dx = sub - dy * kk;
                        base = (((int64_t)b * g.in_h * kk + y * kk + dy) * (g.in_w * kk) + x * kk + dx) *
                                   cout + co;
                    } else {
                        for (int u = 0; u < 8 && n + u < g.N; ++u) {
                            const int sub = (int)((n + u) / cout), co = (int)(n + u - (int64_t)sub * cout);
                            const int dy = sub / kk, dx = sub - dy * kk;
                            ((__bf16 *)g.out)[(((int64_t)b * g.in_h * kk + y * kk + dy) * (g.in_w * kk) +
                                               x * kk + dx) * cout + co] = (__bf16)v[u];
                        }
                        continue;
                    }
                } else {
                    base = m * g.ldo + n;
                }
                if (EPI == SD_EPI_F32) {  // f32 rows (the channels-last DPT grid): 2 x 16 B
                    float *o = (float *)g.out + base;
                    if (full) {
                        vt_store16(o, vf4{v[0], v[1], v[2], v[3]});
                        vt_store16(o + 4, vf4{v[4], v[5], v[6], v[7]});
                    } else {
                        for (int u = 0; u < 8 && n + u < g.N; ++u) o[u] = v[u];
                    }
                    continue;
                }
                if (full) {
                    bf16x8 o;
#pragma unroll
                    for (int u = 0; u < 8; ++u) o[u] = (__bf16)v[u];
                    vt_store16((__bf16 *)g.out + base, o);
                } else {
                    for (int u = 0; u < 8 && n + u < g.N; ++u) ((__bf16 *)g.out)[base + u] = (__bf16)v[u];
                }
            }
        }
        return;
    }
    // unstaged epilogues (residual update, patch embedding): lane-scattered 4-B stores.
    // The residual update issues every load (bias, layer scale, the residual rows) before
    // its first store: interleaved, each store-then-load pair drained the vector memory
    // counter (it counts stores too), one memory round trip per accumulator register
    static_assert(!VT_MF16, "the unstaged epilogues take one output column per lane and tile");
    // SD_EPI_RESID, outputs < 2 GiB: buffer loads / stores whose offsets (out-of-range
    // rows and columns -> past the buffer: loads read 0, stores are dropped) and data sit
    // in registers of their own, computed before the first store, so the 16 stores of a
    // tile issue back to back (a store whose address or data register is rewritten while
    // the store is pending, or one under its own exec branch, costs a vmcnt(0) drain)
    bool resid_done = false;
    if constexpr (EPI == SD_EPI_RESID) {
        if (g.M * g.ldo < ((int64_t)1 << 29) && (!g.q || g.M * g.N < ((int64_t)1 << 30))) {
            resid_done = true;
            if (!(SK && wave != 0)) {
                const __amdgpu_buffer_rsrc_t rsO =
                    __builtin_amdgcn_make_buffer_rsrc(g.out, 0, (uint32_t)(g.M * g.ldo * 4), 0x00020000);
                const uint32_t T = g.tokens > 1 ? (uint32_t)g.tokens : 1u;
                const __amdgpu_buffer_rsrc_t rsQ = __builtin_amdgcn_make_buffer_rsrc(
                    g.q ? g.q : g.out, 0, g.q ? (uint32_t)((g.M / T) * (T - 1) * g.N * 2) : 0u, 0x00020000);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int64_t n = n0 + wn * WN + j * 32 + vt_col(0, lane);
                    const bool nok = n < g.N;
                    const float bias = (g.bias && nok) ? g.bias[n] : 0.f;
                    const float gam = (g.gamma && nok) ? g.gamma[n] : 1.f;
#pragma unroll
                    for (int i = 0; i < TM; ++i) {
                        uint32_t va[16];
                        float nv[16];
#pragma unroll
                        for (int q = 0; q < 16; ++q) {
                            const int64_t m = m0 + wm * WM + i * 32 + vt_row(q, lane);
                            va[q] = (nok && m < g.M) ? (uint32_t)((m * g.ldo + n) * 4) : 0x80000000u;
                            nv[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsO, va[q], 0, 0));
                        }
#pragma unroll
                        for (int q = 0; q < 16; ++q) nv[q] = nv[q] + gam * (acc[i][j][q] + bias);
#pragma unroll
                        for (int q = 0; q < 16; ++q)
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, nv[q]), rsO, va[q], 0, 0);
                        if (g.k) {  // an f32 copy of the updated rows (sd_vit_mlp's LayerNorm input)
                            const __amdgpu_buffer_rsrc_t rsK =
                                __builtin_amdgcn_make_buffer_rsrc(g.k, 0, (uint32_t)(g.M * g.ldo * 4), 0x00020000);
#pragma unroll
                            for (int q = 0; q < 16; ++q)
                                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, nv[q]), rsK, va[q], 0, 0);
                        }
                        if (g.q) {  // the intermediate-layer grid (k_tokens_to_nhwc's rounding)
                            uint32_t qa[16];
                            uint16_t qv[16];
#pragma unroll
                            for (int q = 0; q < 16; ++q) {
                                const int64_t m = m0 + wm * WM + i * 32 + vt_row(q, lane);
                                const uint32_t b = (uint32_t)m / T, tok = (uint32_t)m - b * T;
                                qa[q] = (nok && m < g.M && tok > 0)
                                            ? (uint32_t)((((int64_t)b * (T - 1) + tok - 1) * g.N + n) * 2)
                                            : 0x80000000u;
                                qv[q] = __builtin_bit_cast(uint16_t, (__bf16)nv[q]);
                            }
#pragma unroll
                            for (int q = 0; q < 16; ++q) __builtin_amdgcn_raw_buffer_store_b16(qv[q], rsQ, qa[q], 0, 0);
                        }
                    }
                }
            }
        }
    }
    if constexpr (EPI == SD_EPI_RESID || EPI == VT_EPI_RESID_LN) {
        if (!(SK && wave != 0) && !resid_done) {
            float bj[TN], gj[TN], ov[TM][TN][16];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int64_t n = n0 + wn * WN + j * 32 + vt_col(0, lane);
                bj[j] = (g.bias && n < g.N) ? g.bias[n] : 0.f;
                gj[j] = (g.gamma && n < g.N) ? g.gamma[n] : 1.f;
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int64_t m = m0 + wm * WM + i * 32 + vt_row(q, lane);
                        ov[i][j][q] = (m < g.M && n < g.N) ? ((const float *)g.out)[m * g.ldo + n] : 0.f;
                    }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int64_t n = n0 + wn * WN + j * 32 + vt_col(q, lane);
                        const int64_t m = m0 + wm * WM + i * 32 + vt_row(q, lane);
                        if (m >= g.M || n >= g.N) continue;
                        const float v = acc[i][j][q] + bj[j];
                        const float nv = ov[i][j][q] + gj[j] * v;
                        float *o = (float *)g.out + m * g.ldo + n;
                        if (EPI == VT_EPI_RESID_LN) __hip_atomic_store(o, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        else *o = nv;
                        if (EPI == SD_EPI_RESID && g.k) ((float *)g.k)[m * g.ldo + n] = nv;
                        if (g.q) {  // the intermediate-layer grid (k_tokens_to_nhwc's rounding)
                            const uint32_t T = (uint32_t)g.tokens, b = (uint32_t)m / T, tok = (uint32_t)m - b * T;
                            if (tok > 0) ((__bf16 *)g.q)[((int64_t)b * (T - 1) + tok - 1) * g.N + n] = (__bf16)nv;
                        }
                    }
        }
    }
    if constexpr (EPI == SD_EPI_PATCH) {  // patch row m = b * patches + p -> token 1 + p
        if (!(SK && wave != 0)) {
            float bj[TN], pv[TM][TN][16];  // (loads first, as above)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int64_t n = n0 + wn * WN + j * 32 + vt_col(0, lane);
                bj[j] = (g.bias && n < g.N) ? g.bias[n] : 0.f;
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int64_t m = m0 + wm * WM + i * 32 + vt_row(q, lane);
                        const int64_t tok = 1 + (m - (int64_t)((uint32_t)m / (uint32_t)g.patches) * g.patches);
                        pv[i][j][q] = (m < g.M && n < g.N) ? g.pos[tok * g.N + n] : 0.f;
                    }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int64_t n = n0 + wn * WN + j * 32 + vt_col(q, lane);
                        const int64_t m = m0 + wm * WM + i * 32 + vt_row(q, lane);
                        if (m >= g.M || n >= g.N) continue;
                        const int64_t b = (uint32_t)m / (uint32_t)g.patches, p = m - b * g.patches;
                        const int64_t T = g.patches + 1;
                        ((float *)g.out)[(b * T + 1 + p) * g.ldo + n] = (acc[i][j][q] + bj[j]) + pv[i][j][q];
                    }
        }
    }
    if constexpr (EPI == VT_EPI_RESID_LN) vt_ln_tail<BM>(g, lt, m0, smem, tid);
}

#undef SA
#undef SB

// ---------------------------------------------------------------------------
// flash attention (head_dim 64)
// ---------------------------------------------------------------------------
// A wave owns 32 queries of one (batch, head) and walks 64-key blocks with an online
// softmax: S^T = K Q^T (2 tiles of 32 keys x 4 k-steps, v_mfma_f32_32x32x16_bf16: a query's
// scores sit in its lane), P straight from the S^T accumulator into the B operand of
// O^T += V^T P (2 head-dim tiles x 2 key tiles x 2 k-steps).  The K rows of a 32-key tile
// are fed to the MFMA in the order at_perm (bits 2 and 3 of the row swapped): then the keys
// a lane holds for k-step s of the P operand are 8 consecutive keys, so every K and V^T
// fragment is one 16-B load (from LDS or straight from L2) with no register shuffles.
//   k_attn_lds : 4 waves = 128 consecutive queries share each K / V^T block, staged once
//                per workgroup through double-buffered LDS (one barrier per block).
//   k_attn_dir : 4 waves = 32 queries x 4 key quarters (fills the chip when there are few
//                query tiles, e.g. 481-token ViTs); fragments loaded straight from L2 into
//                registers a block ahead; the 4 partial softmax states merge through LDS.
// exp2 in the log2 domain (scores scaled by scale * log2 e) on the raw v_exp_f32; the O
// rescale is skipped while no query's running maximum moved.
#define AT_HD 64
#define AT_ROW 72  // bf16 per LDS tile row: 64 + 8 pad (144-B rows: conflict-free b128 reads)

__device__ __forceinline__ int at_perm(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }

struct AtState {
    f32x16 o[2];
    float m, l;
};

// key of accumulator register i (lane half h) of S^T tile t under at_perm
__device__ __forceinline__ int at_key(int t, int i, int h) {
    return 32 * t + 16 * (i >> 3) + 8 * h + 4 * ((i >> 2) & 1) + (i & 3);
}

__device__ __forceinline__ void at_block(AtState &S, const bf16x8 qb[4], const bf16x8 kf[2][4],
                                         const bf16x8 vf[2][2][2], int kb, int T, int h,
                                         float sl2e) {
    f32x16 st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        st[t] = vt_zero16();
#pragma unroll
        for (int s = 0; s < 4; ++s) st[t] = VT_MFMA(kf[t][s], qb[s], st[t]);
    }
    if (kb + 64 > T) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (kb + at_key(t, i, h) >= T) st[t][i] = -INFINITY;
    }
    float mx = st[0][0];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, st[t][i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float mnew = fmaxf(S.m, mx * sl2e);
    const float alpha = __builtin_amdgcn_exp2f(S.m - mnew);
    S.m = mnew;
    bf16x8 pb[2][2];
    float ps = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float p = __builtin_amdgcn_exp2f(fmaf(st[t][i], sl2e, -mnew));
            ps += p;
            pb[t][i >> 3][i & 7] = (__bf16)p;
        }
    S.l = fmaf(S.l, alpha, ps);
    if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
            for (int i = 0; i < 16; ++i) S.o[ht][i] *= alpha;
    }
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) S.o[ht] = VT_MFMA(vf[ht][t][s], pb[t][s], S.o[ht]);
}

// Q^T as B operand: lane (query r, half h), k-step s: Q[q][16 s + 8 h + j]
__device__ __forceinline__ void at_load_q(const __bf16 *Qh, int q, int T, int h, bf16x8 qb[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        if (q < T)
            qb[s] = *(const bf16x8 *)(Qh + (int64_t)q * AT_HD + 16 * s + 8 * h);
        else
#pragma unroll
            for (int j = 0; j < 8; ++j) qb[s][j] = (__bf16)0.f;
    }
}

// out[b, q, head * 64 + e] = O^T[e][q] / l: registers i of tile ht hold e = 32 ht + 8 (i >> 2)
// + 4 h + (i & 3) -> four 8-B stores per tile
__device__ __forceinline__ void at_store(const f32x16 o[2], float inv, __bf16 *dst, int h) {
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            bf16x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (__bf16)(o[ht][4 * g + e] * inv);
            *(bf16x4 *)(dst + 32 * ht + 8 * g + 4 * h) = v;
        }
}

// KS = key splits per workgroup.  KS = 1: 4 waves = 128 queries over all keys.  KS = 2 (small
// grids, e.g. ViT-B/8 at batch 1: 12 heads x 15 query tiles = 180 workgroups for 256 CUs):
// 2 waves = 64 queries per key half, each half staging its own K / V^T blocks, twice the
// workgroups; the halves' (m, l, O) states merge through LDS at the end.
template <int KS>
__global__ void __launch_bounds__(256) k_attn_lds(const __bf16 *__restrict__ Q,
                                                  const __bf16 *__restrict__ K,
                                                  const __bf16 *__restrict__ Vt, int T, int Tp,
                                                  int H, float sl2e, __bf16 *__restrict__ out) {
    constexpr int QW = 4 / KS;          // query waves per key split
    constexpr int ST = 64 * QW;         // staging threads per key split
    constexpr int CH = 512 / ST;        // 16-B chunks per thread per K (or V^T) block
    __shared__ __attribute__((aligned(16))) __bf16 s_kv[KS][2][2][64 * AT_ROW];  // [split][buf][K | V^T]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int ks = wave / QW, qw = wave - ks * QW, stid = tid - ks * ST;
    const int bh = blockIdx.y;
    const int q = blockIdx.x * (32 * QW) + 32 * qw + r;
    const __bf16 *Kh = K + (int64_t)bh * Tp * AT_HD;
    const __bf16 *Vh = Vt + (int64_t)bh * AT_HD * Tp;
    bf16x8 qb[4];
    at_load_q(Q + (int64_t)bh * T * AT_HD, q, T, h, qb);
    AtState S;
    S.o[0] = vt_zero16();
    S.o[1] = vt_zero16();
    S.m = -INFINITY;
    S.l = 0.f;
    // this split's 64-key blocks [b0, b1)
    const int nb = Tp >> 6;
    const int b0 = nb * ks / KS, b1 = nb * (ks + 1) / KS, nmax = (nb + KS - 1) / KS;
    // staging: chunk c = stid + ST i of a 64-row x 128-B tile, row c / 8, 16-B column c % 8
    bf16x8 gk[CH], gv[CH];
    auto gload = [&](int kb) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int c = stid + ST * i, row = c >> 3, col = (c & 7) * 8;
            gk[i] = *(const bf16x8 *)(Kh + (int64_t)(kb + row) * AT_HD + col);
            gv[i] = *(const bf16x8 *)(Vh + (int64_t)row * Tp + kb + col);
        }
    };
    auto swrite = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int c = stid + ST * i, row = c >> 3, col = (c & 7) * 8;
            *(bf16x8 *)(s_kv[ks][buf][0] + row * AT_ROW + col) = gk[i];
            *(bf16x8 *)(s_kv[ks][buf][1] + row * AT_ROW + col) = gv[i];
        }
    };
    if (b0 < b1) {
        gload(64 * b0);
        swrite(0);
    }
    __syncthreads();
    const int pr = at_perm(r);
    // both splits run nmax steps (a split with fewer blocks idles through its last one):
    // the barrier is workgroup-wide
    for (int i = 0; i < nmax; ++i) {
        const int b = b0 + i;
        const bool live = b < b1;
        if (b + 1 < b1) gload(64 * (b + 1));
        if (live) {
            const __bf16 *sK = s_kv[ks][i & 1][0], *sV = s_kv[ks][i & 1][1];
            bf16x8 kf[2][4], vf[2][2][2];
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    kf[t][s] = *(const bf16x8 *)(sK + (32 * t + pr) * AT_ROW + 16 * s + 8 * h);
#pragma unroll
            for (int ht = 0; ht < 2; ++ht)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s)
                        vf[ht][t][s] =
                            *(const bf16x8 *)(sV + (32 * ht + r) * AT_ROW + 32 * t + 16 * s + 8 * h);
            at_block(S, qb, kf, vf, 64 * b, T, h, sl2e);
        }
        if (b + 1 < b1) swrite((i + 1) & 1);
        __syncthreads();
    }
    if (KS == 2) {
        // merge: the second half's waves park (m, l, O) in the (now idle) staging area, the
        // first half's combine them (exp2 domain: m is scaled by scale * log2 e)
        float *park = (float *)&s_kv[0][0][0][0] + (size_t)qw * 34 * 64;
        if (ks == 1) {
            park[lane] = S.m;
            park[64 + lane] = S.l;
#pragma unroll
            for (int ht = 0; ht < 2; ++ht)
#pragma unroll
                for (int i = 0; i < 16; ++i) park[(2 + 16 * ht + i) * 64 + lane] = S.o[ht][i];
        }
        __syncthreads();
        if (ks == 1) return;
        const float m1 = park[lane], l1 = park[64 + lane];
        const float m = fmaxf(S.m, m1);
        const float a0 = S.m == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(S.m - m);
        const float a1 = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m1 - m);
        S.l = S.l * a0 + l1 * a1;
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
            for (int i = 0; i < 16; ++i) S.o[ht][i] = S.o[ht][i] * a0 + park[(2 + 16 * ht + i) * 64 + lane] * a1;
    }
    const float l = S.l + __shfl_xor(S.l, 32);
    if (q < T) {
        const int bb = bh / H, head = bh - bb * H;
        at_store(S.o, 1.f / l, out + ((int64_t)bb * T + q) * (int64_t)(H * AT_HD) + head * AT_HD, h);
    }
}

// AT_DIR_NW (build knob): waves per k_attn_dir workgroup = key blocks of 64 in flight per
// 32 queries (4: two blocks per wave at 481 tokens; 8: one -- measured no faster, 7.41 vs
// 7.31 us at ViT-S/16, `profiles/r6_vit/lg_nw_ab.txt`)
#ifndef AT_DIR_NW
#define AT_DIR_NW 4
#endif
constexpr int at_dir_lds(int nwa) { return nwa * (2 * 16 * 64 + 2 * 64) * 4; }
template <int NWA>
__global__ void __launch_bounds__(64 * NWA) k_attn_dir(const __bf16 *__restrict__ Q,
                                                       const __bf16 *__restrict__ K,
                                                       const __bf16 *__restrict__ Vt, int T, int Tp,
                                                       int H, float sl2e, __bf16 *__restrict__ out) {
    // dynamic LDS: [wave][hd tile][acc register][lane] partial O, then m and l per wave
    extern __shared__ __attribute__((aligned(16))) float at_dyn[];
    float (*s_o)[2][16][64] = (float (*)[2][16][64])at_dyn;
    float (*s_m)[64] = (float (*)[64])(at_dyn + NWA * 2 * 16 * 64);
    float (*s_l)[64] = s_m + NWA;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int bh = blockIdx.y;
    const int q = blockIdx.x * 32 + r;
    bf16x8 qb[4];
    at_load_q(Q + (int64_t)bh * T * AT_HD, q, T, h, qb);
    AtState S;
    S.o[0] = vt_zero16();
    S.o[1] = vt_zero16();
    S.m = -INFINITY;
    S.l = 0.f;
    // K rows (at_perm order) and V^T rows of this lane as byte offsets into the head's planes
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16 *>(K + (int64_t)bh * Tp * AT_HD), 0, (uint32_t)Tp * AT_HD * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16 *>(Vt + (int64_t)bh * AT_HD * Tp), 0, (uint32_t)Tp * AT_HD * 2, 0x00020000);
    const uint32_t ko = (uint32_t)(at_perm(r) * AT_HD + 8 * h) * 2;
    const uint32_t vo = (uint32_t)(r * Tp + 8 * h) * 2;
    const uint32_t vrow32 = (uint32_t)(32 * Tp) * 2;
    bf16x8 kf[2][4], vf[2][2][2], kn[2][4], vn[2][2][2];
    auto fload = [&](int kb, bf16x8 (&kd)[2][4], bf16x8 (&vd)[2][2][2]) {
        const uint32_t ks = (uint32_t)kb * AT_HD * 2, vs = (uint32_t)kb * 2;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 4; ++s)
                kd[t][s] = __builtin_bit_cast(
                    bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, ko + (32 * t * AT_HD + 16 * s) * 2, ks, 0));
#pragma unroll
        for (int ht = 0; ht < 2; ++ht)
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 2; ++s)
                    vd[ht][t][s] = __builtin_bit_cast(
                        bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                    rv, vo + ht * vrow32 + (32 * t + 16 * s) * 2, vs, 0));
    };
    int kb = 64 * wave;
    if (kb < Tp) fload(kb, kf, vf);
    for (; kb < Tp; kb += 64 * NWA) {
        const bool more = kb + 64 * NWA < Tp;
        if (more) fload(kb + 64 * NWA, kn, vn);  // next block in flight under this one
        at_block(S, qb, kf, vf, kb, T, h, sl2e);
        if (more) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < 4; ++s) kf[t][s] = kn[t][s];
#pragma unroll
            for (int ht = 0; ht < 2; ++ht)
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int s = 0; s < 2; ++s) vf[ht][t][s] = vn[ht][t][s];
        }
    }
    // merge the NWA waves' partial softmax states
    s_m[wave][lane] = S.m;  // identical in both halves
    s_l[wave][lane] = S.l;  // per-half partial sums
#pragma unroll
    for (int ht = 0; ht < 2; ++ht)
#pragma unroll
        for (int i = 0; i < 16; ++i) s_o[wave][ht][i][lane] = S.o[ht][i];
    __syncthreads();
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NWA; ++w) M = fmaxf(M, s_m[w][lane]);
    float fw[NWA], L = 0.f;
#pragma unroll
    for (int w = 0; w < NWA; ++w) {
        const float mw = s_m[w][lane];
        fw[w] = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M);  // a wave with no block
        L = fmaf(fw[w], s_l[w][r] + s_l[w][r + 32], L);
    }
    const float inv = 1.f / L;
    if (q < T) {
        // wave w writes accumulator registers i0 .. i0 + RW - 1 (i0 = RW w, RW = 16 / NWA)
        // of both head-dim tiles: register i holds row 32 ht + 8 (i / 4) + 4 h + i % 4, so
        // the wave's RW values are contiguous head-dim entries (one 8-B / 4-B store)
        constexpr int RW = 16 / NWA;
        const int i0 = RW * wave;
        const int b = bh / H, head = bh - b * H;
        __bf16 *dst = out + ((int64_t)b * T + q) * (int64_t)(H * AT_HD) + head * AT_HD;
#pragma unroll
        for (int ht = 0; ht < 2; ++ht) {
            typedef __attribute__((ext_vector_type(RW))) __bf16 bfv;
            bfv v;
#pragma unroll
            for (int e = 0; e < RW; ++e) {
                float acc = 0.f;
#pragma unroll
                for (int w = 0; w < NWA; ++w) acc = fmaf(fw[w], s_o[w][ht][i0 + e][lane], acc);
                v[e] = (__bf16)(acc * inv);
            }
            *(bfv *)(dst + 32 * ht + 8 * (i0 >> 2) + 4 * h + (i0 & 3)) = v;
        }
    }
}

// ---------------------------------------------------------------------------
// LayerNorm (one wave per row), patchify, tokens -> grid
// ---------------------------------------------------------------------------
// sum over the 64 lanes, result in every lane: DPP row reductions (row_ror 8, 4, 2, 1) then
// the four row sums by readlane (no LDS round trip, unlike a __shfl_xor butterfly)
__device__ __forceinline__ float vt_wave_sum(float x) {
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x128, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x124, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x122, 0xf, 0xf, true));
    x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x121, 0xf, 0xf, true));
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 0));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 16));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 32));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 48));
    return (r0 + r1) + (r2 + r3);
}

// One wave per row; lane = 4 consecutive channels per 256-channel chunk (16-B loads, 8-B
// bf16 / 16-B f32 stores); PER4 chunks of 256 channels (C <= 256 PER4, C % 4 == 0).
template <int PER4, bool F32OUT>
__global__ void __launch_bounds__(256) k_layernorm(const float *__restrict__ x, int64_t rows,
                                                   int C, const float *__restrict__ w,
                                                   const float *__restrict__ b, float eps,
                                                   void *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float *xr = x + row * C;
    vf4 v[PER4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER4; ++i) {
        const int c = 4 * lane + 256 * i;
        v[i] = c < C ? *(const vf4 *)(xr + c) : vf4{0.f, 0.f, 0.f, 0.f};
        s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    }
    const float inv_c = 1.f / (float)C;
    const float mean = vt_wave_sum(s) * inv_c;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < C) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float d = v[i][u] - mean;
                q = fmaf(d, d, q);
            }
        }
    }
    const float rstd = __builtin_amdgcn_rsqf(vt_wave_sum(q) * inv_c + eps);
#pragma unroll
    for (int i = 0; i < PER4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < C) {
            const vf4 wv = *(const vf4 *)(w + c), bv = *(const vf4 *)(b + c);
            vf4 y;
#pragma unroll
            for (int u = 0; u < 4; ++u) y[u] = (v[i][u] - mean) * rstd * wv[u] + bv[u];
            if (F32OUT) {
                *(vf4 *)((float *)out + row * C + c) = y;
            } else {
                bf16x4 o;
#pragma unroll
                for (int u = 0; u < 4; ++u) o[u] = (__bf16)y[u];
                *(bf16x4 *)((__bf16 *)out + row * C + c) = o;
            }
        }
    }
}

// The encoder's final norm straight into the DPT's last token grid: k_layernorm's f32 rows
// (same arithmetic) of the non-prefix tokens, then k_tokens_to_nhwc's optional L2
// normalisation (its lane order, through a wave-private LDS row) and bf16 NHWC store --
// one launch instead of two, bit-equal to them (test_layernorm_nhwc_equals_two_launches).
template <int PER4>
__global__ void __launch_bounds__(256) k_layernorm_nhwc(const float *__restrict__ x, int B, int T, int C,
                                                        int n_prefix, int npix,
                                                        const float *__restrict__ w,
                                                        const float *__restrict__ b, float eps,
                                                        int l2, __bf16 *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float srow[4][256 * PER4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t tok = (int64_t)blockIdx.x * 4 + wv;
    if (tok >= (int64_t)B * npix) return;  // wave-uniform
    const int bi = (int)(tok / npix), pi = (int)(tok - (int64_t)bi * npix);
    const float *xr = x + ((int64_t)bi * T + n_prefix + pi) * C;
    vf4 v[PER4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER4; ++i) {
        const int c = 4 * lane + 256 * i;
        v[i] = c < C ? *(const vf4 *)(xr + c) : vf4{0.f, 0.f, 0.f, 0.f};
        s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    }
    const float inv_c = 1.f / (float)C;
    const float mean = vt_wave_sum(s) * inv_c;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < C) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float d = v[i][u] - mean;
                q = fmaf(d, d, q);
            }
        }
    }
    const float rstd = __builtin_amdgcn_rsqf(vt_wave_sum(q) * inv_c + eps);
    float *row = srow[wv];
#pragma unroll
    for (int i = 0; i < PER4; ++i) {
        const int c = 4 * lane + 256 * i;
        if (c < C) {
            const vf4 wv4 = *(const vf4 *)(w + c), bv = *(const vf4 *)(b + c);
            vf4 y;
#pragma unroll
            for (int u = 0; u < 4; ++u) y[u] = (v[i][u] - mean) * rstd * wv4[u] + bv[u];
            *(vf4 *)(row + c) = y;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    float scale = 1.f;
    if (l2) {
        float s2 = 0.f;
        for (int c = lane; c < C; c += 64) s2 = fmaf(row[c], row[c], s2);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s2 += __shfl_xor(s2, off);
        scale = 1.f / fmaxf(sqrtf(s2), 1e-12f);
    }
    for (int c = lane; c < C; c += 64) out[tok * C + c] = (__bf16)(row[c] * scale);
}

// patches (B * Np, Kp) bf16, Kp >= 3 p p (zero-padded), column c * p * p + ky * p + kx;
// class-token rows x[b, 0, :] = cls + pos[0].
__global__ void __launch_bounds__(256) k_patchify(const float *__restrict__ img, int B, int Hh,
                                                  int Ww, int p, int Kp, vf4 mean, vf4 stdv,
                                                  __bf16 *__restrict__ patches,
                                                  const float *__restrict__ cls,
                                                  const float *__restrict__ pos,
                                                  float *__restrict__ x, int C) {
    const int gw = Ww / p, gh = Hh / p, Np = gw * gh;
    const int64_t n_patch = (int64_t)B * Np * Kp;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid < n_patch) {
        const int64_t row = gid / Kp;
        const int col = (int)(gid - row * Kp);
        float v = 0.f;
        if (col < 3 * p * p) {
            const int b = (int)(row / Np), pi = (int)(row - (int64_t)b * Np);
            const int py = pi / gw, px = pi - py * gw;
            const int c = col / (p * p), rem = col - c * p * p, ky = rem / p, kx = rem - ky * p;
            const float raw = img[(((int64_t)b * 3 + c) * Hh + py * p + ky) * Ww + px * p + kx];
            // torchvision Normalize(mean, std)(x / 2 + 0.5): (t - mean) / std
            v = ((raw / 2.f + 0.5f) - mean[c]) / stdv[c];
        }
        patches[gid] = (__bf16)v;
    } else if (gid < n_patch + (int64_t)B * C) {
        const int64_t k = gid - n_patch;
        const int b = (int)(k / C), c = (int)(k - (int64_t)b * C);
        x[((int64_t)b * (Np + 1)) * C + c] = cls[c] + pos[c];
    }
}

// A workgroup transposes a block of 64 consecutive output tokens x 64 channels (blockIdx.y):
// rows read coalesced into a padded LDS tile, written along the pixel axis (a wave stores 64
// consecutive pixels of one channel plane: 256 B).  With L2 normalisation each block first
// computes its 64 tokens' norms (a wave per token, full-row reads from L2).
__global__ void __launch_bounds__(256) k_tokens_to_grid(const float *__restrict__ x, int B, int T,
                                                        int C, int n_prefix, int gh, int gw,
                                                        int l2, float *__restrict__ out) {
    __shared__ float tile[64][65];
    __shared__ float sc[64];
    __shared__ const float *rows[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ghw = gh * gw;
    const int n_tok = B * ghw, tok0 = blockIdx.x * 64;  // < 2^31 (checked at the ABI)
    const int c0 = blockIdx.y * 64;
    // the block's 64 input rows, one 32-bit division per token
    const int tok = tok0 + lane;
    const int bb = (unsigned)min(tok, n_tok - 1) / (unsigned)ghw;
    const int pi = min(tok, n_tok - 1) - bb * ghw;
    if (wave == 0) rows[lane] = x + ((int64_t)bb * T + n_prefix + pi) * C;
    __syncthreads();
    if (l2 && C <= 1024) {
        // 4 tokens' rows loaded together per round trip (one token at a time: 16 dependent
        // L2 round trips per wave); the same per-lane sums in the same order
        for (int i0 = wave; i0 < 64; i0 += 16) {
            float v[4][16];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + 4 * u;
                const bool ok = tok0 + i < n_tok;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const int c = lane + 64 * k;
                    v[u][k] = (ok && c < C) ? rows[i][c] : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                float s2 = 0.f;
#pragma unroll
                for (int k = 0; k < 16; ++k) s2 = fmaf(v[u][k], v[u][k], s2);
                // F.normalize(p=2, eps=1e-12) applied twice (vit.py:188,
                // dinov2_module.py:282): the second pass divides a unit vector by its norm
                const float scale = 1.f / fmaxf(sqrtf(vt_wave_sum(s2)), 1e-12f);
                if (lane == 0) sc[i0 + 4 * u] = tok0 + i0 + 4 * u < n_tok ? scale : 1.f;
            }
        }
        __syncthreads();
    } else if (l2) {
        for (int i = wave; i < 64; i += 4) {
            float scale = 1.f;
            if (tok0 + i < n_tok) {
                const float *xr = rows[i];
                float s2 = 0.f;
                for (int c = lane; c < C; c += 64) s2 = fmaf(xr[c], xr[c], s2);
                scale = 1.f / fmaxf(sqrtf(vt_wave_sum(s2)), 1e-12f);
            }
            if (lane == 0) sc[i] = scale;
        }
        __syncthreads();
    }
    for (int e = tid; e < 64 * 64; e += 256) {
        const int i = e >> 6, c = c0 + (e & 63);
        float v = (tok0 + i < n_tok && c < C) ? rows[i][c] : 0.f;
        if (l2) v *= sc[i];
        tile[i][e & 63] = v;
    }
    __syncthreads();
    if (tok < n_tok) {
        float *o = out + ((int64_t)bb * C + c0) * ghw + pi;
        for (int cc = wave; cc < 64 && c0 + cc < C; cc += 4) o[(int64_t)cc * ghw] = tile[lane][cc];
    }
}

// tokens (B, T, C) f32 -> NHWC bf16 (B, gh*gw, C) (prefix tokens dropped, optional L2
// normalisation): the DPT decoder's inputs.  One wave per token.
__global__ void __launch_bounds__(256) k_tokens_to_nhwc(const float *__restrict__ x, int B, int T,
                                                        int C, int n_prefix, int npix, int l2,
                                                        __bf16 *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t tok = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tok >= (int64_t)B * npix) return;
    const int b = (int)(tok / npix), pi = (int)(tok - (int64_t)b * npix);
    const float *xr = x + ((int64_t)b * T + n_prefix + pi) * C;
    float scale = 1.f;
    if (l2) {
        float s = 0.f;
        for (int c = lane; c < C; c += 64) s = fmaf(xr[c], xr[c], s);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off);
        scale = 1.f / fmaxf(sqrtf(s), 1e-12f);
    }
    for (int c = lane; c < C; c += 64) out[tok * C + c] = (__bf16)(xr[c] * scale);
}

// F.interpolate(scale_factor=2, mode="bilinear", align_corners=True) on NHWC bf16, one
// thread per (output pixel, 8 channels); source coordinate = dst * (in - 1) / (out - 1) in
// f32, lambda weights as aten's upsample_bilinear2d.
__global__ void __launch_bounds__(256) k_upsample2x(const __bf16 *__restrict__ in, int B, int H,
                                                    int W, int C, __bf16 *__restrict__ out) {
    const int OH = 2 * H, OW = 2 * W, C8 = C / 8;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= (int64_t)B * OH * OW * C8) return;
    const int c8 = (int)(gid % C8);
    const int64_t pix = gid / C8;
    const int ox = (int)(pix % OW);
    const int64_t t = pix / OW;
    const int oy = (int)(t % OH), b = (int)(t / OH);
    const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
    const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
    const float fy = sh * (float)oy, fx = sw * (float)ox;
    const int y0 = (int)fy, x0 = (int)fx;
    const int yp = y0 < H - 1 ? 1 : 0, xp = x0 < W - 1 ? 1 : 0;
    const float ly = fy - (float)y0, lx = fx - (float)x0;
    const float hy = 1.f - ly, hx = 1.f - lx;
    const __bf16 *base = in + ((int64_t)b * H * W) * C + c8 * 8;
    const bf16x8 v00 = *(const bf16x8 *)(base + ((int64_t)y0 * W + x0) * C);
    const bf16x8 v01 = *(const bf16x8 *)(base + ((int64_t)y0 * W + x0 + xp) * C);
    const bf16x8 v10 = *(const bf16x8 *)(base + ((int64_t)(y0 + yp) * W + x0) * C);
    const bf16x8 v11 = *(const bf16x8 *)(base + ((int64_t)(y0 + yp) * W + x0 + xp) * C);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        o[j] = (__bf16)(hy * (hx * (float)v00[j] + lx * (float)v01[j]) +
                        ly * (hx * (float)v10[j] + lx * (float)v11[j]));
    *(bf16x8 *)(out + pix * C + c8 * 8) = o;
}

// ---------------------------------------------------------------------------
// LayerNorm-prologue GEMM (the ViT's norm1 -> qkv and norm2 -> fc1 at small token counts)
// ---------------------------------------------------------------------------
// out = EPI(LN(x) W^T + b) for x (M, C) f32 residual-stream rows and W (N, C) bf16: the
// LayerNorm runs in the prologue of every 32-row tile (k_layernorm's arithmetic and order,
// rounded to bf16 as its output is) into LDS, so the normalised rows never reach HBM and the
// separate norm launch (~5 us at 481 tokens, as long as the GEMM itself) disappears.  The
// whole K = C of the weight tile is loaded into registers before the norm starts: its
// latency hides under the norm.  A 64 LG_NW-thread workgroup computes a 32 x 16 LG_NW tile, wave w
// the columns 16 w .. 16 w + 15 by v_mfma_f32_16x16x32_bf16 (A from LDS, B from registers).
// LG_NW (build knob): waves per workgroup -- the tile is 32 x 16 LG_NW, each wave normalises
// 32 / LG_NW rows, so every row's LayerNorm is recomputed once per 16 LG_NW output columns.
// Round 6: 8 (32 x 128 tiles, 4 rows per wave) instead of 4: ViT-S/16 qkv 7.68 -> 6.85 us,
// fc1 7.51 -> 6.61 us, pass 0.521 -> 0.496 ms; 2 and 16 waves slower
// (`profiles/r6_vit/lg_nw_ab.txt`)
#ifndef LG_NW
#define LG_NW 8
#endif
#define LG_BM 32
#define LG_BN (16 * LG_NW)

template <int PER, int EPI>
__global__ void __launch_bounds__(64 * LG_NW) k_lngemm(sd_gemm_args g, const float *__restrict__ x,
                                                       const float *__restrict__ lw,
                                                       const float *__restrict__ lb, float eps) {
    constexpr int C = 64 * PER, LDA = C + 8, NK = C / 32;
    constexpr int RW = LG_BM / LG_NW;  // LayerNorm rows per wave
    __shared__ __attribute__((aligned(16))) __bf16 sA[LG_BM * LDA];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, kq = lane >> 4;
    const int64_t m0 = (int64_t)blockIdx.y * LG_BM, n0 = (int64_t)blockIdx.x * LG_BN;
    const int64_t n = n0 + 16 * wave + j;
    // this lane's weight column (8 consecutive k per K step), all K steps in flight
    const __bf16 *wr = (const __bf16 *)g.w + min(n, g.N - 1) * C + 8 * kq;
    bf16x8 wb[NK];
#pragma unroll
    for (int s = 0; s < NK; ++s) wb[s] = *(const bf16x8 *)(wr + 32 * s);
    // LayerNorm of rows RW w .. RW w + RW - 1 (lane = columns lane + 64 i), RB rows at a
    // time with all their loads issued first (one memory latency per batch, the reductions
    // of the batch's rows interleaved)
    constexpr int RB = (PER <= 6 ? 8 : 4) < RW ? (PER <= 6 ? 8 : 4) : RW;
    // lane = column pairs 2 lane + 128 i: 8-B loads, packed f32 math (v_pk_*), one packed
    // bf16 pair per LDS write
    constexpr int P2 = PER / 2;
    f32x2 lwv[P2], lbv[P2];
#pragma unroll
    for (int i = 0; i < P2; ++i) {
        lwv[i] = *(const f32x2 *)(lw + 2 * lane + 128 * i);
        lbv[i] = *(const f32x2 *)(lb + 2 * lane + 128 * i);
    }
#pragma unroll
    for (int r0 = 0; r0 < RW; r0 += RB) {
        f32x2 v[RB][P2];
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
            const float *xr = x + min(m0 + RW * wave + r0 + rr, g.M - 1) * C;
#pragma unroll
            for (int i = 0; i < P2; ++i) v[rr][i] = *(const f32x2 *)(xr + 2 * lane + 128 * i);
        }
        // the row statistics by vt_wave_sum (DPP + readlane: no LDS round trip per level,
        // unlike a __shfl_xor butterfly), the divisions by C as multiplications by 1 / C
        constexpr float INV_C = 1.f / (float)C;
        float mean[RB], rstd[RB];
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
            f32x2 s2 = v[rr][0];
#pragma unroll
            for (int i = 1; i < P2; ++i) s2 += v[rr][i];
            mean[rr] = vt_wave_sum(s2.x + s2.y) * INV_C;
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
            const f32x2 mu = {mean[rr], mean[rr]};
            f32x2 q2 = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < P2; ++i) {
                v[rr][i] -= mu;  // centred in place (the output reuses it)
                q2 = __builtin_elementwise_fma(v[rr][i], v[rr][i], q2);
            }
            rstd[rr] = __builtin_amdgcn_rsqf(vt_wave_sum(q2.x + q2.y) * INV_C + eps);
        }
#pragma unroll
        for (int rr = 0; rr < RB; ++rr) {
            const int rl = RW * wave + r0 + rr;
            const f32x2 rs = {rstd[rr], rstd[rr]};
#pragma unroll
            for (int i = 0; i < P2; ++i) {
                const f32x2 y = __builtin_elementwise_fma(v[rr][i] * rs, lwv[i], lbv[i]);
                bf16x2 o;
                o[0] = (__bf16)y.x;
                o[1] = (__bf16)y.y;
                *(bf16x2 *)&sA[rl * LDA + 2 * lane + 128 * i] = o;
            }
        }
    }
    __syncthreads();
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
#pragma unroll
    for (int s = 0; s < NK; ++s) {
        const bf16x8 a0 = *(const bf16x8 *)&sA[j * LDA + 32 * s + 8 * kq];
        const bf16x8 a1 = *(const bf16x8 *)&sA[(16 + j) * LDA + 32 * s + 8 * kq];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, wb[s], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wb[s], acc1, 0, 0, 0);
    }
    if (n >= g.N) return;
    // D layout: lane (j, kq) holds rows 4 kq + r of each 16-row tile, column n
    const float bias = g.bias ? g.bias[n] : 0.f;
    if (EPI == SD_EPI_QKV) {
        // 32-bit index math (sd_ln_gemm checks every destination < 2^31 elements)
        const uint32_t Cq = (uint32_t)(g.heads * g.head_dim), nn = (uint32_t)n;
        const uint32_t which = nn / Cq, rem = nn - which * Cq;
        const uint32_t head = rem / (uint32_t)g.head_dim, e = rem - head * (uint32_t)g.head_dim;
        const uint32_t T = (uint32_t)g.tokens, Tp = (uint32_t)g.tokens_pad, HD = (uint32_t)g.head_dim;
        __bf16 *const dq = (__bf16 *)(which == 0 ? g.q : which == 1 ? g.k : g.vt);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x4 a = t ? acc1 : acc0;
            const uint32_t mb = (uint32_t)m0 + 16 * t + 4 * kq;
            // (image, token) of row mb by one divide; rows mb + 1 .. mb + 3 step from it
            const uint32_t b0 = mb / T, tk0 = mb - b0 * T;
            if (which == 2 && mb + 3 < (uint32_t)g.M && tk0 + 3 < T && (tk0 & 3) == 0) {
                // V^T: the lane's 4 rows are 4 consecutive tokens of its head-dim row
                bf16x4 v4;
#pragma unroll
                for (int u = 0; u < 4; ++u) v4[u] = (__bf16)(a[u] + bias);
                *(bf16x4 *)(dq + ((b0 * g.heads + head) * HD + e) * Tp + tk0) = v4;
                continue;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t m = mb + u;
                if (m >= (uint32_t)g.M) break;
                uint32_t b, tk;
                if (T >= 4) {  // at most one image boundary in 4 rows
                    const bool wrap = tk0 + u >= T;
                    b = b0 + (wrap ? 1u : 0u);
                    tk = tk0 + u - (wrap ? T : 0u);
                } else {
                    b = m / T;
                    tk = m - b * T;
                }
                const uint32_t bh = b * g.heads + head;
                const uint32_t off = which == 0 ? (bh * T + tk) * HD + e
                                   : which == 1 ? (bh * Tp + tk) * HD + e : (bh * HD + e) * Tp + tk;
                dq[off] = (__bf16)(a[u] + bias);
            }
        }
    } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const f32x4 a = t ? acc1 : acc0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t m = m0 + 16 * t + 4 * kq + u;
                if (m >= g.M) break;
                float v = a[u] + bias;
                if (EPI == SD_EPI_GELU) v = vt_gelu(v);
                ((__bf16 *)g.out)[m * g.ldo + n] = (__bf16)v;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// One ViT block's MLP half in one launch (timm Block, vit.py:112-189):
//   x += ls2 * (fc2(gelu(fc1(norm2(x)))) + b2)
// for C = 384 (ViT-S: five launches per block -> four).  A 512-thread workgroup owns a
// 32-row band and a 256-wide hidden chunk: LayerNorm of its rows from x_ln (an f32 copy of x
// the preceding residual GEMM wrote, so the atomics below never meet a row another
// workgroup is still normalising) into LDS as bf16 (k_lngemm's arithmetic), fc1 + bias +
// exact GELU on the chunk (bf16 rows in LDS: the rounding of the GEMM path's hidden rows),
// then the chunk's partial fc2 product, added into x as ls2 * (partial [+ b2 on chunk 0]) by
// f32 atomics (the sum over chunks is in arrival order).  Each wave's W1 slice (32 hidden x
// C) is in registers before the LayerNorm starts and its W2 slice (48 columns x the chunk)
// is loaded while fc1 finishes: one weight round trip each, no K loop.  v_mfma_f32_16x16x32.
// ---------------------------------------------------------------------------
#define VM_BM 32
#define VM_HC 256

template <int PER>
__global__ void __launch_bounds__(512) k_vit_mlp(const float *__restrict__ xln, float *__restrict__ x,
                                                 int M, int hidden, const float *__restrict__ lw,
                                                 const float *__restrict__ lb, float eps,
                                                 const __bf16 *__restrict__ w1,
                                                 const float *__restrict__ b1,
                                                 const __bf16 *__restrict__ w2,
                                                 const float *__restrict__ b2,
                                                 const float *__restrict__ gamma) {
    constexpr int C = 64 * PER, LDA = C + 8, NK1 = C / 32, LDH = VM_HC + 8, NK2 = VM_HC / 32;
    constexpr int NT2 = C / 128;  // fc2: 16-column subtiles per wave (8 waves)
    __shared__ __attribute__((aligned(16))) __bf16 sA[VM_BM * LDA];
    __shared__ __attribute__((aligned(16))) __bf16 sH[VM_BM * LDH];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.y * VM_BM, c0 = blockIdx.x * VM_HC;
    // this wave's fc1 columns c0 + 32 w + 16 t + j: all of K in flight
    bf16x8 wb1[2][NK1];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const __bf16 *wr = w1 + (int64_t)(c0 + 32 * wave + 16 * t + j) * C + 8 * kq;
#pragma unroll
        for (int s = 0; s < NK1; ++s) wb1[t][s] = *(const bf16x8 *)(wr + 32 * s);
    }
    // LayerNorm of rows 4 w .. 4 w + 3 (lane = column pairs 2 lane + 128 i; k_lngemm's order)
    {
        constexpr int P2 = PER / 2;
        f32x2 lwv[P2], lbv[P2], v[4][P2];
#pragma unroll
        for (int i = 0; i < P2; ++i) {
            lwv[i] = *(const f32x2 *)(lw + 2 * lane + 128 * i);
            lbv[i] = *(const f32x2 *)(lb + 2 * lane + 128 * i);
        }
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const float *xr = xln + (int64_t)min(m0 + 4 * wave + rr, M - 1) * C;
#pragma unroll
            for (int i = 0; i < P2; ++i) v[rr][i] = *(const f32x2 *)(xr + 2 * lane + 128 * i);
        }
        constexpr float INV_C = 1.f / (float)C;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            f32x2 s2 = v[rr][0];
#pragma unroll
            for (int i = 1; i < P2; ++i) s2 += v[rr][i];
            const float mean = vt_wave_sum(s2.x + s2.y) * INV_C;
            const f32x2 mu = {mean, mean};
            f32x2 q2 = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < P2; ++i) {
                v[rr][i] -= mu;
                q2 = __builtin_elementwise_fma(v[rr][i], v[rr][i], q2);
            }
            const float rstd = __builtin_amdgcn_rsqf(vt_wave_sum(q2.x + q2.y) * INV_C + eps);
            const f32x2 rs = {rstd, rstd};
            const int rl = 4 * wave + rr;
#pragma unroll
            for (int i = 0; i < P2; ++i) {
                const f32x2 y = __builtin_elementwise_fma(v[rr][i] * rs, lwv[i], lbv[i]);
                bf16x2 o;
                o[0] = (__bf16)y.x;
                o[1] = (__bf16)y.y;
                *(bf16x2 *)&sA[rl * LDA + 2 * lane + 128 * i] = o;
            }
        }
    }
    __syncthreads();
    // fc1 on the chunk: rows j / 16 + j, columns of subtile t
    f32x4 acc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NK1; ++s) {
        const bf16x8 a0 = *(const bf16x8 *)&sA[j * LDA + 32 * s + 8 * kq];
        const bf16x8 a1 = *(const bf16x8 *)&sA[(16 + j) * LDA + 32 * s + 8 * kq];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, wb1[t][s], acc[t][0], 0, 0, 0);
            acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wb1[t][s], acc[t][1], 0, 0, 0);
        }
    }
    // this wave's fc2 columns 48 w + 16 t + j over the chunk's K, in flight under the GELU
    bf16x8 wb2[NT2][NK2];
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
        const __bf16 *wr = w2 + (int64_t)(16 * NT2 * wave + 16 * t + j) * hidden + c0 + 8 * kq;
#pragma unroll
        for (int s = 0; s < NK2; ++s) wb2[t][s] = *(const bf16x8 *)(wr + 32 * s);
    }
    // bias + GELU -> bf16 hidden rows (D layout: lane (j, kq) holds rows 4 kq + u, column j)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int hc = 32 * wave + 16 * t + j;
        const float bias = b1[c0 + hc];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                sH[(16 * rt + 4 * kq + u) * LDH + hc] = (__bf16)vt_gelu(acc[t][rt][u] + bias);
    }
    __syncthreads();
    f32x4 acc2[NT2][2];
#pragma unroll
    for (int t = 0; t < NT2; ++t) acc2[t][0] = acc2[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NK2; ++s) {
        const bf16x8 a0 = *(const bf16x8 *)&sH[j * LDH + 32 * s + 8 * kq];
        const bf16x8 a1 = *(const bf16x8 *)&sH[(16 + j) * LDH + 32 * s + 8 * kq];
#pragma unroll
        for (int t = 0; t < NT2; ++t) {
            acc2[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, wb2[t][s], acc2[t][0], 0, 0, 0);
            acc2[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, wb2[t][s], acc2[t][1], 0, 0, 0);
        }
    }
    // x += ls2 * (partial [+ b2]): one f32 atomic per element (the chunks' partials meet in x)
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
        const int n = 16 * NT2 * wave + 16 * t + j;
        const float gm = gamma ? gamma[n] : 1.f;
        const float bb = (c0 == 0 && b2) ? b2[n] : 0.f;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = m0 + 16 * rt + 4 * kq + u;
                if (m < M) unsafeAtomicAdd(x + (int64_t)m * C + n, gm * (acc2[t][rt][u] + bb));
            }
    }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int sd_vit_mlp(const float *x_ln, float *x, int64_t M, int32_t C, int32_t hidden,
                          const float *ln_w, const float *ln_b, float eps, const void *fc1_w,
                          const float *fc1_b, const void *fc2_w, const float *fc2_b,
                          const float *gamma, void *stream) {
    if (!x_ln || !x || !ln_w || !ln_b || !fc1_w || !fc1_b || !fc2_w || M < 0 || C != 384 ||
        hidden <= 0 || hidden % VM_HC || M * (int64_t)C >= ((int64_t)1 << 31) || x_ln == x) {
        sd_set_error("sd_vit_mlp: invalid argument (C = 384, hidden % 256 == 0, x_ln a separate copy)");
        return -1;
    }
    if (M == 0) return 0;
    const dim3 grid((unsigned)(hidden / VM_HC), (unsigned)((M + VM_BM - 1) / VM_BM));
    hipLaunchKernelGGL(k_vit_mlp<6>, grid, dim3(512), 0, (hipStream_t)stream, x_ln, x, (int)M,
                       hidden, ln_w, ln_b, eps, (const __bf16 *)fc1_w, fc1_b,
                       (const __bf16 *)fc2_w, fc2_b, gamma);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_vit_mlp: launch failed");
        return -2;
    }
    return 0;
}

// cross-workgroup split-K workspace (per device, allocated once outside graph capture):
// 32 x 32 f32 partials and self-resetting tickets (zeroed at allocation)
#define VT_SK_SLABS 2048
#define VT_SK_TILES 4096
struct VtSplitWs {
    float *slab = nullptr;
    uint32_t *cnt = nullptr;
};
static bool vt_split_ws(hipStream_t s, VtSplitWs &w) {
    static VtSplitWs ws[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    if (!ws[dev].slab) {
        hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return false;
        float *p = nullptr;
        uint32_t *c = nullptr;
        if (hipMalloc((void **)&p, (size_t)VT_SK_SLABS * 4096) != hipSuccess) return false;
        if (hipMalloc((void **)&c, (size_t)VT_SK_TILES * 4) != hipSuccess ||
            hipMemset(c, 0, (size_t)VT_SK_TILES * 4) != hipSuccess) {
            (void)hipFree(p);
            return false;
        }
        ws[dev].slab = p;
        ws[dev].cnt = c;
    }
    w = ws[dev];
    return true;
}

template <int BM, int BN, int BK, bool CONV>
static void vt_launch_gemm(const sd_gemm_args &g, hipStream_t s, int ksplit = 1, const VtLnTail &lt = VtLnTail{}) {
    dim3 grid((unsigned)((g.N + BN - 1) / BN), (unsigned)((g.M + BM - 1) / BM));
    VtSplitWs w;
    if (ksplit > 1 && vt_ring_tile(BM) && (int64_t)grid.x * grid.y <= VT_SK_TILES &&
        (int64_t)grid.x * grid.y * ksplit <= VT_SK_SLABS && vt_split_ws(s, w))
        grid.z = (unsigned)ksplit;
    // the ring kernels take their LDS dynamically (the ring, reused by the epilogue: > 64 KiB
    // for the 128 x 128 tiles)
    constexpr int ep = BM * (BN + 8) * 4;  // the widest staged epilogue tile (k_gemm's OST)
    const int lds = vt_ring_tile(BM) ? (vt_ring_bytes<BM, BN, BK>() > ep ? vt_ring_bytes<BM, BN, BK>() : ep) : 0;
    auto go = [&](auto kern) {
        if (lds) sd_lds_attr((const void *)kern, lds);
        hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, g, w.slab, w.cnt, lt);
    };
    switch (g.epi) {
    case SD_EPI_BF16: go(k_gemm<BM, BN, BK, SD_EPI_BF16, CONV>); break;
    case SD_EPI_GELU: go(k_gemm<BM, BN, BK, SD_EPI_GELU, CONV>); break;
    case SD_EPI_F32: go(k_gemm<BM, BN, BK, SD_EPI_F32, CONV>); break;
    case SD_EPI_RESID:
        if (lt.out && !CONV) go(k_gemm<BM, BN, BK, VT_EPI_RESID_LN, false>);
        else go(k_gemm<BM, BN, BK, SD_EPI_RESID, CONV>);
        break;
    case SD_EPI_QKV: go(k_gemm<BM, BN, BK, SD_EPI_QKV, CONV>); break;
    case SD_EPI_SHUF: go(k_gemm<BM, BN, BK, SD_EPI_SHUF, CONV>); break;
    case SD_EPI_NCHW: go(k_gemm<BM, BN, BK, SD_EPI_NCHW, CONV>); break;
    default: go(k_gemm<BM, BN, BK, SD_EPI_PATCH, CONV>); break;
    }
}

#ifndef VT_SK256
#define VT_SK256 1
#endif
#ifndef SD_CONV_SK_MID
#define SD_CONV_SK_MID 256  // conv: split-K tiles below this many 64x64 tiles (1024: no gain)
#endif

// SD_GEMM_TILE (diagnostic A/B runs, read once): "128", "64" or "sk" forces that tiling
// (64x128 tiles and 64x64 tiles with BK = 128 were measured slower on every encoder shape)
static int vt_forced_tile() {
    static int f = -2;
    if (f == -2) {
        const char *e = getenv("SD_GEMM_TILE");
        f = !e ? -1 : !strcmp(e, "128") ? 128 : !strcmp(e, "64") ? 64 : !strcmp(e, "sk") ? 32 : -1;
    }
    return f;
}

template <bool CONV>
static void vt_pick_gemm(const sd_gemm_args &g, hipStream_t s, const VtLnTail &lt = VtLnTail{}) {
    const int ft = vt_forced_tile();
    if (ft == 32 && g.K % 128 == 0 && g.K >= 256 && (!CONV || g.Cin % 128 == 0)) {
        vt_launch_gemm<32, 32, 128, CONV>(g, s, 1, lt);
        return;
    }
    if (ft == 128 || ft == 64) {
        if (g.K % 64 == 0) {
            if (ft == 128) vt_launch_gemm<128, 128, 64, CONV>(g, s, 1, lt); else vt_launch_gemm<64, 64, 64, CONV>(g, s, 1, lt);
        } else {
            if (ft == 128) vt_launch_gemm<128, 128, 32, CONV>(g, s, 1, lt); else vt_launch_gemm<64, 64, 32, CONV>(g, s, 1, lt);
        }
        return;
    }
    // K steps of 64 whenever K allows (half the barriers, twice the work under each
    // prefetch); 128x128 tiles once they fill the chip, else 64x64
    const int64_t big = ((g.M + 127) / 128) * ((g.N + 127) / 128);
    const int64_t mid = ((g.M + 63) / 64) * ((g.N + 63) / 64);
    // conv: a 128-deep K step must stay inside one 3x3 tap (Cin % 128 == 0); the DPT's
    // low-resolution 256-channel convolutions (12x40, 24x80) are exactly these small-M,
    // large-K GEMMs
    // split-K tiles that leave CUs idle (ViT-S/16 fc2 at 481 tokens: 192; the DPT's 12x40
    // convolutions: 120) take 256-deep K steps: half the dependent ring steps per tile, a
    // 128-KiB ring (one tile per CU is all there is anyway)
    const int64_t t32 = ((g.M + 31) / 32) * ((g.N + 31) / 32);
    // and, where the tiles leave most CUs idle, optionally their K range split over
    // workgroups (deterministic last-arriver combine): the largest of 2, 4, 8 slices keeping
    // tiles x slices <= SD_SPLITK_WG and >= 2 K steps per slice.  Off by default: the
    // tickets and partial slabs are one workspace per device, so two split launches must
    // not run concurrently -- and the encoder now runs the DPT's level fronts on side
    // streams beside the ViT.  Measured (profiles/r4_splitk_ab.txt, interleaved, one
    // stream): at one tile per CU only the 12x40 convolutions split (encode 1.16 -> 1.15 ms);
    // at two per CU the ViT-S/16 fc2 splits too and runs slower (0.576 -> 0.624 ms)
    auto ksplit = [&](int bk) {
        const char *e = getenv("SD_SPLITK_WG");
        const int64_t cap = (e && e[0]) ? atoll(e) : 0;
        // SD_SPLITK_STEPS: the fewest K steps a slice may keep (default 2)
        const char *es = getenv("SD_SPLITK_STEPS");
        const int64_t mst = (es && es[0]) ? atoll(es) : 2;
        int ks = 1;
        while (ks < 8 && t32 * ks * 2 <= cap && g.K / bk >= mst * ks * 2) ks *= 2;
        return ks;
    };
    if (VT_SK256 && VT_RING && t32 <= (int64_t)sd_num_cus() && g.K % 256 == 0 &&
        (CONV ? g.Cin % 256 == 0 && mid < SD_CONV_SK_MID : mid < 256)) {
        vt_launch_gemm<32, 32, 256, CONV>(g, s, ksplit(256), lt);
        return;
    }
    if ((CONV ? g.Cin % 128 == 0 && mid < SD_CONV_SK_MID : mid < 256) && g.K % 128 == 0 &&
        g.K >= 256) {
        vt_launch_gemm<32, 32, 128, CONV>(g, s, ksplit(128), lt);  // split-K over the 4 waves
        return;
    }
    // 128x128 tiles need about two per CU, or one per CU with a long K loop to amortise
    // their prologue / epilogue; below that the 64x64 tiling wins (sd_gemm on the ViT-B/8
    // block shapes at 1921 tokens, tools/gemm_bench.py: qkv 24.6 -> 18.6 us, fc1 22.4 ->
    // 20.3 us; the DPT's 3x3 convolutions at K = 2304 keep 128x128)
    const bool use128 = big >= 512 || (big >= 256 && g.K >= 2048);
    if (g.K % 64 == 0) {
        if (use128)
            vt_launch_gemm<128, 128, 64, CONV>(g, s, 1, lt);
        else
            vt_launch_gemm<64, 64, 64, CONV>(g, s, 1, lt);
    } else {
        if (use128)
            vt_launch_gemm<128, 128, 32, CONV>(g, s, 1, lt);
        else
            vt_launch_gemm<64, 64, 32, CONV>(g, s, 1, lt);
    }
}

extern "C" int sd_gemm(const sd_gemm_args *args, void *stream) {
    if (!args) {
        sd_set_error("sd_gemm: null args");
        return -1;
    }
    const sd_gemm_args &g = *args;
    bool ok = g.a && g.w && g.M >= 0 && g.N > 0 && g.K > 0 && g.K % GK == 0 && g.lda >= g.K &&
              g.lda % 8 == 0 && g.epi >= SD_EPI_BF16 && g.epi <= SD_EPI_NCHW &&
              g.M * (int64_t)g.lda < ((int64_t)1 << 31) && g.N * g.K < ((int64_t)1 << 31);
    if (g.conv)
        ok = ok && g.H > 0 && g.W > 0 && g.Cin > 0 && g.Cin % 64 == 0 && g.K == 9LL * g.Cin &&
             g.stride >= 1 && g.OH > 0 && g.OW > 0 && g.M % ((int64_t)g.OH * g.OW) == 0 &&
             (g.M / ((int64_t)g.OH * g.OW)) * g.H * g.W * g.Cin < ((int64_t)1 << 30);
    if (g.epi == SD_EPI_SHUF)
        ok = ok && g.out && g.shuf_k > 0 && g.N % (g.shuf_k * g.shuf_k) == 0 && g.in_h > 0 &&
             g.in_w > 0 && g.M % ((int64_t)g.in_h * g.in_w) == 0;
    else if (g.epi == SD_EPI_NCHW)
        ok = ok && g.out && g.tokens > 0 && g.M % g.tokens == 0;
    else if (g.epi == SD_EPI_QKV)
        ok = ok && g.q && g.k && g.vt && g.head_dim > 0 && g.heads > 0 && g.tokens > 0 &&
             g.tokens_pad >= g.tokens && g.N == 3LL * g.heads * g.head_dim &&
             g.M % g.tokens == 0 && g.head_dim % 8 == 0 && g.tokens_pad % 8 == 0;
    else if (g.epi == SD_EPI_PATCH)
        ok = ok && g.out && g.pos && g.patches > 0 && g.M % g.patches == 0 && g.ldo >= g.N;
    else if (g.epi == SD_EPI_RESID && g.q)
        ok = ok && g.out && g.ldo >= g.N && g.tokens > 1 && g.M % g.tokens == 0;
    else
        ok = ok && g.out && g.ldo >= g.N;
    if (!ok) {
        sd_set_error("sd_gemm: invalid argument (K % 32 == 0, lda >= K and lda % 8 == 0, "
                     "operands < 4 GiB, epilogue fields)");
        return -1;
    }
    if (g.M == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int big = sd_conv_big_try(&g, stream);  // the DPT's 192x640 / 96x320 layers
    if (big < 0) {
        sd_set_error("sd_gemm: launch failed");
        return -2;
    }
    if (!big) {
        if (g.conv)
            vt_pick_gemm<true>(g, s);
        else
            vt_pick_gemm<false>(g, s);
    }
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_gemm: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_gemm_resid_ln(const sd_gemm_args *args, const float *ln_w, const float *ln_b,
                                float eps, void *ln_out, uint32_t *ln_ws, void *stream) {
    if (!args) {
        sd_set_error("sd_gemm_resid_ln: null args");
        return -1;
    }
    const sd_gemm_args &g = *args;
    const bool ok = g.epi == SD_EPI_RESID && !g.conv && g.a && g.w && g.out && g.M >= 0 &&
                    g.N > 0 && g.N <= 1024 && g.N % 4 == 0 && g.K > 0 && g.K % GK == 0 &&
                    g.lda >= g.K && g.lda % 8 == 0 && g.ldo >= g.N &&
                    g.M * (int64_t)g.lda < ((int64_t)1 << 31) && g.M * (int64_t)g.ldo < ((int64_t)1 << 31) &&
                    g.N * g.K < ((int64_t)1 << 31) && (!g.q || (g.tokens > 1 && g.M % g.tokens == 0)) &&
                    ln_w && ln_b && ln_out && ln_ws && g.ldo % 4 == 0 &&
                    !(((uintptr_t)ln_w | (uintptr_t)ln_b | (uintptr_t)g.out) & 15) && !((uintptr_t)ln_out & 7);
    if (!ok) {
        sd_set_error("sd_gemm_resid_ln: invalid argument (SD_EPI_RESID, N <= 1024 and N % 4 == 0, "
                     "16-B aligned rows, LayerNorm weights / output / ticket workspace)");
        return -1;
    }
    if (g.M == 0) return 0;
    const VtLnTail lt{ln_w, ln_b, eps, (__bf16 *)ln_out, ln_ws};
    vt_pick_gemm<false>(g, (hipStream_t)stream, lt);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_gemm_resid_ln: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_ln_gemm(const sd_gemm_args *args, const float *x, const float *ln_w,
                          const float *ln_b, float eps, void *stream) {
    if (!args || !x || !ln_w || !ln_b) {
        sd_set_error("sd_ln_gemm: null argument");
        return -1;
    }
    const sd_gemm_args &g = *args;
    const int64_t C = g.K;
    bool ok = g.w && g.M >= 0 && g.N > 0 && (C == 384 || C == 768) &&
              (g.epi == SD_EPI_QKV || g.epi == SD_EPI_GELU || g.epi == SD_EPI_BF16) &&
              g.M * C < ((int64_t)1 << 31) && g.N * C < ((int64_t)1 << 31);
    if (g.epi == SD_EPI_QKV)
        ok = ok && g.q && g.k && g.vt && g.head_dim > 0 && g.heads > 0 && g.tokens > 0 &&
             g.tokens_pad >= g.tokens && g.N == 3LL * g.heads * g.head_dim && g.M % g.tokens == 0 &&
             g.head_dim % 8 == 0 && g.tokens_pad % 8 == 0 &&  // 8-B V^T stores, as sd_gemm
             (g.M / g.tokens) * g.heads * g.tokens_pad * g.head_dim < ((int64_t)1 << 31);
    else
        ok = ok && g.out && g.ldo >= g.N;
    if (!ok) {
        sd_set_error("sd_ln_gemm: invalid argument (K = C in {384, 768}, epi QKV / GELU / BF16)");
        return -1;
    }
    if (g.M == 0) return 0;
    dim3 grid((unsigned)((g.N + LG_BN - 1) / LG_BN), (unsigned)((g.M + LG_BM - 1) / LG_BM));
    hipStream_t s = (hipStream_t)stream;
#define SD_LG(PER, E) hipLaunchKernelGGL((k_lngemm<PER, E>), grid, dim3(64 * LG_NW), 0, s, g, x, ln_w, ln_b, eps)
    if (C == 384) {
        if (g.epi == SD_EPI_QKV) SD_LG(6, SD_EPI_QKV);
        else if (g.epi == SD_EPI_GELU) SD_LG(6, SD_EPI_GELU);
        else SD_LG(6, SD_EPI_BF16);
    } else {
        if (g.epi == SD_EPI_QKV) SD_LG(12, SD_EPI_QKV);
        else if (g.epi == SD_EPI_GELU) SD_LG(12, SD_EPI_GELU);
        else SD_LG(12, SD_EPI_BF16);
    }
#undef SD_LG
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_ln_gemm: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_attention(const void *q, const void *k, const void *vt, int32_t B,
                            int32_t heads, int32_t tokens, int32_t tokens_pad, int32_t head_dim,
                            float scale, void *out, void *stream) {
    if (!q || !k || !vt || !out || B <= 0 || heads <= 0 || tokens <= 0 || head_dim != AT_HD ||
        tokens_pad < tokens || tokens_pad % 64 || (int64_t)B * heads > 65535) {
        sd_set_error("sd_attention: invalid argument (head_dim 64, tokens_pad % 64 == 0)");
        return -1;
    }
    // 128-query workgroups sharing K / V^T through LDS once they cover half the CUs
    // (ViT-B/8, 1921 tokens x 12 heads: 30.7 us vs 47.7 us split); below that 32-query
    // workgroups splitting the keys (481 tokens: 7.9 us vs 10.5 us).  SD_ATTN=lds / dir
    // forces one (A/B runs).
    const float sl2e = scale * 1.4426950408889634f;
    const int64_t wg128 = (int64_t)((tokens + 127) / 128) * B * heads;
    const char *force = getenv("SD_ATTN");
    const bool lds = (force && force[0]) ? force[0] == 'l' || force[0] == '2' : 2 * wg128 >= (int64_t)sd_num_cus();
    // under one 128-query workgroup per CU: 64-query workgroups over two key halves
    const bool split = (force && force[0]) ? force[0] == '2' : wg128 < (int64_t)sd_num_cus();
    if (lds && split) {
        dim3 grid((unsigned)((tokens + 63) / 64), (unsigned)(B * heads));
        hipLaunchKernelGGL(k_attn_lds<2>, grid, dim3(256), 0, (hipStream_t)stream, (const __bf16 *)q,
                           (const __bf16 *)k, (const __bf16 *)vt, tokens, tokens_pad, heads, sl2e,
                           (__bf16 *)out);
    } else if (lds) {
        dim3 grid((unsigned)((tokens + 127) / 128), (unsigned)(B * heads));
        hipLaunchKernelGGL(k_attn_lds<1>, grid, dim3(256), 0, (hipStream_t)stream, (const __bf16 *)q,
                           (const __bf16 *)k, (const __bf16 *)vt, tokens, tokens_pad, heads, sl2e,
                           (__bf16 *)out);
    } else {
        dim3 grid((unsigned)((tokens + 31) / 32), (unsigned)(B * heads));
        constexpr int lds_b = at_dir_lds(AT_DIR_NW);
        if (lds_b > 64 * 1024) sd_lds_attr((const void *)k_attn_dir<AT_DIR_NW>, lds_b);
        hipLaunchKernelGGL(k_attn_dir<AT_DIR_NW>, grid, dim3(64 * AT_DIR_NW), lds_b, (hipStream_t)stream, (const __bf16 *)q,
                           (const __bf16 *)k, (const __bf16 *)vt, tokens, tokens_pad, heads, sl2e,
                           (__bf16 *)out);
    }
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_attention: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_layernorm(const float *x, int64_t rows, int32_t C, const float *w,
                            const float *b, float eps, void *out, int32_t out_f32,
                            void *stream) {
    if (!x || !w || !b || !out || rows < 0 || C <= 0 || C > 1024 || C % 4 != 0 ||
        ((uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)out) & 15) {
        sd_set_error("sd_layernorm: invalid argument (C <= 1024, C % 4 == 0, 16-B aligned)");
        return -1;
    }
    if (rows == 0) return 0;
    dim3 grid((unsigned)((rows + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
#define SD_LN(PER)                                                                          \
    do {                                                                                    \
        if (out_f32)                                                                        \
            hipLaunchKernelGGL((k_layernorm<PER, true>), grid, dim3(256), 0, s, x, rows, C, w, \
                               b, eps, out);                                                \
        else                                                                                \
            hipLaunchKernelGGL((k_layernorm<PER, false>), grid, dim3(256), 0, s, x, rows, C,   \
                               w, b, eps, out);                                             \
    } while (0)
    if (C <= 512)
        SD_LN(2);
    else if (C <= 768)
        SD_LN(3);
    else
        SD_LN(4);
#undef SD_LN
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_layernorm: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_patchify(const float *img, int32_t B, int32_t H, int32_t W, int32_t p,
                           int32_t Kp, const float *mean3, const float *std3, void *patches,
                           const float *cls, const float *pos, float *x, int32_t C, void *stream) {
    if (!img || !mean3 || !std3 || !patches || !cls || !pos || !x || B <= 0 || p <= 0 ||
        H % p || W % p || Kp < 3 * p * p || C <= 0) {
        sd_set_error("sd_patchify: invalid argument (H, W multiples of the patch size)");
        return -1;
    }
    vf4 mean, stdv;
    for (int c = 0; c < 3; ++c) {
        mean[c] = mean3[c];
        stdv[c] = std3[c];
    }
    mean[3] = 0.f;
    stdv[3] = 1.f;
    const int64_t Np = (int64_t)(H / p) * (W / p);
    const int64_t n = (int64_t)B * Np * Kp + (int64_t)B * C;
    hipLaunchKernelGGL(k_patchify, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, img, B, H, W, p, Kp, mean, stdv, (__bf16 *)patches,
                       cls, pos, x, C);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_patchify: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_tokens_to_grid(const float *x, int32_t B, int32_t T, int32_t C,
                                 int32_t n_prefix, int32_t gh, int32_t gw, int32_t l2norm,
                                 float *out, void *stream) {
    if (!x || !out || B <= 0 || C <= 0 || n_prefix < 0 || gh <= 0 || gw <= 0 ||
        (int64_t)n_prefix + (int64_t)gh * gw > T || (int64_t)B * gh * gw >= ((int64_t)1 << 31)) {
        sd_set_error("sd_tokens_to_grid: invalid argument");
        return -1;
    }
    const int64_t n = (int64_t)B * gh * gw;
    hipLaunchKernelGGL(k_tokens_to_grid, dim3((unsigned)((n + 63) / 64), (unsigned)((C + 63) / 64)), dim3(256), 0,
                       (hipStream_t)stream, x, B, T, C, n_prefix, gh, gw, l2norm, out);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_tokens_to_grid: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_tokens_to_nhwc(const float *x, int32_t B, int32_t T, int32_t C,
                                 int32_t n_prefix, int32_t npix, int32_t l2norm, void *out,
                                 void *stream) {
    if (!x || !out || B <= 0 || C <= 0 || n_prefix < 0 || npix <= 0 ||
        (int64_t)n_prefix + npix > T) {
        sd_set_error("sd_tokens_to_nhwc: invalid argument");
        return -1;
    }
    const int64_t n = (int64_t)B * npix;
    hipLaunchKernelGGL(k_tokens_to_nhwc, dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, x, B, T, C, n_prefix, npix, l2norm, (__bf16 *)out);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_tokens_to_nhwc: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_layernorm_nhwc(const float *x, int32_t B, int32_t T, int32_t C,
                                 const float *w, const float *b, float eps, int32_t n_prefix,
                                 int32_t npix, int32_t l2norm, void *out, void *stream) {
    if (!x || !w || !b || !out || B <= 0 || C <= 0 || C > 1024 || C % 4 != 0 || n_prefix < 0 ||
        npix <= 0 || (int64_t)n_prefix + npix > T ||
        ((uintptr_t)x | (uintptr_t)w | (uintptr_t)b) & 15) {
        sd_set_error("sd_layernorm_nhwc: invalid argument (C <= 1024, C % 4 == 0, 16-B aligned)");
        return -1;
    }
    const int64_t n = (int64_t)B * npix;
    dim3 grid((unsigned)((n + 3) / 4));
    hipStream_t s = (hipStream_t)stream;
#define SD_LNG(PER) hipLaunchKernelGGL((k_layernorm_nhwc<PER>), grid, dim3(256), 0, s, x, B, T, C, \
                                       n_prefix, npix, w, b, eps, l2norm, (__bf16 *)out)
    if (C <= 512)
        SD_LNG(2);
    else if (C <= 768)
        SD_LNG(3);
    else
        SD_LNG(4);
#undef SD_LNG
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_layernorm_nhwc: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_upsample2x(const void *in, int32_t B, int32_t H, int32_t W, int32_t C,
                             void *out, void *stream) {
    if (!in || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8) {
        sd_set_error("sd_upsample2x: invalid argument (C % 8 == 0)");
        return -1;
    }
    const int64_t n = (int64_t)B * 4 * H * W * (C / 8);
    hipLaunchKernelGGL(k_upsample2x, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, (const __bf16 *)in, B, H, W, C, (__bf16 *)out);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_upsample2x: launch failed");
        return -2;
    }
    return 0;
}
