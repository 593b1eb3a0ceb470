// sdhip_tile.hip -- LDS-staged projected-grid render (gfx950 / CDNA4, 16-bit modes).
//
// Same computation as k_render_proj (sdhip_proj.hip: NeRFRenderer.composite over
// BTSNet.forward, nerf.py:230-449 / bts.py:271-595, on the projected grid
// P = W_in[:, :C] G + b_in), organised so that the bilinear P taps come from LDS instead
// of the vector-memory path.  Per sample the taps are 4 x 256 B; through global loads
// every byte passes the CU's texture path (~64 B/clk), which bounds k_render_proj.  Rays
// of neighbouring pixels sample neighbouring texels, so one workgroup renders a GROUP of
// 8 consecutive rays at a time (one per wave) and stages the bounding box of all their
// taps, read once from L2 by LDS-DMA, in LDS.
//
// Workgroup = 8 waves, one workgroup per CU.  Step n: wave w renders ray 8 G_n + w.
//   item 0    ray pass of the wave's NEXT ray (geometry, taps, colours -> LDS records,
//             tap bounding box -> LDS), the DINO head of the previous group (below),
//             then item 0 of the current ray
//   barrier X union of the next group's boxes; if it fits the tile buffer, every wave
//             issues its share of the LDS-DMA of those P texels (else the group goes to
//             the overflow list and the fallback kernel renders it)
//   items 1.. of the current ray (taps from the current tile buffer), ray epilogue:
//             depth / colour stored, the composited hidden sum_k w_k relu(h_k) -> LDS
//   vmcnt(0), barrier Y
// Blend as MFMA: hidden[h][j] = sum_{tap q, sample s} P_q(s)[h] * Wb[(s, q)][j] with the
// block-diagonal bilinear weights Wb[(s, q)][j] = w_q(j) [s == j]; A (P taps) is read with
// ds_read_b64_tr_b16 (lane 4q + p of a 16-lane group addresses tap q of the group's
// sample, columns 4p..4p+3; lane i receives hidden 16 t + i of the 4 taps).  Per 16-sample
// item: 2 K-chunks of 8 samples x 8 hidden tiles = 16 MFMA 16x16x32, no blend VALU.
// Then as k_render_proj: + W_code . code (16 MFMA), ReLU, sigma (4 MFMA), softplus,
// alpha, DPP transmittance scan, and hidden-space compositing (v_dot2 of the packed
// hidden pairs with (w, 0) / (0, w)).  The output layer is linear, so
//   dino = sum_k w_k (W h_k + b) = W (sum_k w_k h_k) + b sum_k w_k          (nerf.py:394)
// and is applied per GROUP: hsum of the 8 rays as the B operand (8 of 16 columns),
// D / 16 MFMA tiles spread over the waves.
#include "sdhip_render.h"

// waves per workgroup = rays per group (NW): 8 (2 waves per SIMD), or for K <= 64 the
// ST_NW_SMALLK-wave variant (12: 3 waves per SIMD, the kernel compiled for <= 168 VGPRs)
#ifndef ST_NW_SMALLK
#define ST_NW_SMALLK 8
#endif
#define ST_TEX 288          // LDS bytes per staged texel: 256 B of P + 32 B pad
#define ST_TEXQ 18          // 16-byte chunks per staged texel
#define ST_MAXP 2           // K <= 128 (two samples per lane in the ray pass)

// diagnostic ablation switches (timing experiments only; outputs are wrong when set)
#ifndef ST_PIPE
#define ST_PIPE 0           // 1: item i + 1's MLP beside item i's compositing (measured slower)
#endif
#ifndef ST_HC_MFMA
#define ST_HC_MFMA 0        // 1: hidden-space compositing as MFMA (transpose + contract; measured slower)
#endif
#ifndef ST_ABL_NOHEAD
#define ST_ABL_NOHEAD 0
#endif
#ifndef ST_ABL_NORAY
#define ST_ABL_NORAY 0
#endif
#ifndef ST_ABL_NODMA
#define ST_ABL_NODMA 0
#endif
#ifndef ST_ABL_NOITEM
#define ST_ABL_NOITEM 0
#endif
#ifndef ST_ABL_NOTR
#define ST_ABL_NOTR 0
#endif
#ifndef ST_ABL_NOPE
#define ST_ABL_NOPE 0
#endif
#ifndef ST_ABL_NOCODE
#define ST_ABL_NOCODE 0
#endif
#ifndef ST_EPI_BFLY
#define ST_EPI_BFLY 1    // hidden sums of the ray epilogue by a bank-masked DPP butterfly
#endif
#ifndef ST_ABL_NOHSUM
#define ST_ABL_NOHSUM 0  // cost probe: the epilogue's 32 hidden-sum reductions skipped (wrong dino)
#endif
#ifndef ST_ABL_NOHC
#define ST_ABL_NOHC 0
#endif
#ifndef ST_HOIST_W
#define ST_HOIST_W 1        // the code-column weight fragments held in VGPRs (48 of them; 230 in all)
#endif
#ifndef ST_HOIST_SIG
#define ST_HOIST_SIG 1      // the sigma A fragments held in VGPRs as well (16 more: 244 in all)
#endif
#ifndef ST_SIG_VALU
#define ST_SIG_VALU 0       // sigma by v_dot2 on the relu tiles + permlane swaps (1: weights in VGPRs, 2: from LDS) instead of 4 MFMAs
#endif
#ifndef ST_ABL_NOSIG
#define ST_ABL_NOSIG 0
#endif

// diagnostic build only (ST_PROF=1): per-phase s_memtime cycles summed over all waves
#ifndef ST_PROF
#define ST_PROF 0
#endif
#if ST_PROF
__device__ unsigned long long st_prof[32];
#define ST_T(i)                                                  \
    {                                                            \
        const uint64_t _t = __builtin_amdgcn_s_memtime();        \
        pacc[i] += (uint32_t)(_t - tlast);                       \
        tlast = _t;                                              \
    }
extern "C" int sd_tile_prof(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(st_prof), sizeof(st_prof)) != hipSuccess) return -2;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(st_prof), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define ST_T(i)
#endif
#if ST_PROF >= 2  // item sub-phases (each marker also drains LDS: diagnostic only)
#define ST_T2(i) ST_T(i)
#else
#define ST_T2(i)
#endif

#ifndef ST_PREADDR
#define ST_PREADDR 1        // tap LDS addresses written into the records once the tile is staged
#endif
#ifndef ST_EPI_STORES
#define ST_EPI_STORES 1     // per-sample outputs staged in the records, stored per ray (coalesced)
#endif
#ifndef ST_BLEND_DEEP
#define ST_BLEND_DEEP 0     // > 0: tap reads that many blend tiles ahead of the MFMAs
#endif
#ifndef ST_CODE_FIRST
#define ST_CODE_FIRST 0     // 1: positional-code MFMAs before the tap blend (spills)
#endif
#ifndef ST_HEAD_PF
#define ST_HEAD_PF 0        // 0: the DINO head loads its W_dino fragments itself (no prefetch across the ray pass)
#endif
#ifndef ST_COL_EARLY
#define ST_COL_EARLY 0      // 1: the next ray's colour texels blended right after its ray pass (not after item 0)
#endif
#ifndef ST_HEAD_FIRST
#define ST_HEAD_FIRST 0     // 1: the previous group's DINO head at the top of the step (before the ray pass)
#endif
#ifndef ST_SAME_CAM
#define ST_SAME_CAM 1       // colour taps re-use the encoder-view projection when cam_c == cam_f
#endif
#ifndef ST_FASTPROJ
#define ST_FASTPROJ 1       // fused-record projection (0: the two-step reference one)
#endif
#if ST_FASTPROJ
#define ST_GEO sd_point_geo_fast
#define ST_CTAPS sd_color_taps_fast
#else
#define ST_GEO sd_point_geo<true>
#define ST_CTAPS sd_color_taps
#endif

struct st_args {
    sd_render_args a;
    sd_head m;
    int32_t *ovf;           // [0]: overflow count, [1 + i]: overflowed group index
    int32_t ngroups;        // ceil(R / NW)
    int32_t tile_bytes;     // bytes per tile buffer (multiple of 1024)
};

// LDS image (byte offsets)
// the code / sigma A fragments go through LDS only in the diagnostic builds that read them
// there per item; the shipped kernel holds them in VGPRs, loaded from global memory once,
// and gives their 16 KiB to the tile buffers
#ifndef ST_FRAG_LDS_FORCE
#define ST_FRAG_LDS_FORCE 0  // 1: keep the fragment copy in LDS (A/B of the larger tile buffers)
#endif
#define ST_FRAG_LDS (ST_FRAG_LDS_FORCE || !(ST_HOIST_W && ST_HOIST_SIG) || ST_CODE_FIRST || ST_SIG_VALU == 2)
#define ST_L_PE 0                              // [8][64] x 16 B code A fragments (16x16x32)
#define ST_L_PE1 (ST_L_PE + 8 * 64 * 16)      // [8][64] x 8 B code A fragments (16x16x16)
#define ST_L_SIG (ST_L_PE1 + 8 * 64 * 8)      // [4][64] x 16 B sigma A fragments
#define ST_L_BOX (ST_FRAG_LDS ? ST_L_SIG + 4 * 64 * 16 : 0)  // [2][NW waves][2 halves] u32 (min, max) packed
// then, sized by NW (waves = rays per group):
__host__ __device__ constexpr int st_l_hs(int nw) { return ST_L_BOX + 2 * nw * 16; }  // [NW rays][128] 16-bit hidden sums
__host__ __device__ constexpr int st_l_ws(int nw) { return st_l_hs(nw) + nw * 128 * 2; }  // [NW] f32 weight sums
__host__ __device__ constexpr int st_l_ray(int nw) { return st_l_ws(nw) + 16 * 4; }  // [NW waves][2] x 32 B ray words 0..7 (LDS-DMA)
__host__ __device__ constexpr int st_l_rec(int nw) { return st_l_ray(nw) + nw * 2 * 32; }  // records: [NW waves][2][K] x 40 B
static_assert(st_l_rec(8) % 16 == 0 && st_l_rec(12) % 16 == 0, "record area alignment");

__host__ __device__ constexpr int st_rec_bytes(int nw, int K) { return nw * 2 * K * 40; }

// packed u16x2 (x | y << 16) component-wise min / max
// one butterfly level of a 16-lane row sum over two values: lanes of banks MA (groups of 4
// lanes) get a + a(lane - RA), lanes of banks MB get b + b(lane - RB), both into a.  The
// bank-masked DPP add is inline asm (the compiler does not fold a partially masked DPP move
// into its user); s_nop 1 covers the VALU-write -> DPP-read hazard of the sources.
#define ST_BFLY(a, b, RA, RB, MA, MB)                                                         \
    do {                                                                                      \
        asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_ror:" #RA " row_mask:0xf bank_mask:" #MA \
            : "+v"(a));                                                                       \
        asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_ror:" #RB " row_mask:0xf bank_mask:" #MB \
            : "+v"(a) : "v"(b));                                                              \
    } while (0)

__device__ __forceinline__ uint32_t st_min2(uint32_t a, uint32_t b) {
    typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t st_max2(uint32_t a, uint32_t b) {
    typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
// component-wise min / max over each 16-lane row by DPP (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror: every step's sources are inside the row), no LDS round trip
template <bool MAX>
__device__ __forceinline__ uint32_t st_row_red2(uint32_t v) {
#define ST_RSTEP(ctrl)                                                                        \
    {                                                                                         \
        const uint32_t o = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, (ctrl), 0xf, 0xf, false); \
        v = MAX ? st_max2(v, o) : st_min2(v, o);                                              \
    }
    ST_RSTEP(0xB1)
    ST_RSTEP(0x4E)
    ST_RSTEP(0x141)
    ST_RSTEP(0x140)
#undef ST_RSTEP
    return v;
}
// row-reduced value -> wave-uniform reduction of rows [r0, r1]
template <bool MAX>
__device__ __forceinline__ uint32_t st_rows2(uint32_t v, int r0, int r1) {
    uint32_t acc = (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * r0);
    for (int r = r0 + 1; r <= r1; ++r) {
        const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * r);
        acc = MAX ? st_max2(acc, o) : st_min2(acc, o);
    }
    return acc;
}
__device__ __forceinline__ uint32_t st_wave_min2(uint32_t v) { return st_rows2<false>(st_row_red2<false>(v), 0, 3); }
__device__ __forceinline__ uint32_t st_wave_max2(uint32_t v) { return st_rows2<true>(st_row_red2<true>(v), 0, 3); }

// tile pitch (texels per staged row): pitch mod 8 in 2..6, so that the four taps
// n, n + 1, n + pitch, n + pitch + 1 of a sample (288 B = 8 banks apart per texel) land
// on four disjoint 8-bank groups of a transposed read
__device__ __forceinline__ int st_pitch(int tw) {
    const int r = tw & 7;
    return tw + (r == 7 ? 3 : r == 0 ? 2 : r == 1 ? 1 : 0);
}

__device__ __forceinline__ void st_barrier_lds() {
    // wave's LDS writes visible, then the workgroup barrier; vector-memory loads (and
    // LDS-DMA) stay in flight across it
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

typedef __attribute__((address_space(3))) void lds_void;

// LDS-DMA (global_load_lds) as inline asm.  Issued through the builtin, the compiler
// treats every later LDS read as a possible alias of the in-flight DMA and puts an
// s_waitcnt vmcnt(0) in front of it -- the item loop then waits for the next tile's DMA
// at its first record read.  The kernel orders these DMAs itself (s_waitcnt vmcnt(0) +
// barrier before the staged data is read); vector-memory returns are in order, so the
// compiler's own vmcnt waits stay conservative with these extra loads in flight.
// (m0 = LDS destination of lane 0; one wait state between the SALU write and the DMA.)
#ifndef ST_DMA_ASM
#define ST_DMA_ASM 1
#endif
__device__ __forceinline__ void st_dma16(const void *src, uint32_t lds_addr) {
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);  // wave-uniform by construction
    if (!ST_DMA_ASM) {
        __builtin_amdgcn_global_load_lds(src, (lds_void *)(uintptr_t)lds_addr, 16, 0, 0);
        return;
    }
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src), "s"(lds_addr) : "memory");
}
__device__ __forceinline__ void st_dma4(const void *src, uint32_t lds_addr) {
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    if (!ST_DMA_ASM) {
        __builtin_amdgcn_global_load_lds(src, (lds_void *)(uintptr_t)lds_addr, 4, 0, 0);
        return;
    }
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                 :: "v"(src), "s"(lds_addr) : "memory");
}
typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ __forceinline__ uint2 st_tr(uint32_t addr) {
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(uintptr_t)addr);
    return __builtin_bit_cast(uint2, v);
}

// ZIN: depths given (args.z, parity tests) instead of drawn in the kernel.  A template
// parameter, not a branch: with both paths in one body the compiler's wait for the z loads
// also drains the head-weight prefetch on the drawing path.
template <int P, bool ZIN, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4)))
k_render_tile(const st_args sa) {
    constexpr int ST_WAVES = NW;
    constexpr int ST_L_HS = st_l_hs(NW), ST_L_WS = st_l_ws(NW), ST_L_RAY = st_l_ray(NW),
                  ST_L_REC = st_l_rec(NW);
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    typedef typename Tr::Frag4 Frag4;
    typedef typename Tr::E E;
    const sd_render_args &a = sa.a;
    const sd_head &m = sa.m;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
#if ST_PROF
    uint32_t pacc[19] = {};
    uint64_t tlast = __builtin_amdgcn_s_memtime();
#endif
    {
        const uint4 *pe = (const uint4 *)m.w_pe, *sg = (const uint4 *)m.w_sig;
        uint4 *d = (uint4 *)lds;
        if (ST_FRAG_LDS) {
            for (int i = threadIdx.x; i < 12 * SD_WAVE; i += blockDim.x) d[ST_L_PE / 16 + i] = pe[i];
            for (int i = threadIdx.x; i < 4 * SD_WAVE; i += blockDim.x) d[ST_L_SIG / 16 + i] = sg[i];
        }
    }
    const Frag *lf = (const Frag *)lds;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_void *)lds;  // LDS byte address of lds[0]

    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = a.K, nsub = K >> 4;
    const int R = (int)a.R, rps = (int)a.rays_per_sb;
    const int D = m.D, ndt = D >> 4;
    const int Wf = a.Wf, Hf = a.Hf;
    const uint32_t plane_bytes = (uint32_t)Hf * Wf * SD_DH * 2;

    // records: SoA per (wave, buffer): q0 [K] x 16 B | q1 [K] x 16 B | c [K] x 8 B
    //   q0 = {x0 | y0 << 15 | inv_f << 30 | invc << 31, (w00, w01), (w10, w11), r}
    //   q1 = {x, y, z~, z}   c = {g, b}
    const uint32_t rec_base = ST_L_REC + (uint32_t)wave * 2 * K * 40;
    auto rq0 = [&](int buf) { return (uint4 *)(lds + rec_base + buf * K * 40); };
    auto rq1 = [&](int buf) { return (f32x4 *)(lds + rec_base + buf * K * 40 + K * 16); };
    auto rqc = [&](int buf) { return (float2 *)(lds + rec_base + buf * K * 40 + K * 32); };
    const uint32_t tile0 = ST_L_REC + st_rec_bytes(NW, K);
    const int tcap = sa.tile_bytes / ST_TEX;

    // XCD-aware group ranges (workgroups b, b + 8, ... share an XCD, speed only)
    const int NG = sa.ngroups;
    const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
    const int xcd = blockIdx.x % nx, lb = blockIdx.x / nx, nwg = gridDim.x / nx;
    const int glo = (int)((int64_t)NG * xcd / nx), ghi = (int)((int64_t)NG * (xcd + 1) / nx);
    const int gfirst = glo + lb;
    const int nsteps = gfirst < ghi ? (ghi - gfirst + nwg - 1) / nwg : 0;
    __syncthreads();
    if (nsteps == 0) return;  // workgroup-uniform

    const float zstep = (float)(1.0 / (double)K), zend = (float)(1.0 - 1.0 / (double)K);
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;

    // ---- ray pass: lane = sample k = 64 p + lane --------------------------------------
    // ray words 0..7 (origin, direction, near, far) of a later step's ray, fetched by
    // LDS-DMA one step ahead (completed by the step's closing vmcnt(0)), so the ray pass
    // reads them from LDS instead of waiting on scalar loads
    const int nrw = min(a.ray_dim, 8);
    auto ray_fetch = [&](int ray, int slot) {
        if (ray < R && lane < nrw)
            st_dma4(a.rays + (int64_t)ray * a.ray_dim + lane, lds0 + ST_L_RAY + (wave * 2 + slot) * 32);
    };
    const float *rl = nullptr;  // this ray pass's words (set by ray_pass)
    auto load_ray_z = [&](int ray, float zq[2 * ST_MAXP]) {
        float zo[ST_MAXP];
        if (ZIN) {
            const float *zr = a.z + (int64_t)ray * K;
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) zo[p] = zr[min(64 * p + lane, K - 1)];
        } else {
            const float near = rl[6], far = rl[7];
            const uint64_t base = a.z_offset + (uint64_t)ray * (uint64_t)K;
            zo[1] = 0.f;
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) {
                if (64 * p >= K) break;  // wave-uniform: K <= 64 draws one sample per lane
                const int k = min(64 * p + lane, K - 1);
                zo[p] = sd_z_sample(near, far, K, k, sd_uniform(a.z_seed, base + k), zstep, zend,
                                    a.z_lindisp);
            }
        }
#pragma unroll
        for (int p = 0; p < ST_MAXP; ++p) {
            float nx2 = __shfl_down(zo[p], 1, 64);
            const float first_next = p + 1 < ST_MAXP
                ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                      __builtin_bit_cast(int, zo[p + 1 < ST_MAXP ? p + 1 : p]), 0))
                : zo[p];
            if (lane == 63) nx2 = (p + 1 < ST_MAXP && 64 * (p + 1) < K) ? first_next : zo[p];
            zq[2 * p] = zo[p];
            zq[2 * p + 1] = nx2;
        }
    };
    // the colour texel loads of sample k = lane are left in flight (cpend) and finished
    // by ray_col at the end of the item that ran the pass
    ColPend cpend;
    uint32_t cp_x0y0 = 0;
    // tap boxes per half ray: samples [0, kh) and [kh, K), kh = 16 (nsub / 2) -- a group
    // whose whole box does not fit a tile buffer is staged and rendered half by half
    const int kh = 16 * (nsub >> 1);
    auto ray_pass = [&](int ray, int buf, int slot) {
        uint32_t bmin0 = 0xffffffffu, bmax0 = 0u, bmin1 = 0xffffffffu, bmax1 = 0u;
        if (ray < R) {
            // wave-uniform (readfirstlane: the u32 divide runs on the VALU, and a VGPR
            // address would turn the camera-record reads into vector loads)
            const int sbi = __builtin_amdgcn_readfirstlane((int)((unsigned)ray / (unsigned)rps));
            rl = (const float *)(lds + ST_L_RAY + (wave * 2 + slot) * 32);
            // colour view = encoder view (the single-frame render, ids_render = ids_encoder):
            // the host passes the same camera records for both (cam_c == cam_f), so the
            // colour taps are the encoder-view taps at equal resolution (kernel-uniform test)
            const bool same_cam = ST_SAME_CAM && a.cam_c == a.cam_f && a.Wc == Wf && a.Hc == Hf;
            float zq[2 * ST_MAXP];
            load_ray_z(ray, zq);
            ST_T(10);
            const float ox = rl[0], oy = rl[1], oz = rl[2], dx = rl[3], dy = rl[4], dz = rl[5];
            uint4 *r0 = rq0(buf);
            f32x4 *r1 = rq1(buf);
            float2 *rc = rqc(buf);
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) {
                const int k = 64 * p + lane;
                if (64 * p < K && k < K) {
                    const float z0 = zq[2 * p];
                    const float px = ox + z0 * dx, py = oy + z0 * dy, pz = oz + z0 * dz;  // nerf.py:252
                    const PointGeo geo = ST_GEO((sd_cfloat *)(a.cam_f + sbi * SD_CAM_WORDS), px, py, pz,
                                                            Wf, Hf);
                    const uint32_t x0 = (uint32_t)geo.t.x0, y0 = (uint32_t)geo.t.y0;
                    bool ic;
                    Taps tc;
                    if (same_cam) {  // colour view = encoder view: the same projection and taps
                        tc = geo.t;
                        ic = geo.inv_f;
                    } else {
                        tc = ST_CTAPS((sd_cfloat *)(a.cam_c + sbi * SD_CAM_WORDS), a.Wc, a.Hc, px, py, pz, ic);
                    }
                    const uint32_t xy = x0 | (y0 << 15) | (geo.inv_f ? 1u << 30 : 0u) |
                                        (ic ? 1u << 31 : 0u);
                    const uint4 wp = sd_pack_w<P>(geo.t.w00, geo.t.w01, geo.t.w10, geo.t.w11);
                    r1[k] = f32x4{geo.v[0], geo.v[1], geo.v[2], z0};
                    if (p == 0) {
                        sd_color_issue(a.img + (int64_t)sbi * cplane, tc, cpend);
                        cp_x0y0 = xy;
                        r0[k] = uint4{xy, wp.x, wp.y, 0u};  // colour word written by ray_col
                    } else {
                        float col[3];
                        sd_sample_rgb(a.img + (int64_t)sbi * cplane, tc, col);
                        r0[k] = uint4{xy, wp.x, wp.y, __builtin_bit_cast(uint32_t, col[0])};
                        rc[k] = float2{col[1], col[2]};
                    }
                    const uint32_t lo = x0 | (y0 << 16);
                    if (k < kh) {
                        bmin0 = st_min2(bmin0, lo);
                        bmax0 = st_max2(bmax0, lo + 0x00010001u);
                    } else {
                        bmin1 = st_min2(bmin1, lo);
                        bmax1 = st_max2(bmax1, lo + 0x00010001u);
                    }
                }
            }
        }
        ST_T(11);
        if (K == 64) {
            // one sample per lane, halves = lanes [0, 32) and [32, 64): rows 0-1 / 2-3
            const uint32_t mnv = st_row_red2<false>(lane < 32 ? bmin0 : bmin1);
            const uint32_t mxv = st_row_red2<true>(lane < 32 ? bmax0 : bmax1);
            bmin0 = st_rows2<false>(mnv, 0, 1);
            bmax0 = st_rows2<true>(mxv, 0, 1);
            bmin1 = st_rows2<false>(mnv, 2, 3);
            bmax1 = st_rows2<true>(mxv, 2, 3);
        } else {
            bmin0 = st_wave_min2(bmin0);
            bmax0 = st_wave_max2(bmax0);
            bmin1 = st_wave_min2(bmin1);
            bmax1 = st_wave_max2(bmax1);
        }
        ST_T(12);
        if (lane == 0)
            *(uint4 *)(lds + ST_L_BOX + (slot * ST_WAVES + wave) * 16) = uint4{bmin0, bmax0, bmin1, bmax1};
    };
    auto ray_col = [&](int ray, int buf) {
        if (ray < R && lane < K) {
            float col[3];
            sd_color_finish(cpend, col);
            rq0(buf)[lane].w = __builtin_bit_cast(uint32_t, col[0]);
            rqc(buf)[lane] = float2{col[1], col[2]};
        }
    };

    // ---- per-step tile geometry (workgroup-uniform) -----------------------------------
    struct Tile {
        int bx0, by0, pitch, ok, split, ninstr;
    };
    // union of the 8 waves' boxes of slot: which = 0 / 1 (half ray), 2 (whole ray)
    auto box_union = [&](int slot, int which, uint32_t &mn, uint32_t &mx) {
        const uint4 *bx = (const uint4 *)(lds + ST_L_BOX + slot * ST_WAVES * 16);
        mn = 0xffffffffu;
        mx = 0u;
#pragma unroll
        for (int i = 0; i < ST_WAVES; ++i) {
            const uint4 v = bx[i];
            mn = st_min2(mn, which == 0 ? v.x : which == 1 ? v.z : st_min2(v.x, v.z));
            mx = st_max2(mx, which == 0 ? v.y : which == 1 ? v.w : st_max2(v.y, v.w));
        }
        mn = __builtin_amdgcn_readfirstlane(mn);
        mx = __builtin_amdgcn_readfirstlane(mx);
    };
    auto geom = [&](uint32_t mn, uint32_t mx) {
        Tile t;
        t.bx0 = (int)(mn & 0xffffu);
        t.by0 = (int)(mn >> 16);
        const int tw = (int)(mx & 0xffffu) - t.bx0 + 1, th = (int)(mx >> 16) - t.by0 + 1;
        t.pitch = tw > 0 ? st_pitch(tw) : 1;
        t.ninstr = (th * t.pitch * ST_TEXQ + 63) >> 6;  // 1-KiB DMA instructions
        t.ok = (mn != 0xffffffffu) && tw > 0 && th > 0 && t.ninstr * 1024 <= sa.tile_bytes;
        t.split = 0;
        return t;
    };
    // this wave's share of the LDS-DMA of tile t's texels into tile buffer tb
    auto dma = [&](const Tile &t, int tb, int sbi) {
        const uint8_t *plane = (const uint8_t *)a.grid + (int64_t)sbi * plane_bytes;
        const float inv_pitch = 1.f / (float)t.pitch;
        const uint32_t dst0 = tile0 + (uint32_t)tb * (uint32_t)sa.tile_bytes;
        for (int i = wave; i < t.ninstr; i += ST_WAVES) {
            const uint32_t ci = (uint32_t)i * 64u + (uint32_t)lane;
            const uint32_t n = __umulhi(ci, 238609295u);  // ci / 18
            const uint32_t part = ci - 18u * n;
            const int ty = (int)(((float)n + 0.5f) * inv_pitch);
            const int tx = (int)n - ty * t.pitch;
            const int sx = min(max(t.bx0 + tx, 0), Wf - 1), sy = min(max(t.by0 + ty, 0), Hf - 1);
            const uint8_t *src = plane + ((int64_t)sy * Wf + sx) * 256 + (part < 16u ? part : 0u) * 16u;
            if (!ST_ABL_NODMA) st_dma16(src, lds0 + dst0 + (uint32_t)i * 1024u);
        }
    };
    // geometry of slot's group for tile buffer tb, DMA issued: the whole box if it fits,
    // else (nsub >= 2) the first half's box when both halves fit (split = 1: the second
    // half is staged mid-step), else the group goes to the overflow list (ok = 0)
    auto stage = [&](int slot, int tb, int grp, int sbi) {
        uint32_t mn, mx;
        box_union(slot, 2, mn, mx);
        Tile t = geom(mn, mx);
        if (mn == 0xffffffffu) return t;  // no valid ray in the group
        if (!t.ok && nsub >= 2 && !ST_PIPE) {
            uint32_t mn0, mx0, mn1, mx1;
            box_union(slot, 0, mn0, mx0);
            box_union(slot, 1, mn1, mx1);
            const Tile h0 = geom(mn0, mx0), h1 = geom(mn1, mx1);
            if (h0.ok && h1.ok) {
                t = h0;
                t.split = 1;
            }
        }
        if (!t.ok) {
            if (wave == 0 && lane == 0) {  // the group's rays as NW / SD_LIST_BLK list blocks
                const int i = atomicAdd(sa.ovf, NW / SD_LIST_BLK);
                for (int b = 0; b < NW / SD_LIST_BLK; ++b)
                    sa.ovf[1 + i + b] = grp * (NW / SD_LIST_BLK) + b;
            }
            return t;
        }
        dma(t, tb, sbi);
        return t;
    };

    // once a group's tile geometry is known (after stage), each wave rewrites its ray's
    // record words q0.x = {x0 | y0 << 15 | flags << 30} as {LDS byte address of tap (x0, y0)
    // in tile buffer tb | flags << 30}: an item then reads the 4 tap bases it needs with
    // two ds_read2_b32 instead of computing its own and exchanging them by ds_bpermute (a
    // chain of dependent LDS round trips at the head of every item).  Split groups: the
    // second half ray's samples get the second half's geometry.
    auto tap_addrs = [&](int rbuf, int tb, const Tile &t, int ray_) {
        if (!ST_PREADDR || !t.ok || ray_ >= R) return;
        Tile t2 = t;
        if (t.split) {
            uint32_t mn1, mx1;
            box_union(rbuf, 1, mn1, mx1);
            t2 = geom(mn1, mx1);
        }
        const uint32_t tbase = lds0 + tile0 + (uint32_t)tb * (uint32_t)sa.tile_bytes;
        uint32_t *w = (uint32_t *)rq0(rbuf);
#pragma unroll
        for (int p = 0; p < ST_MAXP; ++p) {
            const int k = 64 * p + lane;
            if (64 * p < K && k < K) {
                const uint32_t xy = w[4 * k];
                const Tile &tt = (t.split && k >= kh) ? t2 : t;
                const int x0 = (int)(xy & 0x7fffu), y0 = (int)((xy >> 15) & 0x7fffu);
                const uint32_t ad = tbase + (uint32_t)(((y0 - tt.by0) * tt.pitch + (x0 - tt.bx0)) * ST_TEX);
                w[4 * k] = ad | (xy & 0xc0000000u);
            }
        }
    };

    // ---- DINO head of one group (hsum of its 8 rays in LDS) ---------------------------
    // W_dino fragments of the wave's first head tile (dt = wave), loaded one phase ahead
    Frag Wh[4];
    auto head_prefetch = [&]() {
        if (ST_HEAD_PF && wave < ndt) {
            const Frag *wo = (const Frag *)m.w_out + (int64_t)wave * 4 * SD_WAVE + lane;
#pragma unroll
            for (int s = 0; s < 4; ++s) Wh[s] = wo[s * SD_WAVE];
        }
    };
    auto head = [&](int grp) {
        if (wave >= ndt) return;
        const int slot = j < NW ? j : 0;  // B columns j >= NW: not stored
        Frag Bh[4];
        const uint8_t *hs = lds + ST_L_HS + slot * 256;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint2 lo = *(const uint2 *)(hs + (32 * s + 4 * g) * 2);
            const uint2 hi = *(const uint2 *)(hs + (32 * s + 16 + 4 * g) * 2);
            Bh[s] = __builtin_bit_cast(Frag, uint4{lo.x, lo.y, hi.x, hi.y});
        }
        const float ws = *(const float *)(lds + ST_L_WS + slot * 4);
        const int ray = NW * grp + j;
        const bool store = j < NW && ray < R;
        for (int dt = wave; dt < ndt; dt += ST_WAVES) {
            const Frag *wo = (const Frag *)m.w_out + (int64_t)dt * 4 * SD_WAVE + lane;
            f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) o = Tr::mma(ST_HEAD_PF && dt == wave ? Wh[s] : wo[s * SD_WAVE], Bh[s], o);
            // rows 4 g + r of tile dt = dims 16 dt + 4 g + r, column j = ray slot
            const int dim = 16 * dt + 4 * g;
            const f32x4 bd = *(const f32x4 *)(m.b_dino + dim);
            f32x4 res;
#pragma unroll
            for (int r = 0; r < 4; ++r) res[r] = o[r] + ws * bd[r];
            if (store) *(f32x4 *)(a.dino + (int64_t)ray * a.ld_dino + dim) = res;
        }
    };

    // per-lane constant part of the transposed-read addresses: tap q = (lane & 15) >> 2
    // of a sample, columns 4 p .. 4 p + 3
    const int tq = (lane & 15) >> 2, tp = lane & 3;
    // B operand masks: lane (j, g) carries sample j's weights in K-chunk j >> 3 iff
    // ((j & 7) >> 1) == g, at elements 4 (j & 1) .. + 3
    const bool bsel = ((j & 7) >> 1) == g;
    const bool bc0 = bsel && (j >> 3) == 0, bc1 = bsel && (j >> 3) == 1;
    const bool br1 = (j & 1) != 0;
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    // ST_HOIST_W: this lane's code-column weight fragments held in VGPRs for the whole kernel
    Frag wpe[8];
    Frag4 wpe1[8];
    if (ST_HOIST_W) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            wpe[t] = ((const Frag *)m.w_pe)[t * SD_WAVE + lane];
            wpe1[t] = ((const Frag4 *)((const uint8_t *)m.w_pe + 8 * SD_WAVE * 16))[t * SD_WAVE + lane];
        }
    }
#if ST_SIG_VALU == 1 || ST_HOIST_SIG
    // sigma weights of this lane's relu elements (every row of the sigma A fragment holds
    // W_out[0] at hid(s, g, e), mlp_pack.py), kept in registers
    uint4 wsig_r[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) wsig_r[s2] = ((const uint4 *)m.w_sig)[s2 * SD_WAVE + lane];
#endif
    // identity B operand of the 16x16x16 transposition (lane (n, g): rows 4 g + e)
    const Frag4 Iden = __builtin_bit_cast(
        Frag4, uint2{sd_pack2<E>(4 * g == j ? 1.f : 0.f, 4 * g + 1 == j ? 1.f : 0.f),
                     sd_pack2<E>(4 * g + 2 == j ? 1.f : 0.f, 4 * g + 3 == j ? 1.f : 0.f)});

    // ---- prologue: records + tile of step 0 -------------------------------------------
    int grp = gfirst;
    int ray = NW * grp + wave;
    int sbi = __builtin_amdgcn_readfirstlane((int)((unsigned)min(NW * grp, R - 1) / (unsigned)rps));
    ray_fetch(ray, 0);
    ray_fetch(NW * (grp + nwg) + wave, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ray_pass(ray, 0, 0);
    ray_col(ray, 0);
    st_barrier_lds();
    Tile cur = stage(0, 0, grp, sbi);
    tap_addrs(0, 0, cur, ray);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    int prev_grp = -1, prev_ok = 0;
#if ST_PROF
#pragma unroll
    for (int i = 0; i < 19; ++i) pacc[i] = 0;
    tlast = __builtin_amdgcn_s_memtime();
#endif
    for (int n = 0; n < nsteps; ++n) {
        const int buf = n & 1;
        const bool has_next = n + 1 < nsteps;
        const int ngrp = grp + nwg;
        const int nray = NW * ngrp + wave;
        const int nsbi = has_next ? __builtin_amdgcn_readfirstlane((int)((unsigned)min(NW * ngrp, R - 1) / (unsigned)rps)) : 0;
        const bool active = cur.ok && ray < R;
        const uint32_t tileb = lds0 + tile0 + (uint32_t)buf * (uint32_t)sa.tile_bytes;
        uint32_t lane_off = (uint32_t)((tq & 1) + (tq >> 1) * cur.pitch) * ST_TEX + 8u * (uint32_t)tp;

        float Tc = 1.f, dpart = 0.f, wpart = 0.f, cpart[3] = {0.f, 0.f, 0.f};
        f32x4 hacc[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) hacc[t] = zero4;

        // An item is split in two so that consecutive items overlap (software pipeline):
        // A = records, taps, MFMA MLP, sigma, alpha, local transmittance scan;
        // B = weights with the carried transmittance, compositing sums, per-sample outputs.
        struct IState {
            Frag X[4];
            float alpha, excl, tmul, zk, col[3];
            uint32_t flags;  // bit 0: outside the encoder frustum, bit 1: outside the render view
        };
        auto itemA = [&](int sub, IState &st) {
            const int k = sub * 16 + j;
            const uint4 q0 = rq0(buf)[k];
            const f32x4 q1 = rq1(buf)[k];
            const float2 cgb = rqc(buf)[k];
            const float znext = k + 1 < K ? rq1(buf)[k + 1][3] : 0.f;
            const uint32_t xy = q0.x;
            st.flags = ((xy >> 30) & 1u) | ((xy >> 30) & 2u);
            const float v[3] = {q1[0], q1[1], q1[2]};
            st.zk = q1[3];
            const float delta = k + 1 < K ? znext - st.zk : 1e10f;
            st.col[0] = __builtin_bit_cast(float, q0.w);
            st.col[1] = cgb.x;
            st.col[2] = cgb.y;
            uint32_t base[2][2];
            if (ST_PREADDR) {
                // tap bases of samples 8 c + 2 g + r, written by tap_addrs
                const uint32_t *aw = (const uint32_t *)rq0(buf) + 4 * (sub * 16 + 2 * g);
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int r = 0; r < 2; ++r) base[c][r] = (aw[4 * (8 * c + r)] & 0x3ffffu) + lane_off;
            } else {
                // this lane's sample: LDS byte address of its tap (x0, y0)
                const int x0 = (int)(xy & 0x7fffu), y0 = (int)((xy >> 15) & 0x7fffu);
                const int nb = (int)tileb + ((y0 - cur.by0) * cur.pitch + (x0 - cur.bx0)) * ST_TEX;
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int r = 0; r < 2; ++r)
                        base[c][r] = (uint32_t)__builtin_amdgcn_ds_bpermute((8 * c + 2 * g + r) << 2, nb) +
                                     lane_off;
            }
            // block-diagonal weight fragments of the two K-chunks
            const uint32_t w01 = q0.y, w23 = q0.z;
            ST_T2(13);
            const uint4 b0 = {bc0 && !br1 ? w01 : 0u, bc0 && !br1 ? w23 : 0u,
                              bc0 && br1 ? w01 : 0u, bc0 && br1 ? w23 : 0u};
            const uint4 b1 = {bc1 && !br1 ? w01 : 0u, bc1 && !br1 ? w23 : 0u,
                              bc1 && br1 ? w01 : 0u, bc1 && br1 ? w23 : 0u};
            const Frag B0 = __builtin_bit_cast(Frag, b0), B1 = __builtin_bit_cast(Frag, b1);
            f32x4 acc[8];
#if ST_CODE_FIRST
            // code columns first: they need only the record, so the tap reads' latency
            // overlaps the code evaluation and its MFMAs
            ST_T2(14);
            // positional-code columns
            const int lo = ST_HOIST_W ? 0 : sd_opaque0();
            const Frag *lw = lf + lo;
            {
                Frag f0;
                Frag4 f1;
#if ST_ABL_NOPE
                for (int e = 0; e < 8; ++e) f0[e] = (E)v[e % 3];
                f1 = __builtin_bit_cast(Frag4, uint2{__builtin_bit_cast(uint32_t, v[0]), 0u});
#else
                sd_code_frags<Frag, Frag4, E>(v, g, f0, f1);
#endif
                const Frag4 *lw1 = (const Frag4 *)(lds + ST_L_PE1) + lo;
                // all 16x16x32 steps first, then the 16x16x16 ones: a 16x16x16 MFMA whose
                // accumulator input is the result of the directly preceding 16x16x32 MFMA
                // read a stale accumulator (hipcc 7.2, gfx950, VGPR-form accumulators)
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (!ST_ABL_NOCODE || t == 0)
                        acc[t] = Tr::mma(lw[ST_L_PE / 16 + t * SD_WAVE + lane], f0, ST_CODE_FIRST ? zero4 : acc[t]);
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (!ST_ABL_NOCODE || t == 0)
                        acc[t] = Tr::mma16(lw1[t * SD_WAVE + lane], f1, acc[t]);
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {
#if ST_ABL_NOTR
                const uint2 a00 = {base[0][0] + t, base[0][1]}, a01 = {base[1][0], base[1][1] + t};
                const uint2 a10 = a01, a11 = a00;
#else
                const uint2 a00 = st_tr(base[0][0] + 32u * t), a01 = st_tr(base[0][1] + 32u * t);
                const uint2 a10 = st_tr(base[1][0] + 32u * t), a11 = st_tr(base[1][1] + 32u * t);
#endif
                const Frag A0 = __builtin_bit_cast(Frag, uint4{a00.x, a00.y, a01.x, a01.y});
                const Frag A1 = __builtin_bit_cast(Frag, uint4{a10.x, a10.y, a11.x, a11.y});
                acc[t] = Tr::mma(A0, B0, ST_CODE_FIRST ? acc[t] : zero4);
                acc[t] = Tr::mma(A1, B1, acc[t]);
            }
            ST_T2(14);
#else
#if ST_BLEND_DEEP
            // the tap reads run ST_BLEND_DEEP tiles ahead of the blend MFMAs (one LDS latency
            // per item instead of one per tile)
            uint2 tv[8][4];
#pragma unroll
            for (int t = 0; t < ST_BLEND_DEEP; ++t) {
                tv[t][0] = st_tr(base[0][0] + 32u * t); tv[t][1] = st_tr(base[0][1] + 32u * t);
                tv[t][2] = st_tr(base[1][0] + 32u * t); tv[t][3] = st_tr(base[1][1] + 32u * t);
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them)
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (t + ST_BLEND_DEEP < 8) {
                    const int u = t + ST_BLEND_DEEP;
                    tv[u][0] = st_tr(base[0][0] + 32u * u); tv[u][1] = st_tr(base[0][1] + 32u * u);
                    tv[u][2] = st_tr(base[1][0] + 32u * u); tv[u][3] = st_tr(base[1][1] + 32u * u);
                }
                __builtin_amdgcn_sched_barrier(0);
                const Frag A0 = __builtin_bit_cast(Frag, uint4{tv[t][0].x, tv[t][0].y, tv[t][1].x, tv[t][1].y});
                const Frag A1 = __builtin_bit_cast(Frag, uint4{tv[t][2].x, tv[t][2].y, tv[t][3].x, tv[t][3].y});
                acc[t] = Tr::mma(A0, B0, zero4);
                acc[t] = Tr::mma(A1, B1, acc[t]);
            }
#else
#pragma unroll
            for (int t = 0; t < 8; ++t) {
#if ST_ABL_NOTR
                const uint2 a00 = {base[0][0] + t, base[0][1]}, a01 = {base[1][0], base[1][1] + t};
                const uint2 a10 = a01, a11 = a00;
#else
                const uint2 a00 = st_tr(base[0][0] + 32u * t), a01 = st_tr(base[0][1] + 32u * t);
                const uint2 a10 = st_tr(base[1][0] + 32u * t), a11 = st_tr(base[1][1] + 32u * t);
#endif
                const Frag A0 = __builtin_bit_cast(Frag, uint4{a00.x, a00.y, a01.x, a01.y});
                const Frag A1 = __builtin_bit_cast(Frag, uint4{a10.x, a10.y, a11.x, a11.y});
                acc[t] = Tr::mma(A0, B0, zero4);
                acc[t] = Tr::mma(A1, B1, acc[t]);
            }
#endif
            ST_T2(14);
            // positional-code columns
            const int lo = ST_HOIST_W ? 0 : sd_opaque0();
            const Frag *lw = lf + lo;
            {
                Frag f0;
                Frag4 f1;
#if ST_ABL_NOPE
                for (int e = 0; e < 8; ++e) f0[e] = (E)v[e % 3];
                f1 = __builtin_bit_cast(Frag4, uint2{__builtin_bit_cast(uint32_t, v[0]), 0u});
#else
                sd_code_frags<Frag, Frag4, E>(v, g, f0, f1);
#endif
                const Frag4 *lw1 = (const Frag4 *)(lds + ST_L_PE1) + lo;
                // all 16x16x32 steps first, then the 16x16x16 ones: a 16x16x16 MFMA whose
                // accumulator input is the result of the directly preceding 16x16x32 MFMA
                // read a stale accumulator (hipcc 7.2, gfx950, VGPR-form accumulators)
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (!ST_ABL_NOCODE || t == 0)
                        acc[t] = Tr::mma(ST_HOIST_W ? wpe[t] : lw[ST_L_PE / 16 + t * SD_WAVE + lane], f0, acc[t]);
#pragma unroll
                for (int t = 0; t < 8; ++t)
                    if (!ST_ABL_NOCODE || t == 0)
                        acc[t] = Tr::mma16(ST_HOIST_W ? wpe1[t] : lw1[t * SD_WAVE + lane], f1, acc[t]);
            }
#endif
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 u = {sd_relu2(sd_pack2<E>(acc[2 * s2][0], acc[2 * s2][1])),
                                 sd_relu2(sd_pack2<E>(acc[2 * s2][2], acc[2 * s2][3])),
                                 sd_relu2(sd_pack2<E>(acc[2 * s2 + 1][0], acc[2 * s2 + 1][1])),
                                 sd_relu2(sd_pack2<E>(acc[2 * s2 + 1][2], acc[2 * s2 + 1][3]))};
                st.X[s2] = __builtin_bit_cast(Frag, u);
            }
#if ST_ABL_NOSIG
            const float sigma = __builtin_bit_cast(float, __builtin_bit_cast(uint4, st.X[0]).x & 0x3fffffffu) + m.b_sigma;
#else
            ST_T2(15);
#if ST_SIG_VALU
            // sigma = sum_h W_out[0][h] relu(h): this lane's 32 hidden by v_dot2 (4 chains),
            // then the sum over the 4 lane groups g (rows) by two permlane swaps -- every
            // lane of column j ends with sample j's sigma, as from the MFMA
            float sp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 x4 = __builtin_bit_cast(uint4, st.X[s2]);
#if ST_SIG_VALU == 1
                const uint4 w4 = wsig_r[s2];
#else
                const uint4 w4 = *(const uint4 *)(lds + ST_L_SIG + ((s2 + lo) * SD_WAVE + lane) * 16);
#endif
                sp[0] = Tr::dot2(x4.x, w4.x, sp[0]);
                sp[1] = Tr::dot2(x4.y, w4.y, sp[1]);
                sp[2] = Tr::dot2(x4.z, w4.z, sp[2]);
                sp[3] = Tr::dot2(x4.w, w4.w, sp[3]);
            }
            float sa = (sp[0] + sp[1]) + (sp[2] + sp[3]), sb = sa;
            asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(sa), "+v"(sb));
            float sc = sa + sb, sd = sc;
            asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(sc), "+v"(sd));
            const float sv = (sc + sd) + m.b_sigma;
#else
            f32x4 sg = zero4;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2)
                sg = Tr::mma(ST_HOIST_SIG ? __builtin_bit_cast(Frag, wsig_r[s2]) : lw[ST_L_SIG / 16 + s2 * SD_WAVE + lane],
                             st.X[s2], sg);
            const float sv = sg[0] + m.b_sigma;
#endif
            const float sigma = sd_softplus_fast(sv);
#endif
            // alpha compositing (nerf.py:376-389)
            float alpha = 1.f - __expf(-fabsf(delta) * fmaxf(sigma, 0.f));
            if (a.hard_alpha_cap && k == K - 1) alpha = 1.f;
            const float incl = sd_scan_mul16((1.f - alpha) + 1e-10f);
            st.alpha = alpha;
            st.excl = SD_DPP1(incl, 0x111);
            st.tmul = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 15));
            ST_T2(16);
        };
        auto itemB = [&](int sub, const IState &st) {
            const int k = sub * 16 + j;
            const float w = st.alpha * (Tc * st.excl);
            Tc *= st.tmul;
            dpart += w * st.zk;
            wpart += w;
            cpart[0] += w * st.col[0];
            cpart[1] += w * st.col[1];
            cpart[2] += w * st.col[2];
#if !ST_HC_MFMA
            const uint32_t wl = sd_pack2<E>(w, 0.f), wh = sd_pack2<E>(0.f, w);
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 u = __builtin_bit_cast(uint4, st.X[s2]);
                const uint32_t d4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int t = 2 * s2 + (q >> 1), r = 2 * (q & 1);
                    hacc[t][r] = Tr::dot2(d4[q], wl, hacc[t][r]);
                    hacc[t][r + 1] = Tr::dot2(d4[q], wh, hacc[t][r + 1]);
                }
            }
#else
            // hidden-space compositing hc[t] += sum_k w_k relu(h_k) as MFMA over the item's
            // 16 samples.  The MLP tiles hold sample j on the lane axis (lane (j, g):
            // hidden 16 t + 4 g + r), but an MFMA contracts along the lane-group axis, so
            // each relu tile is first transposed by an MFMA with the identity (exact), then
            // contracted with the weights: A[m][k] = w_k on every row (samples 4 g + e
            // gathered by ds_bpermute), B[k][n] = relu(h_k)[16 t + n].
            const int wsrc = g << 4;  // ds_bpermute byte address of lane 4 g (sample 4 g)
            const float w0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(wsrc + 0, __builtin_bit_cast(int, w)));
            const float w1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(wsrc + 4, __builtin_bit_cast(int, w)));
            const float w2 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(wsrc + 8, __builtin_bit_cast(int, w)));
            const float w3 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(wsrc + 12, __builtin_bit_cast(int, w)));
            const Frag4 Aw = __builtin_bit_cast(Frag4, uint2{sd_pack2<E>(w0, w1), sd_pack2<E>(w2, w3)});
            ST_T2(17);
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 u = __builtin_bit_cast(uint4, st.X[s2]);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int t = 2 * s2 + h;
                    if (ST_ABL_NOHC && t) continue;
                    const Frag4 xa = __builtin_bit_cast(Frag4, h ? uint2{u.z, u.w} : uint2{u.x, u.y});
                    const f32x4 xt = Tr::mma16(xa, Iden, zero4);
                    const Frag4 xb = __builtin_bit_cast(Frag4, uint2{sd_pack2<E>(xt[0], xt[1]),
                                                                     sd_pack2<E>(xt[2], xt[3])});
                    hacc[t] = Tr::mma16(Aw, xb, hacc[t]);
                }
            }
#endif
            ST_T2(18);
#if ST_EPI_STORES
            // weight and alpha into the sample's record (q1.x / .y are dead once itemA has
            // read the point); the ray epilogue stores every per-sample output coalesced
            if (g == 0) *(float2 *)&rq1(buf)[k] = float2{w, st.alpha};
#else
            const int64_t rk = (int64_t)ray * K;
            if (g == 0) {
                if (a.weights) (a.weights + rk)[k] = w;
                if (a.alphas) (a.alphas + rk)[k] = st.alpha;
                if (a.invalid_f) (a.invalid_f + rk)[k] = (st.flags & 1u) ? 1 : 0;
                if (a.invalid) (a.invalid + rk)[k] = st.flags ? 1.f : 0.f;
                if (a.rgb_samps) {
                    float *rsp = a.rgb_samps + (rk + k) * 3;
                    rsp[0] = st.col[0]; rsp[1] = st.col[1]; rsp[2] = st.col[2];
                }
            }
#endif
        };

        // item 0 with the next ray's pass and the previous group's head
        if (ST_HEAD_FIRST && prev_ok && !ST_ABL_NOHEAD) head(prev_grp);
        if (!ST_HEAD_FIRST && prev_ok && !ST_ABL_NOHEAD) head_prefetch();
        if (has_next && (!ST_ABL_NORAY || n == 0)) ray_pass(nray, buf ^ 1, buf ^ 1);
        if (ST_COL_EARLY && has_next && (!ST_ABL_NORAY || n == 0)) ray_col(nray, buf ^ 1);
        ST_T(0);
        if (!ST_HEAD_FIRST && prev_ok && !ST_ABL_NOHEAD) head(prev_grp);
        ST_T(1);
        IState s0, s1;
        if (active && !ST_ABL_NOITEM) itemA(0, s0);
        ST_T(2);
        if (!ST_COL_EARLY && has_next && (!ST_ABL_NORAY || n == 0)) ray_col(nray, buf ^ 1);
        ST_T(3);
        st_barrier_lds();  // X: next boxes visible; the head has read the hsum area
        ST_T(4);
        Tile nxt = {0, 0, 1, 0, 0, 0};
        if (has_next) {
            nxt = stage(buf ^ 1, buf ^ 1, ngrp, nsbi);
            tap_addrs(buf ^ 1, buf ^ 1, nxt, nray);
        }
        ST_T(5);
#if ST_PIPE
        if (active && !ST_ABL_NOITEM) {
            // items 1 .. nsub-1, item i + 1's A beside item i's B (ping-pong states)
            int sub = 1;
            for (; sub + 1 < nsub; sub += 2) {
                itemA(sub, s1);
                itemB(sub - 1, s0);
                itemA(sub + 1, s0);
                itemB(sub, s1);
            }
            if (sub < nsub) {
                itemA(sub, s1);
                itemB(sub - 1, s0);
                itemB(sub, s1);
            } else {
                itemB(sub - 1, s0);
            }
        }
#else
        // split group: items of the first half ray from the current tile, then the second
        // half's box is staged into the same buffer (workgroup-uniform branch, taken by
        // every wave: it holds barriers).  One item loop for both cases keeps the kernel
        // small (a second inlined copy of the items measured slower).
        const int nfirst = cur.split ? (nsub >> 1) : nsub;
        for (int sub = 0; sub < nsub; ++sub) {
            if (sub == nfirst) {
                st_barrier_lds();  // every wave is done with the first half's taps
                uint32_t mn1, mx1;
                box_union(buf, 1, mn1, mx1);
                cur = geom(mn1, mx1);  // fits: checked when the split was chosen
                dma(cur, buf, sbi);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_barrier_lds();
                lane_off = (uint32_t)((tq & 1) + (tq >> 1) * cur.pitch) * ST_TEX + 8u * (uint32_t)tp;
            }
            if (active && !ST_ABL_NOITEM) {
                if (sub) itemA(sub, s0);
                itemB(sub, s0);
            }
        }
#endif
        ST_T(6);
        if (active) {
            // ray epilogue: sums over the 16 sample lanes of every row
            const float dsum = sd_rowsum16(dpart), wsum = sd_rowsum16(wpart);
            const float c0s = sd_rowsum16(cpart[0]), c1s = sd_rowsum16(cpart[1]),
                        c2s = sd_rowsum16(cpart[2]);
#if ST_HC_MFMA
            // hacc[t]: lane (n, g) holds hidden 16 t + n (every row alike)
            uint16_t *hs = (uint16_t *)(lds + ST_L_HS + wave * 256);
            if (g == 0) {
#pragma unroll
                for (int t = 0; t < 8; ++t) hs[16 * t + j] = Tr::bits(hacc[t][0]);
            }
#else
            uint8_t *hs = lds + ST_L_HS + wave * 256;
#if ST_EPI_BFLY
            if (!ST_ABL_NOHSUM) {
                // the 32 hidden sums q = 4 t + r reduced over the 16 sample lanes of the row
                // as a butterfly (64 VALU ops instead of 32 x 4): bank-masked DPP halves the
                // live values at the first two levels, quad permutes finish -- lane bank b
                // then holds q = i + 8 b, i = 0..7 (hidden 16 (2 b + (i >> 2)) + 4 g + (i & 3))
                float v[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    v[i] = hacc[i >> 2][i & 3];
                    ST_BFLY(v[i], hacc[(i + 16) >> 2][i & 3], 8, 8, 0x3, 0xc);
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) ST_BFLY(v[i], v[i + 8], 12, 4, 0x5, 0xa);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    v[i] += SD_DPP0(v[i], 0xb1);  // quad_perm [1, 0, 3, 2]
                    v[i] += SD_DPP0(v[i], 0x4e);  // quad_perm [2, 3, 0, 1]
                }
                if ((j & 3) == 0) {
                    const int b = j >> 2;
                    *(uint2 *)(hs + (32 * b + 4 * g) * 2) =
                        uint2{sd_pack2<E>(v[0], v[1]), sd_pack2<E>(v[2], v[3])};
                    *(uint2 *)(hs + (32 * b + 16 + 4 * g) * 2) =
                        uint2{sd_pack2<E>(v[4], v[5]), sd_pack2<E>(v[6], v[7])};
                }
            }
#else
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                f32x4 vsum;
#pragma unroll
                for (int r = 0; r < 4; ++r) vsum[r] = ST_ABL_NOHSUM ? hacc[t][r] : sd_rowsum16(hacc[t][r]);
                // hidden 16 t + 4 g + r
                if (j == 0)
                    *(uint2 *)(hs + (16 * t + 4 * g) * 2) =
                        uint2{sd_pack2<E>(vsum[0], vsum[1]), sd_pack2<E>(vsum[2], vsum[3])};
            }
#endif
#endif
#if ST_EPI_STORES
            {
                // per-sample outputs, lane = sample (one coalesced store per array)
                const int64_t rk = (int64_t)ray * K;
#pragma unroll
                for (int p = 0; p < ST_MAXP; ++p) {
                    const int k = 64 * p + lane;
                    if (64 * p < K && k < K) {
                        const f32x4 q1v = rq1(buf)[k];
                        const uint4 q0v = rq0(buf)[k];
                        const uint32_t fl = q0v.x >> 30;
                        if (a.weights) a.weights[rk + k] = q1v[0];
                        if (a.alphas) a.alphas[rk + k] = q1v[1];
                        if (a.invalid_f) a.invalid_f[rk + k] = (uint8_t)(fl & 1u);
                        if (a.invalid) a.invalid[rk + k] = fl ? 1.f : 0.f;
                        if (a.rgb_samps) {
                            const float2 cgb = rqc(buf)[k];
                            float *rsp = a.rgb_samps + (rk + k) * 3;
                            rsp[0] = __builtin_bit_cast(float, q0v.w); rsp[1] = cgb.x; rsp[2] = cgb.y;
                        }
                    }
                }
            }
#endif
            if (lane == 0) {
                *(float *)(lds + ST_L_WS + wave * 4) = wsum;
                a.depth[(int64_t)ray * a.ld_depth] = dsum;
                float *rp = a.rgb + (int64_t)ray * a.ld_rgb;
                rp[0] = c0s; rp[1] = c1s; rp[2] = c2s;
            }
        }
        ST_T(7);
        prev_grp = grp;
        prev_ok = cur.ok;
        grp = ngrp;
        ray = nray;
        sbi = nsbi;
        cur = nxt;
        if (n + 2 < nsteps) ray_fetch(NW * (ngrp + nwg) + wave, buf);  // ray of step n + 2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
        ST_T(8);
        st_barrier_lds();  // Y: next tile complete; hsum of this group written
        ST_T(9);
    }
    if (prev_ok) {
        head_prefetch();
        head(prev_grp);
    }
#if ST_PROF
    if (lane < 19) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 19; ++i) v = lane == i ? pacc[i] : v;
        atomicAdd(&st_prof[lane], (unsigned long long)v);
    }
    if (lane == 0) atomicAdd(&st_prof[31], 1ull);
#endif
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int sd_check_last(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error(hipGetErrorString(e));
        (void)what;
        return -2;
    }
    return 0;
}

static int st_nw(int K) { return K <= 64 ? ST_NW_SMALLK : 8; }

static int st_tile_bytes(int K) {
    const int nw = st_nw(K);
    const int fixed = st_l_rec(nw) + st_rec_bytes(nw, K);
    const int avail = 160 * 1024 - fixed;
    return ((avail / 2) / 1024) * 1024;
}

// Can the tile kernel take this render?  (colour in exactly one render view, batches of
// whole groups, K <= 128, room for one tile buffer pair.)
extern "C" int sd_render_tile_ok(const sd_render_args *a, const sd_head *m) {
    return a->nv == 1 && a->K % 16 == 0 && a->K <= 128 && a->rays_per_sb % st_nw(a->K) == 0 &&
           m->D % 16 == 0 && m->D <= 512 && a->Wf < 32768 && a->Hf < 32768 &&
           st_tile_bytes(a->K) >= 16 * 1024;
}

// Launch; ovf: device int32 [1 + ceil(R/8)] zeroed at [0] by this call.
extern "C" int sd_render_tile_launch(const sd_render_args *a, const sd_head *m, int32_t *ovf,
                                     void *stream) {
    hipStream_t s = (hipStream_t)stream;
    st_args sa;
    sa.a = *a;
    sa.m = *m;
    sa.ovf = ovf;
    const int nw = st_nw(a->K);
    sa.ngroups = (int)((a->R + nw - 1) / nw);
    sa.tile_bytes = st_tile_bytes(a->K);
    const int lds_bytes = st_l_rec(nw) + st_rec_bytes(nw, a->K) + 2 * sa.tile_bytes;
    if (hipMemsetAsync(ovf, 0, sizeof(int32_t), s) != hipSuccess) {
        sd_set_error("sd_render_proj: overflow counter reset failed");
        return -2;
    }
    int ncu = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        ncu = 256;
    auto go = [&](auto kern) {
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
        hipLaunchKernelGGL(kern, dim3((unsigned)ncu), dim3(64 * nw), lds_bytes, s, sa);
    };
    const bool zin = a->z != nullptr;
#define ST_GO(NWV)                                                                              \
    if (m->dtype == SD_F16) {                                                                   \
        if (zin) go(k_render_tile<SD_F16, true, NWV>); else go(k_render_tile<SD_F16, false, NWV>); \
    } else {                                                                                    \
        if (zin) go(k_render_tile<SD_BF16, true, NWV>); else go(k_render_tile<SD_BF16, false, NWV>); \
    }
    if (nw == 8) {
        ST_GO(8)
    } else {
        ST_GO(ST_NW_SMALLK)
    }
#undef ST_GO
    return sd_check_last("sd_render_proj (tile kernel)");
}
