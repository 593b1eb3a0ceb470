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
//   barrier X union of the next group's boxes; if it fits the tile buffer, the waves
//             issue the LDS-DMA of those P texels, row by row of the box (else the group
//             goes to the overflow list and the fallback kernel renders it)
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
#include <stdlib.h>

// waves per workgroup = rays per group (NW): 8 (2 waves per SIMD), or for K <= 64 the
// ST_NW_SMALLK-wave variant (12: 3 waves per SIMD, the kernel compiled for <= 168 VGPRs)
#ifndef ST_NW_SMALLK
#define ST_NW_SMALLK 8
#endif
#define ST_TEX 288          // LDS bytes per staged texel: 256 B of P + 32 B pad
#define ST_TEXQ 18          // 16-byte chunks per staged texel
#define ST_MAXP 2           // K <= 128 (two samples per lane in the ray pass)
#define ST_MAXKW 8          // DMA columns (1-KiB pieces of a box row) per wave: rows <= 8 x 8 x 64 / 18 texels

// diagnostic build only (ST_PROF=1): per-phase s_memtime cycles summed over all waves
// (tools/tile_prof.py); the outputs are unchanged
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
#elif defined(ST_MARK) && ST_MARK
#define ST_T(i) asm volatile(";@T " #i)
#else
#define ST_T(i)
#endif
// diagnostic build only (ST_MARK=1): asm comments at the item-loop phase boundaries, for the
// static instruction-category count of tools/tile_isa_count.py (no code of their own; the
// scheduler may still move arithmetic across them, so the split is approximate)
#ifndef ST_MARK
#define ST_MARK 0
#endif
#if ST_MARK
#define ST_M(i) asm volatile(";@M " #i)
// a marker pinned after the value x is computed (and before its later uses)
#define ST_MV(i, x) asm volatile(";@M " #i : "+v"(x))
#else
#define ST_M(i)
#define ST_MV(i, x)
#endif

#ifndef ST_WAIT_FIX
#define ST_WAIT_FIX 1       // compiler-visible vmcnt(0) after the register-resident weight loads
#endif
#ifndef ST_HEAD_PRE
#define ST_HEAD_PRE 3       // 3: the previous group's DINO head before the ray pass, its first
                            // W_dino tile loaded at the end of the step before (the loads land
                            // during the closing vmcnt(0) wait for the tile DMA, and the 16
                            // VGPRs are live only across the step boundary, not the items);
                            // 2: the head before the ray pass, W_dino loaded inside it; 1: the
                            // first tile preloaded across the pass (spills); 0: after the pass
#endif
#ifndef ST_HC16
#define ST_HC16 1           // hidden-space compositing by v_pk_fma_f16 into packed f16 per-lane
                            // partial sums (0: v_dot2 into f32, twice the instructions)
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
    int32_t *ovf;           // overflow lists (sdhip_render.h): [gridDim.x] counts, [gridDim.x][ovf_cap] blocks
    int32_t ovf_cap;
    int32_t ngroups;        // ceil(R / NW)
    int32_t tile_bytes;     // bytes per tile buffer (multiple of 1024)
};

// LDS image (byte offsets): boxes, hidden sums, weight sums, ray words, then the sample
// records [NW waves][2][K] x 40 B and two tile buffers.  The code-column and sigma A
// fragments live in VGPRs for the whole kernel (loaded from global memory once).
// boxes [2][NW waves] x 32 B, u16x2 packed (min, max): per half ray (16 B), or, when a wave
// step holds 64 samples (K R_pw = 64), per quarter = 16-sample row (halves = unions of two)
#define ST_L_BOX 0
// hidden-sum rows padded to 272 B: the DINO head reads the same 8-B slot of the NW rows in
// one instruction (256-B rows put them on one bank pair: 8-way conflicts)
#define ST_HS_ROW 272
// rpw = rays per wave and step (2 for K <= 32: a group is NW rpw rays)
__host__ __device__ constexpr int st_l_hs(int nw) { return ST_L_BOX + 2 * nw * 32; }         // [NW rpw rays][128] 16-bit hidden sums
__host__ __device__ constexpr int st_l_ws(int nw, int rpw) { return st_l_hs(nw) + nw * rpw * ST_HS_ROW; }  // [NW rpw] f32 weight sums
__host__ __device__ constexpr int st_l_ray(int nw, int rpw) { return st_l_ws(nw, rpw) + 16 * 4; }          // [NW waves][2] x rpw x 32 B ray words 0..7 (LDS-DMA)
__host__ __device__ constexpr int st_l_rec(int nw, int rpw) { return st_l_ray(nw, rpw) + nw * 2 * 32 * rpw; }  // records: [NW waves][2][rpw K] x 40 B
static_assert(st_l_rec(8, 1) % 16 == 0 && st_l_rec(12, 1) % 16 == 0 && st_l_rec(8, 2) % 16 == 0,
              "record area alignment");

// record bytes for samples-per-wave-step kw = rpw K
__host__ __device__ constexpr int st_rec_bytes(int nw, int kw) { return nw * 2 * kw * 40; }

// one butterfly level of a 16-lane row sum over two values: out = a + a(lane - RA) on the
// lanes of banks MA (groups of 4 lanes), b + b(lane - RB) on the lanes of banks MB (MA | MB =
// every bank, so both bank-masked DPP adds together write every lane of out).  One asm
// statement: the compiler does not fold a partially masked DPP move into its user.  No
// s_nop past the first statement (NOP = "s_nop 1\n\t" there): the statements are volatile,
// so they stay in program order, and every later one reads values written at least two
// VALU ops before it (the callers' ordering); out is written, never read.
#define ST_BFLY(NOP, out, a, b, RA, RB, MA, MB)                                               \
    asm volatile(NOP "v_add_f32_dpp %0, %1, %1 row_ror:" #RA " row_mask:0xf bank_mask:" #MA "\n\t" \
                 "v_add_f32_dpp %0, %2, %2 row_ror:" #RB " row_mask:0xf bank_mask:" #MB      \
                 : "=&v"(out) : "v"(a), "v"(b))

// packed u16x2 (x | y << 16) component-wise min / max
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
// (round 6: pitch = 4 mod 8, conflict-free for the two samples of a half-wave read when they
// sit 1 or 2 texels apart along an epipolar line, measured C2 neutral and C1 +5 % -- the
// extra pad texels split more boxes; not kept)
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

// Diagnostic switch ST_WT=1: output stores write-through (sc1: the line leaves the XCD's L2
// clean), so that the ~15 MB of outputs still dirty in L2 when the kernel ends are not
// written back at the next kernel boundary (rocprofv3 WRITE_SIZE of the launch behind).
// Measured no faster (C1 0.406-0.409 vs 0.401-0.409, C2 0.620-0.628 vs 0.614-0.616 ms,
// `profiles/r5_wt_ab.txt`): the write-back is overlapped or replaced by the write-through
// traffic inside the kernel.  Off.
#ifndef ST_WT
#define ST_WT 0
#endif
#ifndef ST_WAIT_EARLY
#define ST_WAIT_EARLY 1   // the step's DMA wait before the epilogue's stores (0: after them)
#endif
#ifndef ST_EARLY_HW
#define ST_EARLY_HW ST_WAIT_EARLY  // HPRE 3: the next head's W_dino loaded after staging (0: at step end)
#endif
#ifndef ST_PRIO
#define ST_PRIO 0
#endif
#ifndef ST_EARLY_FETCH
#define ST_EARLY_FETCH 1  // next-next step's ray words fetched after staging (0: at step end)
#endif
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_out(float *p, float v) {
    if (ST_WT)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// 4-byte LDS-DMA (ray words), inline asm for the reason given at sd_dma16 (sdhip_render.h)
__device__ __forceinline__ void st_dma4(const void *src, uint32_t lds_addr) {
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                 :: "v"(src), "s"(lds_addr) : "memory");
}
// 16-byte LDS-DMA through a buffer resource: lane data from rsrc + soff + voff to
// lds_addr + 16 * lane (active lanes only).  The per-lane part of a staged box row's
// address (voff) is the same for every row, the row base (soff) is wave-uniform.
__device__ __forceinline__ void st_dma_buf16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff,
                                             uint32_t lds_addr) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                 :: "v"(voff), "s"(rs), "s"(lds_addr), "s"(soff) : "memory");
}
typedef __attribute__((ext_vector_type(4))) short s16x4;

__device__ __forceinline__ uint2 st_tr(uint32_t addr) {
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4 *)(uintptr_t)addr);
    return __builtin_bit_cast(uint2, v);
}

// ZIN: depths given (args.z, parity tests) instead of drawn in the kernel.  A template
// parameter, not a branch: with both paths in one body the compiler's wait for the z loads
// also drains other loads on the drawing path.
// RPW = 2 (K <= 32): every wave takes TWO neighbouring rays per step -- the ray pass runs
// their 2 K samples on the 64 lanes, a group is 2 NW rays (one tile box, barrier pair, DINO
// head and set of DMA issues per 16 rays), the items of ray A then of ray B, one sum
// epilogue per ray.  The per-step phases that cost the same at any K are paid once per two
// rays (round-4 phase split at K = 32: items only 23 % of the wave time).
template <int P, bool ZIN, int NW, int RPW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4)))
k_render_tile(const st_args sa) {
    // the head's W_dino prefetch across the step boundary (mode 3) costs 16-20 VGPRs: the
    // two-rays-per-wave body (245 VGPRs) would spill, so it loads them inside the head
// RPW = 2 head mode: 2 (the W_dino loads inside the head); 1 (loaded before the ray pass,
// head after it) spills 8 VGPRs at 256
#ifndef ST_HPRE_RPW2
#define ST_HPRE_RPW2 2
#endif
    constexpr int HPRE = (RPW == 2 && ST_HEAD_PRE == 3) ? ST_HPRE_RPW2 : ST_HEAD_PRE;
    constexpr int ST_WAVES = NW;
    constexpr int GR = NW * RPW;  // rays per group
    constexpr int ST_L_HS = st_l_hs(NW), ST_L_WS = st_l_ws(NW, RPW), ST_L_RAY = st_l_ray(NW, RPW),
                  ST_L_REC = st_l_rec(NW, RPW);
    typedef typename RMode<P>::F Tr;  // operands upstream of sigma (f16 in both modes)
    typedef typename RMode<P>::H Th;  // DINO head (bf16 in the bf16 mode)
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
    const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_void *)lds;  // LDS byte address of lds[0]

    const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int K = a.K, nsub = K >> 4;   // samples / items per ray
    const int KW = K * RPW, nsubw = KW >> 4;  // per wave and step
    const int R = (int)a.R, rps = (int)a.rays_per_sb;
    const int D = m.D, ndt = D >> 4;
    const int Wf = a.Wf, Hf = a.Hf;
    const uint32_t plane_bytes = (uint32_t)Hf * Wf * SD_DH * 2;

    // records: SoA per (wave, buffer): q0 [K] x 16 B | q1 [K] x 16 B | c [K] x 8 B
    //   q0 = {x0 | y0 << 15 | inv_f << 30 | invc << 31, (w00, w01), (w10, w11), r}
    //   q1 = {x, y, z~, z}   c = {g, b}
    // (RPW = 2: record k' = r K + k is sample k of the wave's ray r)
    const uint32_t rec_base = ST_L_REC + (uint32_t)wave * 2 * KW * 40;
    auto rq0 = [&](int buf) { return (uint4 *)(lds + rec_base + buf * KW * 40); };
    auto rq1 = [&](int buf) { return (f32x4 *)(lds + rec_base + buf * KW * 40 + KW * 16); };
    auto rqc = [&](int buf) { return (float2 *)(lds + rec_base + buf * KW * 40 + KW * 32); };
    const uint32_t tile0 = ST_L_REC + st_rec_bytes(NW, KW);

    // XCD-aware group ranges (workgroups b, b + 8, ... share an XCD, speed only)
    const int NG = sa.ngroups;
    const int nx = (gridDim.x % 8 == 0) ? 8 : 1;
    const int xcd = blockIdx.x % nx, lb = blockIdx.x / nx, nwg = gridDim.x / nx;
    const int glo = (int)((int64_t)NG * xcd / nx), ghi = (int)((int64_t)NG * (xcd + 1) / nx);
    const int gfirst = glo + lb;
    const int nsteps = gfirst < ghi ? (ghi - gfirst + nwg - 1) / nwg : 0;
    int novf = 0;  // this workgroup's overflow blocks (workgroup-uniform)
    int32_t *ovf_list = sa.ovf + gridDim.x + (int64_t)blockIdx.x * sa.ovf_cap;
    if (nsteps == 0) {  // workgroup-uniform
        if (threadIdx.x == 0) sa.ovf[blockIdx.x] = 0;
        return;
    }

    const float zstep = (float)(1.0 / (double)K), zend = (float)(1.0 - 1.0 / (double)K);
    const int64_t cplane = (int64_t)a.Hc * a.Wc * 4;

    // ---- ray pass: lane = sample k = 64 p + lane --------------------------------------
    // ray words 0..7 (origin, direction, near, far) of a later step's ray, fetched by
    // LDS-DMA one step ahead (completed by the step's closing vmcnt(0)), so the ray pass
    // reads them from LDS instead of waiting on scalar loads
    const int nrw = min(a.ray_dim, 8);
    // memory index of the wave's ray r, given ray = GR grp + RPW wave (the wave's first
    // slot): RPW = 2 pairs ray w with ray w + NW of the group, so the two halves a group
    // splits into when its tap box overflows (kh = K below: the halves are the rays of slot
    // 0 and of slot 1) are the group's left and right 8 rays -- as adjacent pairs (2 w,
    // 2 w + 1) both halves spanned the whole strip and 2.5 % of the C1 offset-pose rays went
    // to the per-ray fallback kernel (52 us of a 0.43 ms frame)
    auto rmap = [&](int ray_, int r) { return RPW == 1 ? ray_ + r : ray_ - RPW * wave + r * NW + wave; };
    // the wave's RPW rays: lane 8 r + w fetches word w of ray r
    auto ray_fetch = [&](int ray, int slot) {
        const int r = lane >> 3, w = lane & 7;
        if (r < RPW && w < nrw && rmap(ray, r) < R)
            st_dma4(a.rays + (int64_t)rmap(ray, r) * a.ray_dim + w,
                    lds0 + ST_L_RAY + (wave * 2 + slot) * 32 * RPW);
    };
    // this lane's ray of the wave's RPW for ray-pass sample slot p (record k' = 64 p + lane
    // = r K + k: K <= 32 -- p = 0 only, r = lane / K; K = 64 -- r = p)
    const int rsl = RPW == 1 ? 0 : min(lane / K, RPW - 1);
    auto rsl_p = [&](int p) { return RPW == 1 ? 0 : min((64 * p + lane) / K, RPW - 1); };
    auto kl_p = [&](int p) { return RPW == 1 ? 64 * p + lane : 64 * p + lane - rsl_p(p) * K; };
    const float *rl = nullptr;  // this ray pass's words of the wave's first ray (set by ray_pass)
    auto load_ray_z = [&](int ray, float zq[2 * ST_MAXP]) {
        float zo[ST_MAXP];
        if (ZIN) {
            if (RPW == 1) {
                const float *zr = a.z + (int64_t)ray * K;
#pragma unroll
                for (int p = 0; p < ST_MAXP; ++p) zo[p] = zr[min(64 * p + lane, K - 1)];
            } else {
                zo[1] = 0.f;
#pragma unroll
                for (int p = 0; p < ST_MAXP; ++p) {
                    if (64 * p >= KW) break;  // wave-uniform
                    const float *zr = a.z + (int64_t)min(rmap(ray, rsl_p(p)), R - 1) * K;
                    zo[p] = zr[min(kl_p(p), K - 1)];  // (lanes past 2 K: K = 16)
                }
            }
        } else {
            zo[1] = 0.f;
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) {
                if (64 * p >= KW) break;  // wave-uniform: KW <= 64 draws one sample per lane
                const int r = rsl_p(p);
                const float *rw = rl + 8 * r;
                const float near = rw[6], far = rw[7];
                const uint64_t base = a.z_offset + (uint64_t)rmap(ray, r) * (uint64_t)K;
                const int k = RPW == 1 ? min(64 * p + lane, K - 1) : kl_p(p);
                zo[p] = sd_z_sample_rng(near, far, K, k, sd_uniform(a.z_seed, base + k), zstep, zend,
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
            if (lane == 63) nx2 = (p + 1 < ST_MAXP && 64 * (p + 1) < KW) ? first_next : zo[p];
            zq[2 * p] = zo[p];
            zq[2 * p + 1] = nx2;
        }
    };
    // the colour texel loads of sample k = lane are left in flight (cpend) and finished
    // by ray_col at the end of the item that ran the pass
    ColPend cpend;
    // tap boxes per half ray: samples [0, kh) and [kh, K), kh = 16 (nsub / 2) -- a group
    // whose whole box does not fit a tile buffer is staged and rendered half by half
    // (RPW = 2: the halves are the two rays)
    const int kh = RPW == 1 ? 16 * (nsub >> 1) : K;
    auto ray_pass = [&](int ray, int buf, int slot) {
        uint32_t bmin0 = 0xffffffffu, bmax0 = 0u, bmin1 = 0xffffffffu, bmax1 = 0u;
        if (ray < R) {
            // wave-uniform (readfirstlane: the u32 divide runs on the VALU, and a VGPR
            // address would turn the camera-record reads into vector loads); a group's rays
            // share their super-batch (rays_per_sb % GR == 0)
            const int sbi = __builtin_amdgcn_readfirstlane((int)((unsigned)ray / (unsigned)rps));
            rl = (const float *)(lds + ST_L_RAY + (wave * 2 + slot) * 32 * RPW);
            // colour view = encoder view (the single-frame render, ids_render = ids_encoder):
            // the host passes the same camera records for both (cam_c == cam_f), so the
            // colour taps are the encoder-view taps at equal resolution (kernel-uniform test)
            const bool same_cam = ST_SAME_CAM && a.cam_c == a.cam_f && a.Wc == Wf && a.Hc == Hf;
            float zq[2 * ST_MAXP];
            load_ray_z(ray, zq);
            ST_T(10);
            uint4 *r0 = rq0(buf);
            f32x4 *r1 = rq1(buf);
            float2 *rc = rqc(buf);
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) {
                const int k = 64 * p + lane;  // record k' (RPW = 2: ray rsl_p(p)'s sample kl_p(p))
                if (64 * p < KW && k < KW && (RPW == 1 || rmap(ray, rsl_p(p)) < R)) {
                    const float *rw = rl + 8 * rsl_p(p);
                    const float ox = rw[0], oy = rw[1], oz = rw[2], dx = rw[3], dy = rw[4], dz = rw[5];
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
                    const uint4 wp = sd_pack_w<SD_F16>(geo.t.w00, geo.t.w01, geo.t.w10, geo.t.w11);
                    r1[k] = f32x4{geo.v[0], geo.v[1], geo.v[2], z0};
                    if (p == 0) {
                        sd_color_issue(a.img + (int64_t)sbi * cplane, tc, cpend);
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
        uint8_t *bw = lds + ST_L_BOX + (slot * ST_WAVES + wave) * 32;
        if (KW == 64) {
            // one sample per lane: quarter q = row q (items 4 q'.. of the step), halves =
            // lanes [0, 32) and [32, 64)
            const uint32_t mnv = st_row_red2<false>(lane < 32 ? bmin0 : bmin1);
            const uint32_t mxv = st_row_red2<true>(lane < 32 ? bmax0 : bmax1);
            uint32_t q[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                q[2 * r] = st_rows2<false>(mnv, r, r);
                q[2 * r + 1] = st_rows2<true>(mxv, r, r);
            }
            ST_T(12);
            if (lane == 0) {
                *(uint4 *)bw = uint4{q[0], q[1], q[2], q[3]};
                *(uint4 *)(bw + 16) = uint4{q[4], q[5], q[6], q[7]};
            }
        } else if (RPW == 2 && KW == 128) {
            // two rays of 64 samples, one sample of each per lane (slot p = ray p): part
            // 2 p + h = lanes [32 h, 32 h + 32) of slot p = items 4 p + 2 h, + 1 (halves = rays)
            const uint32_t mn0 = st_row_red2<false>(bmin0), mx0 = st_row_red2<true>(bmax0);
            const uint32_t mn1 = st_row_red2<false>(bmin1), mx1 = st_row_red2<true>(bmax1);
            uint32_t q[8];
            q[0] = st_rows2<false>(mn0, 0, 1);
            q[1] = st_rows2<true>(mx0, 0, 1);
            q[2] = st_rows2<false>(mn0, 2, 3);
            q[3] = st_rows2<true>(mx0, 2, 3);
            q[4] = st_rows2<false>(mn1, 0, 1);
            q[5] = st_rows2<true>(mx1, 0, 1);
            q[6] = st_rows2<false>(mn1, 2, 3);
            q[7] = st_rows2<true>(mx1, 2, 3);
            ST_T(12);
            if (lane == 0) {
                *(uint4 *)bw = uint4{q[0], q[1], q[2], q[3]};
                *(uint4 *)(bw + 16) = uint4{q[4], q[5], q[6], q[7]};
            }
        } else {
            bmin0 = st_wave_min2(bmin0);
            bmax0 = st_wave_max2(bmax0);
            bmin1 = st_wave_min2(bmin1);
            bmax1 = st_wave_max2(bmax1);
            ST_T(12);
            if (lane == 0) *(uint4 *)bw = uint4{bmin0, bmax0, bmin1, bmax1};
        }
    };
    auto ray_col = [&](int ray, int buf) {
        if (rmap(ray, rsl) < R && lane < KW) {
            float col[3];
            sd_color_finish(cpend, col);
            rq0(buf)[lane].w = __builtin_bit_cast(uint32_t, col[0]);
            rqc(buf)[lane] = float2{col[1], col[2]};
        }
    };

    // ---- per-step tile geometry (workgroup-uniform) -----------------------------------
    struct Tile {
        int bx0, by0, tw, th, pitch, ok, split;
    };
    // union of the NW waves' boxes of slot over parts [p0, p1): a wave's entry holds NPART
    // (min, max) pairs -- the 4 quarters when KW = 64, else the 2 halves -- so half h =
    // parts [h NPART / 2, (h + 1) NPART / 2), the whole group = [0, NPART).  One copy of the
    // code for every part range (a select chain per range grew the kernel by half: i-cache)
    const int NPART = (KW == 64 || (RPW == 2 && KW == 128)) ? 4 : 2;
    auto box_union = [&](int slot, int p0, int p1, uint32_t &mn, uint32_t &mx) {
        // lane 2 i + h reads wave i's parts 2 h, 2 h + 1 (one LDS read; a loop over the parts
        // was four dependent LDS round trips: +45 % stage time at C2), then a wave reduction
        const uint4 *bx = (const uint4 *)(lds + ST_L_BOX + slot * ST_WAVES * 32);
        mn = 0xffffffffu;
        mx = 0u;
        if (lane < 2 * ST_WAVES) {
            const uint4 v = bx[lane];
            const int pa = 2 * (lane & 1);
            if (pa >= p0 && pa < p1) {
                mn = v.x;
                mx = v.y;
            }
            if (pa + 1 >= p0 && pa + 1 < p1) {
                mn = st_min2(mn, v.z);
                mx = st_max2(mx, v.w);
            }
        }
        static_assert(2 * ST_WAVES <= 16, "box entries in lane row 0");
        mn = st_rows2<false>(st_row_red2<false>(mn), 0, 0);
        mx = st_rows2<true>(st_row_red2<true>(mx), 0, 0);
    };
    // a box row of tw texels = tw x 18 16-B chunks = ceil(tw x 18 / 64) 1-KiB DMA pieces;
    // the box fits when its rows at the tile pitch fit the buffer
    auto geom = [&](uint32_t mn, uint32_t mx) {
        Tile t;
        t.bx0 = (int)(mn & 0xffffu);
        t.by0 = (int)(mn >> 16);
        t.tw = (int)(mx & 0xffffu) - t.bx0 + 1;
        t.th = (int)(mx >> 16) - t.by0 + 1;
        t.pitch = t.tw > 0 ? st_pitch(t.tw) : 1;
        t.ok = (mn != 0xffffffffu) && t.tw > 0 && t.th > 0 &&
               t.th * t.pitch * ST_TEX <= sa.tile_bytes && (t.tw * ST_TEXQ + 63) / 64 <= ST_MAXKW * ST_WAVES;
        t.split = 0;
        return t;
    };
    // this wave's share of the LDS-DMA of tile t into tile buffer tb: box row ty, piece c
    // (1 KiB = 64 lanes x 16 B, chunks 64 c .. 64 c + 63 of the row) goes to wave c % NW.
    // The lane's chunk (texel tx, part) and so its offset inside the row are the same for
    // every row: computed once per piece, then each row is one buffer_load ... lds with the
    // row's base as the scalar offset.  The texels' 32-B pad chunks (part 16, 17) and the
    // lanes past the row end are masked off (they are never read).
    auto dma = [&](const Tile &t, int tb, int sbi) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)((const uint8_t *)a.grid + (int64_t)__builtin_amdgcn_readfirstlane(sbi) * plane_bytes), 0,
            plane_bytes, 0x00020000);
        const uint32_t dst0 = lds0 + tile0 + (uint32_t)tb * (uint32_t)sa.tile_bytes;
        const int nk = (t.tw * ST_TEXQ + 63) >> 6;
        const uint32_t rowb = (uint32_t)t.pitch * ST_TEX;
        // the lane id through a volatile move: the per-piece (tx, part) below are then
        // computed here, not hoisted out of the step loop as 8 loop-invariant VGPRs (spilled
        // at 256 VGPRs: a scratch reload -- and its vmcnt(0) -- in front of every DMA piece)
        uint32_t ln = (uint32_t)lane;
#ifndef ST_DMA_LNVOL
#define ST_DMA_LNVOL 1
#endif
        if (ST_DMA_LNVOL) asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
#pragma unroll
        for (int kk = 0; kk < ST_MAXKW; ++kk) {
            const int c = wave + ST_WAVES * kk;
            if (c >= nk) break;  // wave-uniform
            const uint32_t ci = (uint32_t)c * 64u + ln;
            const uint32_t tx = __umulhi(ci, 238609295u);  // ci / 18
            const uint32_t part = ci - 18u * tx;
            const uint32_t sx = (uint32_t)min(t.bx0 + (int)tx, Wf - 1);
            const uint32_t voff = sx * 256u + part * 16u;
            if (part < 16u && (int)tx < t.tw) {
                for (int ty = 0; ty < t.th; ++ty) {
                    const uint32_t sy = (uint32_t)min(t.by0 + ty, Hf - 1);
                    st_dma_buf16(rs, voff, __builtin_amdgcn_readfirstlane(sy * (uint32_t)Wf * 256u),
                                 __builtin_amdgcn_readfirstlane(dst0 + (uint32_t)ty * rowb + (uint32_t)c * 1024u));
                }
            }
        }
    };
    // geometry of slot's group for tile buffer tb, DMA issued: the whole box if it fits,
    // else (nsub >= 2) the first half's box when both halves fit (split = 1: the second
    // half is staged mid-step), else (KW = 64) the first quarter's when all four fit
    // (split = 3: restaged before items 1, 2, 3 -- the C1 offset-pose groups whose halves
    // overflow, 0.25 % of the rays), else the group goes to the overflow list (ok = 0).
    // An empty part (its rays past R) fits.
    auto stage = [&](int slot, int tb, int grp, int sbi) {
        uint32_t mn, mx;
        box_union(slot, 0, NPART, mn, mx);
        Tile t = geom(mn, mx);
        if (mn == 0xffffffffu) return t;  // no valid ray in the group
        if (!t.ok && nsub >= 2) {
#pragma unroll 1
            for (int np = 2; np <= NPART; np *= 2) {  // halves, then quarters
                bool all = true;
                for (int q = 0; q < np && all; ++q) {
                    uint32_t pn, px;
                    box_union(slot, q * NPART / np, (q + 1) * NPART / np, pn, px);
                    all = pn == 0xffffffffu || geom(pn, px).ok;
                }
                if (all) {
                    box_union(slot, 0, NPART / np, mn, mx);
                    t = geom(mn, mx);
                    t.ok = 1;
                    t.split = np - 1;
                    break;
                }
            }
        }
        if (!t.ok) {
            if (wave == 0 && lane == 0) {  // the group's rays as GR / SD_LIST_BLK list blocks
                for (int b = 0; b < GR / SD_LIST_BLK; ++b)
                    ovf_list[novf + b] = grp * (GR / SD_LIST_BLK) + b;
            }
            novf += GR / SD_LIST_BLK;
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
        if (!t.ok || ray_ >= R) return;
        // part q of a split group (split + 1 parts) = items [q nsubw / np, (q + 1) nsubw / np)
        // of the step (as the box halves / quarters of ray_pass): its records' geometry
        int gx[ST_MAXP], gy[ST_MAXP], gp[ST_MAXP];
#pragma unroll
        for (int p = 0; p < ST_MAXP; ++p) {
            gx[p] = t.bx0;
            gy[p] = t.by0;
            gp[p] = t.pitch;
        }
        const int np = t.split + 1;
#pragma unroll 1
        for (int q = 1; q < np; ++q) {
            uint32_t mn1, mx1;
            box_union(rbuf, q * NPART / np, (q + 1) * NPART / np, mn1, mx1);
            const Tile tq = geom(mn1, mx1);
            const int s0 = q * nsubw / np, s1 = (q + 1) * nsubw / np;
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) {
                const int it = (64 * p + lane) >> 4;
                const bool mine = it >= s0 && it < s1;
                gx[p] = mine ? tq.bx0 : gx[p];
                gy[p] = mine ? tq.by0 : gy[p];
                gp[p] = mine ? tq.pitch : gp[p];
            }
        }
        const uint32_t tbase = lds0 + tile0 + (uint32_t)tb * (uint32_t)sa.tile_bytes;
        uint32_t *w = (uint32_t *)rq0(rbuf);
#pragma unroll
        for (int p = 0; p < ST_MAXP; ++p) {
            const int k = 64 * p + lane;
            if (64 * p < KW && k < KW) {
                const uint32_t xy = w[4 * k];
                const int bx0 = gx[p], by0 = gy[p], pch = gp[p];
                const int x0 = (int)(xy & 0x7fffu), y0 = (int)((xy >> 15) & 0x7fffu);
                const uint32_t ad = tbase + (uint32_t)(((y0 - by0) * pch + (x0 - bx0)) * ST_TEX);
                w[4 * k] = ad | (xy & 0xc0000000u);
            }
        }
    };

    // ---- DINO head of one group (hsum of its NW rays in LDS) --------------------------
    // W_dino fragments of tile dt (4 x 16 B per lane).  HPRE: the wave's first tile is
    // loaded before the step's ray pass, so the head's wait for it does not also wait for the
    // ray pass's colour loads (issued later, consumed after item 0)
    typedef typename Th::Frag HFrag;
    // RPW = 2: this wave's DINO bias slice (tile dt = wave) in registers for the whole kernel
    // -- as a global load inside the head it put one memory latency in front of every step's
    // ray pass (C1 -1 %); at RPW = 1 the 4 VGPRs (and the rescheduling) cost more than the
    // load (`profiles/r5_bias_hoist_ab.txt`)
#ifndef ST_BD_HOIST1
#define ST_BD_HOIST1 0
#endif
    constexpr bool BDH = RPW == 2 || ST_BD_HOIST1;
    f32x4 bdw = {0.f, 0.f, 0.f, 0.f};
    if (BDH && wave < ndt) bdw = *(const f32x4 *)(m.b_dino + 16 * wave + 4 * g);
    auto head_w = [&](int dt, HFrag w[4]) {
        const HFrag *wo = (const HFrag *)m.w_out + (int64_t)dt * 4 * SD_WAVE + lane;
#pragma unroll
        for (int s = 0; s < 4; ++s) w[s] = wo[s * SD_WAVE];
    };
    auto head = [&](int grp, const HFrag w0[4]) {
        if (wave >= ndt) return;
        const int slot = j < GR ? j : 0;  // B columns j >= GR: not stored
        typename Th::Frag Bh[4];
        const uint8_t *hs = lds + ST_L_HS + slot * ST_HS_ROW;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const uint2 lo = *(const uint2 *)(hs + (32 * s + 4 * g) * 2);
            const uint2 hi = *(const uint2 *)(hs + (32 * s + 16 + 4 * g) * 2);
            Bh[s] = __builtin_bit_cast(typename Th::Frag, uint4{lo.x, lo.y, hi.x, hi.y});
        }
        const float ws = *(const float *)(lds + ST_L_WS + slot * 4);
        const int ray = GR * grp + (RPW == 1 ? j : (j % RPW) * NW + j / RPW);  // hs row j = wave RPW + r
        const bool store = j < GR && ray < R;
        for (int dt = wave; dt < ndt; dt += ST_WAVES) {
            HFrag wl[4];
            if ((HPRE == 1 || HPRE == 3) && dt == wave) {
#pragma unroll
                for (int s = 0; s < 4; ++s) wl[s] = w0[s];
            } else {
                head_w(dt, wl);
            }
            f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < 4; ++s) o = Th::mma(wl[s], Bh[s], o);
            // rows 4 g + r of tile dt = dims 16 dt + 4 g + r, column j = ray slot
            const int dim = 16 * dt + 4 * g;
            const f32x4 bd = (BDH && dt == wave) ? bdw : *(const f32x4 *)(m.b_dino + dim);
            f32x4 res;
#pragma unroll
            for (int r = 0; r < 4; ++r) res[r] = o[r] + ws * bd[r];
            if (store) {
                if (ST_WT) {  // 16-B write-through store (buffer aux 16 = sc1)
                    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                        (void *)(a.dino + (int64_t)GR * grp * a.ld_dino), 0, 0x7fffffff, 0x00020000);
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(u32x4v, res), rs,
                        (uint32_t)(((int64_t)(ray - GR * grp) * a.ld_dino + dim) * 4), 0, 16);
                } else {
                    *(f32x4 *)(a.dino + (int64_t)ray * a.ld_dino + dim) = res;
                }
            }
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
    // this lane's code-column weight fragments (16x16x32 and 16x16x16 operands) and sigma
    // weights (every row of the sigma A fragment holds W_out[0] at hid(s, g, e),
    // mlp_pack.py), held in VGPRs for the whole kernel
    Frag wpe[8];
    Frag4 wpe1[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        wpe[t] = ((const Frag *)m.w_pe)[t * SD_WAVE + lane];
        wpe1[t] = ((const Frag4 *)((const uint8_t *)m.w_pe + 8 * SD_WAVE * 16))[t * SD_WAVE + lane];
    }
    uint4 wsig_r[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) wsig_r[s2] = ((const uint4 *)m.w_sig)[s2 * SD_WAVE + lane];
    // a wait the compiler SEES (the builtin, not inline asm: vmcnt(0), expcnt / lgkmcnt
    // unconstrained): without it its wait-count tracking keeps these 20 loads pending into
    // the item loop and guards their first uses there with vmcnt(19) .. vmcnt(0) -- which the
    // hardware also counts the in-flight tile LDS-DMA against, so every item waited for the
    // next group's staging to land
#if ST_WAIT_FIX
    __builtin_amdgcn_s_waitcnt(0x0F70);
#endif

    // ---- prologue: records + tile of step 0 -------------------------------------------
    int grp = gfirst;
    int ray = GR * grp + RPW * wave;  // the wave's first ray of the step
    int sbi = __builtin_amdgcn_readfirstlane((int)((unsigned)min(GR * grp, R - 1) / (unsigned)rps));
    ray_fetch(ray, 0);
    ray_fetch(GR * (grp + nwg) + RPW * wave, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ray_pass(ray, 0, 0);
    ray_col(ray, 0);
    st_barrier_lds();
    Tile cur = stage(0, 0, grp, sbi);
    tap_addrs(0, 0, cur, ray);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ST_PRIO (build knob): static issue priority for one half of the workgroup for the whole
    // step loop (MI355X guide, two-waves-per-SIMD item 4: the second-dispatched half, waves
    // NW / 2 .., loses every arbitration; 1 raises that half, 2 the first half, 0 none)
    if (ST_PRIO == 1 && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if (ST_PRIO == 2 && wave < NW / 2) __builtin_amdgcn_s_setprio(1);
    int prev_grp = -1, prev_ok = 0;
    HFrag hwn[4];  // HPRE 3: W_dino tile `wave` for the next step's head
#if ST_PROF
#pragma unroll
    for (int i = 0; i < 19; ++i) pacc[i] = 0;
    tlast = __builtin_amdgcn_s_memtime();
#endif
    for (int n = 0; n < nsteps; ++n) {
        const int buf = n & 1;
        const bool has_next = n + 1 < nsteps;
        const int ngrp = grp + nwg;
        const int nray = GR * ngrp + RPW * wave;
        const int nsbi = has_next ? __builtin_amdgcn_readfirstlane((int)((unsigned)min(GR * ngrp, R - 1) / (unsigned)rps)) : 0;
        uint32_t lane_off = (uint32_t)((tq & 1) + (tq >> 1) * cur.pitch) * ST_TEX + 8u * (uint32_t)tp;

        // per-ray compositing state (RPW = 2: reset between the wave's two rays)
        float Tc, dpart, wpart, cpart[3];
#if ST_HC16
        // per-lane partial sums sum_k w_k relu(h_k) over this lane's samples (one per item:
        // K / 16 = 1..8 terms), packed f16 pairs in X's element order; the 16-lane sums of
        // the epilogue are f32
        f16x2 hacc16[16];
#else
        f32x4 hacc[8];
#endif
        auto reset = [&]() {
            Tc = 1.f;
            dpart = wpart = cpart[0] = cpart[1] = cpart[2] = 0.f;
#if ST_HC16
#pragma unroll
            for (int i = 0; i < 16; ++i) hacc16[i] = f16x2{(_Float16)0.f, (_Float16)0.f};
#else
#pragma unroll
            for (int t = 0; t < 8; ++t) hacc[t] = zero4;
#endif
        };
        reset();

        // An item is split in two: A = records, taps, MFMA MLP, sigma, alpha, local
        // transmittance scan; B = weights with the carried transmittance, compositing sums,
        // per-sample outputs.
        struct IState {
            Frag X[4];
            float alpha, excl, tmul, zk, col[3];
        };
        auto itemA = [&](int sub, IState &st) {
            ST_M(20);
            const int kr = sub * 16 + j;                                 // record k'
            const int k = RPW == 1 ? kr : kr - (sub / nsub) * K;         // sample of its ray
            const uint4 q0 = rq0(buf)[kr];
            const f32x4 q1 = rq1(buf)[kr];
            const float2 cgb = rqc(buf)[kr];
            const float znext = k + 1 < K ? rq1(buf)[kr + 1][3] : 0.f;
            const float v[3] = {q1[0], q1[1], q1[2]};
            st.zk = q1[3];
            const float delta = k + 1 < K ? znext - st.zk : 1e10f;
            st.col[0] = __builtin_bit_cast(float, q0.w);
            st.col[1] = cgb.x;
            st.col[2] = cgb.y;
            // tap bases of samples 8 c + 2 g + r, written by tap_addrs
            uint32_t base[2][2];
            const uint32_t *aw = (const uint32_t *)rq0(buf) + 4 * (sub * 16 + 2 * g);
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < 2; ++r) base[c][r] = (aw[4 * (8 * c + r)] & 0x3ffffu) + lane_off;
            // block-diagonal weight fragments of the two K-chunks
            ST_M(21);
            const uint32_t w01 = q0.y, w23 = q0.z;
            const uint4 b0 = {bc0 && !br1 ? w01 : 0u, bc0 && !br1 ? w23 : 0u,
                              bc0 && br1 ? w01 : 0u, bc0 && br1 ? w23 : 0u};
            const uint4 b1 = {bc1 && !br1 ? w01 : 0u, bc1 && !br1 ? w23 : 0u,
                              bc1 && br1 ? w01 : 0u, bc1 && br1 ? w23 : 0u};
            const Frag B0 = __builtin_bit_cast(Frag, b0), B1 = __builtin_bit_cast(Frag, b1);
            f32x4 acc[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint2 a00 = st_tr(base[0][0] + 32u * t), a01 = st_tr(base[0][1] + 32u * t);
                const uint2 a10 = st_tr(base[1][0] + 32u * t), a11 = st_tr(base[1][1] + 32u * t);
                const Frag A0 = __builtin_bit_cast(Frag, uint4{a00.x, a00.y, a01.x, a01.y});
                const Frag A1 = __builtin_bit_cast(Frag, uint4{a10.x, a10.y, a11.x, a11.y});
                acc[t] = Tr::mma(A0, B0, zero4);
                acc[t] = Tr::mma(A1, B1, acc[t]);
            }
            ST_MV(22, acc[7]);
            // positional-code columns: all 16x16x32 steps first, then the 16x16x16 ones
            // (a 16x16x16 MFMA whose accumulator input is the result of the directly
            // preceding 16x16x32 MFMA read a stale accumulator: hipcc 7.2, gfx950,
            // VGPR-form accumulators)
            {
                Frag f0;
                Frag4 f1;
                sd_code_frags<Frag, Frag4, E>(v, g, f0, f1);
#pragma unroll
                for (int t = 0; t < 8; ++t) acc[t] = Tr::mma(wpe[t], f0, acc[t]);
#pragma unroll
                for (int t = 0; t < 8; ++t) acc[t] = Tr::mma16(wpe1[t], f1, acc[t]);
            }
            ST_MV(23, acc[7]);
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 u = {sd_relu2(sd_pack2<E>(acc[2 * s2][0], acc[2 * s2][1])),
                                 sd_relu2(sd_pack2<E>(acc[2 * s2][2], acc[2 * s2][3])),
                                 sd_relu2(sd_pack2<E>(acc[2 * s2 + 1][0], acc[2 * s2 + 1][1])),
                                 sd_relu2(sd_pack2<E>(acc[2 * s2 + 1][2], acc[2 * s2 + 1][3]))};
                st.X[s2] = __builtin_bit_cast(Frag, u);
            }
            ST_MV(24, st.X[3]);
            f32x4 sg = zero4;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) sg = Tr::mma(__builtin_bit_cast(Frag, wsig_r[s2]), st.X[s2], sg);
            const float sigma = sd_softplus_fast(sg[0] + m.b_sigma);
            // alpha compositing (nerf.py:376-389)
            float alpha = 1.f - __expf(-fabsf(delta) * fmaxf(sigma, 0.f));
            if (a.hard_alpha_cap && k == K - 1) alpha = 1.f;
            const float incl = sd_scan_mul16((1.f - alpha) + 1e-10f);
            st.alpha = alpha;
            st.excl = SD_DPP1(incl, 0x111);
            st.tmul = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 15));
            ST_MV(25, st.tmul);
        };
        auto itemB = [&](int sub, const IState &st) {
            ST_M(26);
            const int k = sub * 16 + j;  // record k'
            const float w = st.alpha * (Tc * st.excl);
            Tc *= st.tmul;
            dpart += w * st.zk;
            wpart += w;
            cpart[0] += w * st.col[0];
            cpart[1] += w * st.col[1];
            cpart[2] += w * st.col[2];
            ST_MV(27, cpart[2]);
#if ST_HC16
            // hidden-space compositing: one v_pk_fma_f16 per packed pair of relu(h) (X is f16
            // in both modes, RMode)
            const f16x2 ww = __builtin_bit_cast(f16x2, sd_pack2<_Float16>(w, w));
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                const uint4 u = __builtin_bit_cast(uint4, st.X[s2]);
                const uint32_t d4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    hacc16[4 * s2 + q] = __builtin_elementwise_fma(__builtin_bit_cast(f16x2, d4[q]), ww,
                                                                   hacc16[4 * s2 + q]);
            }
#else
            // hidden-space compositing: v_dot2 of the packed hidden pairs with (w, 0) / (0, w)
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
#endif
            // weight and alpha into the sample's record (q1.x / .y are dead once itemA has
            // read the point); the ray epilogue stores every per-sample output coalesced
            if (g == 0) *(float2 *)&rq1(buf)[k] = float2{w, st.alpha};
            ST_M(28);
        };

        // item 0 with the next ray's pass and the previous group's head
        HFrag hw[4];
        if (HPRE == 1 && prev_ok && wave < ndt) head_w(wave, hw);
        if (HPRE == 2 && prev_ok) head(prev_grp, hw);
        if (HPRE == 3 && prev_ok) head(prev_grp, hwn);
        if (HPRE >= 2) ST_T(1);
        if (has_next) ray_pass(nray, buf ^ 1, buf ^ 1);
        ST_T(0);
        if (HPRE < 2 && prev_ok) head(prev_grp, hw);
        if (HPRE < 2) ST_T(1);
        IState s0;
        if (cur.ok && ray < R) itemA(0, s0);
        ST_T(2);
        if (has_next) ray_col(nray, buf ^ 1);
        ST_T(3);
        st_barrier_lds();  // X: next boxes visible; the head has read the hsum area
        ST_T(4);
        Tile nxt = {0, 0, 0, 0, 1, 0, 0};
        if (has_next) {
            nxt = stage(buf ^ 1, buf ^ 1, ngrp, nsbi);
            tap_addrs(buf ^ 1, buf ^ 1, nxt, nray);
        }
        // the rays of step n + 2 into ray slot buf (its words, step n's rays, were read by
        // the ray pass of step n - 1): issued here, they land under this step's items (issued
        // in front of the closing vmcnt(0), as before, every step waited one memory latency)
        if (ST_EARLY_FETCH && n + 2 < nsteps) ray_fetch(GR * (ngrp + nwg) + RPW * wave, buf);
        // HPRE 3: the next step's head weights (this group's; hwn was read by this step's head)
        if (ST_EARLY_HW && HPRE == 3 && cur.ok && wave < ndt) head_w(wave, hwn);
        ST_T(5);
        // split group: items of the first half ray from the current tile, then the second
        // half's box is staged into the same buffer (workgroup-uniform branch, taken by
        // every wave: it holds barriers).  One item loop for both cases keeps the kernel
        // small (a second inlined copy of the items measured slower).
        // (RPW = 2: the first half is ray A -- a split group restages at the ray boundary)
        // (split = 3: every quarter = item of the step is staged on its own)
        const int npart = cur.split + 1;
        int qn = 1, bnd = npart > 1 ? nsubw / npart : nsubw;  // the next part, its first item
        // ray epilogue of the wave's ray r: sums over the 16 sample lanes of every row
        auto ray_sums = [&](int r) {
            const float dsum = sd_rowsum16(dpart), wsum = sd_rowsum16(wpart);
            const float c0s = sd_rowsum16(cpart[0]), c1s = sd_rowsum16(cpart[1]),
                        c2s = sd_rowsum16(cpart[2]);
            uint8_t *hs = lds + ST_L_HS + (wave * RPW + r) * ST_HS_ROW;
            // the 32 hidden sums q = 4 t + r reduced over the 16 sample lanes of the row as a
            // butterfly (64 VALU ops instead of 32 x 4): bank-masked DPP halves the live
            // values at the first two levels, quad permutes finish -- lane bank b then holds
            // q = i + 8 b, i = 0..7 (hidden 16 (2 b + (i >> 2)) + 4 g + (i & 3))
            {
#if ST_HC16
                // the packed partial sums in the f32 [t][r] order of the butterfly
                float hacc[8][4];
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int t = 2 * s2 + (q >> 1), r = 2 * (q & 1);
                        // (from the bits: element extraction of the f16x2 array lost one
                        // conversion in an inlined copy of this epilogue, hipcc 7.2)
                        const uint32_t hb = __builtin_bit_cast(uint32_t, hacc16[4 * s2 + q]);
                        hacc[t][r] = (float)__builtin_bit_cast(_Float16, (uint16_t)(hb & 0xffffu));
                        hacc[t][r + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(hb >> 16));
                    }
#endif
                float u[16], v[8];
                // Every level-1 input is pinned in its register by two fence statements ("+v",
                // each with s_nop 1) before the first DPP: the compiler cannot schedule an
                // input's last VALU write (e.g. an f16 -> f32 conversion) right in front of the
                // DPP statement that reads it -- a VALU-write -> DPP-read hazard without the
                // two wait states, which it does not see inside inline asm (round 5: one
                // inlined copy of this epilogue read a packed f16 pair as f32).  Level 2 reads
                // u[i], u[i + 8], written by level-1 statements at least 14 ops earlier.
                asm volatile("s_nop 1" : "+v"(hacc[0][0]), "+v"(hacc[0][1]), "+v"(hacc[0][2]), "+v"(hacc[0][3]),
                             "+v"(hacc[1][0]), "+v"(hacc[1][1]), "+v"(hacc[1][2]), "+v"(hacc[1][3]),
                             "+v"(hacc[2][0]), "+v"(hacc[2][1]), "+v"(hacc[2][2]), "+v"(hacc[2][3]),
                             "+v"(hacc[3][0]), "+v"(hacc[3][1]), "+v"(hacc[3][2]), "+v"(hacc[3][3]));
                asm volatile("s_nop 1" : "+v"(hacc[4][0]), "+v"(hacc[4][1]), "+v"(hacc[4][2]), "+v"(hacc[4][3]),
                             "+v"(hacc[5][0]), "+v"(hacc[5][1]), "+v"(hacc[5][2]), "+v"(hacc[5][3]),
                             "+v"(hacc[6][0]), "+v"(hacc[6][1]), "+v"(hacc[6][2]), "+v"(hacc[6][3]),
                             "+v"(hacc[7][0]), "+v"(hacc[7][1]), "+v"(hacc[7][2]), "+v"(hacc[7][3]));
                ST_BFLY("s_nop 1\n\t", u[0], hacc[0][0], hacc[4][0], 8, 8, 0x3, 0xc);
#pragma unroll
                for (int i = 1; i < 16; ++i)
                    ST_BFLY("", u[i], hacc[i >> 2][i & 3], hacc[(i + 16) >> 2][i & 3], 8, 8, 0x3, 0xc);
#pragma unroll
                for (int i = 0; i < 8; ++i) ST_BFLY("", v[i], u[i], u[i + 8], 12, 4, 0x5, 0xa);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    v[i] += SD_DPP0(v[i], 0xb1);  // quad_perm [1, 0, 3, 2]
                    v[i] += SD_DPP0(v[i], 0x4e);  // quad_perm [2, 3, 0, 1]
                }
                if ((j & 3) == 0) {
                    const int b = j >> 2;
                    typedef typename Th::E EH;  // the head's operand type
                    *(uint2 *)(hs + (32 * b + 4 * g) * 2) =
                        uint2{sd_pack2<EH>(v[0], v[1]), sd_pack2<EH>(v[2], v[3])};
                    *(uint2 *)(hs + (32 * b + 16 + 4 * g) * 2) =
                        uint2{sd_pack2<EH>(v[4], v[5]), sd_pack2<EH>(v[6], v[7])};
                }
            }
            if (lane == 0) {
                *(float *)(lds + ST_L_WS + (wave * RPW + r) * 4) = wsum;
                st_out(a.depth + (int64_t)rmap(ray, r) * a.ld_depth, dsum);
                float *rp = a.rgb + (int64_t)rmap(ray, r) * a.ld_rgb;
                st_out(rp, c0s); st_out(rp + 1, c1s); st_out(rp + 2, c2s);
            }
        };
        for (int sub = 0; sub < nsubw; ++sub) {
            if (sub == bnd) {  // workgroup-uniform
                st_barrier_lds();  // every wave is done with the previous part's taps
                uint32_t mn1, mx1;
                box_union(buf, qn * NPART / npart, (qn + 1) * NPART / npart, mn1, mx1);
                ++qn;
                bnd = qn < npart ? qn * nsubw / npart : nsubw;
                cur = geom(mn1, mx1);  // fits (or is empty): checked when the split was chosen
                cur.ok = 1;
                dma(cur, buf, sbi);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_barrier_lds();
                lane_off = (uint32_t)((tq & 1) + (tq >> 1) * cur.pitch) * ST_TEX + 8u * (uint32_t)tp;
            }
            const int r = RPW == 1 ? 0 : sub / nsub;
            const bool act = cur.ok && rmap(ray, r) < R;
            if (act) {
                if (sub) itemA(sub, s0);
                itemB(sub, s0);
            }
            if (RPW > 1 && (sub + 1) % nsub == 0 && sub + 1 < nsubw) {  // ray r done
                if (act) ray_sums(r);
                reset();
            }
        }
        // this wave's LDS-DMA (next tile, ray words) landed -- waited here, in front of the
        // epilogue's output stores: vmcnt counts stores too, and a wait behind them held every
        // step for their acknowledgement (~1 memory latency)
        if (ST_WAIT_EARLY) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ST_T(6);
        if (cur.ok && rmap(ray, RPW - 1) < R) ray_sums(RPW - 1);
        if (cur.ok) {
            // per-sample outputs of the wave's RPW rays, lane = record k' (one coalesced store
            // per array)
#pragma unroll
            for (int p = 0; p < ST_MAXP; ++p) {
                const int kr = 64 * p + lane;
                const int rr = RPW == 1 ? 0 : min(kr / K, RPW - 1);
                const int k = kr - rr * K;
                if (64 * p < KW && kr < KW && rmap(ray, rr) < R) {
                    const int64_t rk = (int64_t)rmap(ray, rr) * K;
                    const f32x4 q1v = rq1(buf)[kr];
                    const uint4 q0v = rq0(buf)[kr];
                    const uint32_t fl = q0v.x >> 30;
                    if (a.weights) st_out(a.weights + rk + k, q1v[0]);
                    if (a.alphas) st_out(a.alphas + rk + k, q1v[1]);
                    if (a.invalid_f) a.invalid_f[rk + k] = (uint8_t)(fl & 1u);
                    if (a.invalid) st_out(a.invalid + rk + k, fl ? 1.f : 0.f);
                    if (a.rgb_samps) {
                        const float2 cgb = rqc(buf)[kr];
                        float *rsp = a.rgb_samps + (rk + k) * 3;
                        st_out(rsp, __builtin_bit_cast(float, q0v.w));
                        st_out(rsp + 1, cgb.x);
                        st_out(rsp + 2, cgb.y);
                    }
                }
            }
        }
        ST_T(7);
        prev_grp = grp;
        prev_ok = cur.ok;
        grp = ngrp;
        ray = nray;
        sbi = nsbi;
        cur = nxt;
        if (!ST_EARLY_FETCH && n + 2 < nsteps) ray_fetch(GR * (ngrp + nwg) + RPW * wave, buf);
        if (!ST_EARLY_HW && HPRE == 3 && prev_ok && wave < ndt) head_w(wave, hwn);  // the next head's W_dino
        if (!ST_WAIT_EARLY) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA landed
        ST_T(8);
        st_barrier_lds();  // Y: next tile complete; hsum of this group written
        ST_T(9);
    }
    if (threadIdx.x == 0) sa.ovf[blockIdx.x] = novf;
    if (prev_ok) {
        if (HPRE == 1) {
            HFrag hw[4];
            if (wave < ndt) head_w(wave, hw);
            head(prev_grp, hw);
        } else {
            head(prev_grp, hwn);  // (mode 3: loaded at the end of the last step)
        }
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

// rays per wave and step: 2 for K <= 32 (SDHIP_TILE_RPW=1 forces one, diagnostic A/B)
static int st_rpw(int K) {
    static const int force = getenv("SDHIP_TILE_RPW") ? atoi(getenv("SDHIP_TILE_RPW")) : 0;
    // SDHIP_TILE_RPW=2 also takes K = 64 two rays per wave (80 KiB of records, 37-KiB tile
    // buffers; A/B runs)
    const int kmax = force == 2 ? 64 : 32;
    return (K <= kmax && force != 1 && st_nw(K) == 8) ? 2 : 1;
}

static int st_lds_fixed(int K) {
    const int nw = st_nw(K), rpw = st_rpw(K);
    return st_l_rec(nw, rpw) + st_rec_bytes(nw, K * rpw);
}

// test hook (sd_render_tile_cap): tile buffers capped at this many bytes, 0 = no cap
static int st_cap_bytes = 0;
extern "C" int32_t sd_render_tile_cap(int32_t bytes) {
    const int prev = st_cap_bytes;
    st_cap_bytes = bytes > 0 ? bytes : 0;
    return prev;
}

static int st_tile_bytes(int K) {
    const int avail = 160 * 1024 - st_lds_fixed(K);
    const int b = ((avail / 2) / 1024) * 1024;
    return st_cap_bytes ? min(b, (st_cap_bytes / 1024) * 1024) : b;
}

// Can the tile kernel take this render?  (colour in exactly one render view, batches of
// whole groups, K <= 128, room for one tile buffer pair.)
extern "C" int sd_render_tile_ok(const sd_render_args *a, const sd_head *m) {
    return a->nv == 1 && a->K % 16 == 0 && a->K <= 128 &&
           a->rays_per_sb % (st_nw(a->K) * st_rpw(a->K)) == 0 &&
           m->D % 16 == 0 && m->D <= 512 && a->Wf < 32768 && a->Hf < 32768 &&
           st_tile_bytes(a->K) >= 16 * 1024;
}

// Launch; ovf: device int32 [sd_ovf_words(R, sd_num_cus())] (the per-workgroup overflow
// lists, sdhip_render.h; every count written by the kernel).
extern "C" int sd_render_tile_launch(const sd_render_args *a, const sd_head *m, int32_t *ovf,
                                     void *stream) {
    hipStream_t s = (hipStream_t)stream;
    st_args sa;
    sa.a = *a;
    sa.m = *m;
    sa.ovf = ovf;
    const int ncu = sd_num_cus();
    sa.ovf_cap = (int32_t)sd_ovf_cap(a->R, ncu);
    const int nw = st_nw(a->K), rpw = st_rpw(a->K);
    sa.ngroups = (int)((a->R + nw * rpw - 1) / (nw * rpw));
    sa.tile_bytes = st_tile_bytes(a->K);
    const int lds_bytes = st_lds_fixed(a->K) + 2 * sa.tile_bytes;
    auto go = [&](auto kern) {
        sd_lds_attr((const void *)kern, lds_bytes);
        hipLaunchKernelGGL(kern, dim3((unsigned)ncu), dim3(64 * nw), lds_bytes, s, sa);
    };
    const bool zin = a->z != nullptr;
#define ST_GO(NWV, RPWV)                                                                              \
    if (m->dtype == SD_F16) {                                                                         \
        if (zin) go(k_render_tile<SD_F16, true, NWV, RPWV>); else go(k_render_tile<SD_F16, false, NWV, RPWV>); \
    } else {                                                                                          \
        if (zin) go(k_render_tile<SD_BF16, true, NWV, RPWV>); else go(k_render_tile<SD_BF16, false, NWV, RPWV>); \
    }
    if (nw == 8 && rpw == 2) {
        ST_GO(8, 2)
    } else if (nw == 8) {
        ST_GO(8, 1)
    } else {
        ST_GO(ST_NW_SMALLK, 1)
    }
#undef ST_GO
    return sd_check_last("sd_render_proj (tile kernel)");
}
