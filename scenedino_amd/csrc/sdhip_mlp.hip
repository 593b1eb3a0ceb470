// sdhip_mlp.hip -- the ResnetFC field MLP of the training path (resnetfc.py:135-203 with
// n_blocks = 0, under the reference's with_amp autocast: base_trainer.py:223,251) as two
// fused MFMA kernels on the gather rows x = [feat (C) | code (39) | 1]:
//
//   k_mlp_fwd : H^T = relu(W1 X^T) (W1 = [W_in | b_in]: the ones column carries the bias),
//               out = H W_o^T + b_o, sigma = softplus(out_0) (bts.py:516-541, threshold 20),
//               dino = out_1..D; H is kept (16-bit, + a ones column) for the backward.
//   k_mlp_bwd : dY = [d dino | d sigma . sigmoid(out_0)], dH^T = (W_o^T dY^T) * [H > 0],
//               dX = dH W_in[:, :C] (f32 rows for sd_field_gather_bwd, or -- dgrid set --
//               scattered straight into the grid gradient, ml_scatter); dY and dH rows are
//               written for the weight-gradient GEMMs (dW1 = dH^T X, dW_o = dY^T [H | 1]).
//
// Work unit: one wave = 32 points (MFMA v_mfma_f32_32x32x16_{f16,bf16}), 8 waves per
// persistent workgroup (one per CU, 2 waves per SIMD); weights staged once per workgroup in LDS as pre-packed 1-KiB fragments (scenedino_amd/mlp_pack.py,
// PackedTrainMLP).  An accumulator tile is re-used in registers as the next product's
// operand: its rows 32 t + 8 (i >> 2) + 4 h + (i & 3) become the k order
// kappa(s, h, j) = 16 s + 8 (j >> 2) + 4 h + (j & 3) of k-step s, which the host packing of
// the partner operand follows -- no LDS round trip, no shuffles.
#include "sdhip_common.h"
#include "sdhip_render.h"

extern "C" void sd_set_error(const char *msg);

#define ML_WAVES 8  // 2 waves per SIMD share one LDS copy of the weights (~100 KiB: 1 workgroup per CU)
#define ML_DH 128
#define ML_HLD 136  // H row: 128 hidden, the ones column, 7 zeros (16-B aligned rows)
#define ML_DYLD 72  // dY row: D dino (<= 64) ... d out_0, zeros
#define ML_MAXKS 20  // k-steps of x held in registers (kx <= 320)
#define ML_MAXKO ((ML_DYLD + 15) / 16)  // k-steps over the outputs (D + 1 <= 72)
#ifndef ML_FWD_BUF
#define ML_FWD_BUF 1
#endif

template <int P>
__device__ __forceinline__ typename T16<P>::Frag ml_frag(const f32x16 &acc, int c) {
    // registers 8 c .. 8 c + 7 of an accumulator tile as a 16-bit operand fragment
    typedef typename T16<P>::E E;
    typename T16<P>::Frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (E)acc[8 * c + j];
    return f;
}

__device__ __forceinline__ float ml_softplus(float x) { return x > 20.f ? x : log1pf(expf(x)); }

template <int P>
__global__ void __launch_bounds__(ML_WAVES * 64) k_mlp_fwd(const sd_mlp_train_args a) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    typedef typename Tr::E E;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int KS = (a.kx + 15) >> 4;
    const int U = (a.D + 1 + 31) >> 5;
    const int n1 = 4 * KS * 64, n2 = U * 8 * 64;  // 16-B entries
    {
        const uint4 *s1 = (const uint4 *)a.w1f, *s2 = (const uint4 *)a.w2f;
        uint4 *d = (uint4 *)lds;
        for (int i = threadIdx.x; i < n1; i += blockDim.x) d[i] = s1[i];
        for (int i = threadIdx.x; i < n2; i += blockDim.x) d[n1 + i] = s2[i];
        __syncthreads();
    }
    const Frag *w1 = (const Frag *)lds;
    const Frag *w2 = w1 + n1;
    const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int64_t ntile = (a.N + 31) >> 5;
    const __amdgpu_buffer_rsrc_t rx =
        sd_rsrc(a.x, (uint32_t)((a.N * a.ldx) * (int64_t)sizeof(E)));
    // the output stores go through buffers with out-of-range points past the end (dropped)
    // and every value in a register of its own, the output biases loaded once up front: no
    // store drains the memory counter for the next (ML_FWD_BUF 0: the per-element stores)
    const bool obuf = ML_FWD_BUF && a.N * a.D < ((int64_t)1 << 29);
    const __amdgpu_buffer_rsrc_t rdn = sd_rsrc(a.dino, obuf ? (uint32_t)(a.N * a.D * 4) : 0u);
    const __amdgpu_buffer_rsrc_t rsg = sd_rsrc(a.sigma, obuf ? (uint32_t)(a.N * 4) : 0u);
    float bdv[(ML_DYLD + 31) / 32];
#pragma unroll
    for (int u = 0; u < (ML_DYLD + 31) / 32; ++u) {
        const int col = 32 * u + r;
        bdv[u] = (u < U && col < a.D) ? a.b_out[1 + col] : 0.f;
    }
    const float bsg = a.b_out[0];
    for (int64_t tile = (int64_t)blockIdx.x * ML_WAVES + wave; tile < ntile;
         tile += (int64_t)gridDim.x * ML_WAVES) {
        const int64_t p0 = tile * 32;
        const int64_t pt = p0 + r;
        const bool valid = pt < a.N;
        // layer 1 (the bias rides on the ones column of x)
        f32x16 acc[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
        // the whole 32-row x tile in flight at once (one 16-B piece per k-step per lane)
        const uint32_t xo = (uint32_t)(((valid ? pt : a.N - 1) * a.ldx + 8 * h) * sizeof(E));
        uint4 xs[ML_MAXKS];
#pragma unroll
        for (int s = 0; s < ML_MAXKS; ++s)
            if (s < KS)
                xs[s] = __builtin_bit_cast(
                    uint4, __builtin_amdgcn_raw_buffer_load_b128(rx, xo + 32 * s, 0, 0));
#pragma unroll
        for (int s = 0; s < ML_MAXKS; ++s)
            if (s < KS) {
                const Frag xb = __builtin_bit_cast(Frag, xs[s]);
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    acc[t] = Tr::mma32(w1[(t * KS + s) * 64 + lane], xb, acc[t]);
            }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[t][i] = fmaxf(acc[t][i], 0.f);
        if (valid) {  // H row: hidden 32 t + 8 g + 4 h + 0..3 of this lane's point
            E *hr = (E *)a.h + pt * ML_HLD;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    *(uint2 *)(hr + 32 * t + 8 * g + 4 * h) =
                        uint2{sd_pack2<E>(acc[t][4 * g], acc[t][4 * g + 1]),
                              sd_pack2<E>(acc[t][4 * g + 2], acc[t][4 * g + 3])};
            *(uint2 *)(hr + 128 + 4 * h) = uint2{h == 0 ? sd_pack2<E>(1.f, 0.f) : 0u, 0u};
        }
        // layer 2: out = H W_o^T, A = H (rows = points) straight from the accumulators
        Frag af[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) af[s] = ml_frag<P>(acc[s >> 1], s & 1);
#pragma unroll
        for (int u = 0; u < (ML_DYLD + 31) / 32; ++u) {  // (U <= 3: D + 1 <= 72)
            if (u >= U) break;
            f32x16 o;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] = 0.f;
#pragma unroll
            for (int s = 0; s < 8; ++s) o = Tr::mma32(af[s], w2[(u * 8 + s) * 64 + lane], o);
            // o: row = point p0 + 8 (i >> 2) + 4 h + (i & 3), column = output 32 u + r
            // (outputs 0 .. D-1 = dino, D = sigma)
            const int col = 32 * u + r;
            if (obuf) {
                float vd[16], vs[16];
                uint32_t od[16], os[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t p = p0 + 8 * (i >> 2) + 4 * h + (i & 3);
                    const bool pin = p < a.N;
                    vd[i] = o[i] + bdv[u];
                    od[i] = (pin && col < a.D) ? (uint32_t)((p * a.D + col) * 4) : 0x80000000u;
                    os[i] = (pin && col == a.D) ? (uint32_t)(p * 4) : 0x80000000u;
                }
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, vd[i]), rdn, od[i], 0, 0);
                if (32 * u + 32 > a.D) {  // the tile holding sigma (wave-uniform)
#pragma unroll
                    for (int i = 0; i < 16; ++i) vs[i] = ml_softplus(o[i] + bsg);
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, vs[i]), rsg, os[i], 0, 0);
                }
                continue;
            }
            if (col < a.D) {
                const float bd = a.b_out[1 + col];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t p = p0 + 8 * (i >> 2) + 4 * h + (i & 3);
                    if (p < a.N) a.dino[p * a.D + col] = o[i] + bd;
                }
            } else if (col == a.D) {
                const float bs = a.b_out[0];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t p = p0 + 8 * (i >> 2) + 4 * h + (i & 3);
                    if (p < a.N) a.sigma[p] = ml_softplus(o[i] + bs);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Fused grid_sample backward of k_mlp_bwd (dgrid != NULL; bts.py:299-309).  The scatter is
// a product, G = S dX: S (rows = the distinct texels the wave's 32 points tap with a nonzero
// bilinear weight, columns = the points) holds at (texel, point) the sum of the point's
// weights of its taps on that texel, and dX (32 points x 32 channels) is the accumulator
// tile of dX = dH W_in re-used in registers as the B operand -- rounded to the autocast
// dtype, the dtype of the reference's Linear input gradient.  S enters as hi + lo 16-bit
// parts (the weights keep >= 16 bits).  Each nonzero G element is one f32 atomic add into
// the grid gradient.  One row per distinct texel, not per (run of equal tap quads, tap):
// a ray's samples straddle texel borders through rounding (encoder view) or walk along an
// epipolar line (other views), and consecutive quads share texels -- 3.5 rows per wave
// instead of 20.6 on the bench's encoder-view rays (the float atomics run at ~1.3 TB/s of
// added bytes chip-wide, microarch guide: they were most of this kernel's time).
// Per-wave LDS tables: w[32][4] f32 (each point's four tap weights), row[32] (the S row of
// each tap, one byte each, 0xff = none), off[128] (each row's element offset in dgrid).
// ---------------------------------------------------------------------------
#define ML_SCR_WORDS (4 * 32 + 32 + 128)
#ifndef ML_DIAG_NO_ATOMICS
#define ML_DIAG_NO_ATOMICS 0  // diagnostic builds only (tools/build_variant.py): drop the grid-gradient atomics
#endif

__device__ __forceinline__ void ml_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// tables of the wave's tile (at the tile start, while the dY loads are in flight);
// returns the number of S rows (distinct texels, <= 128)
__device__ __forceinline__ int ml_scatter_tables(const sd_mlp_train_args &a, int *scr,
                                                 int64_t pt, bool valid, int lane) {
    const int h = lane >> 5, r = lane & 31;
    float *sw = (float *)scr;
    uint16_t *srow = (uint16_t *)(scr + 128);
    int *soff = scr + 160;
    // geometry of point pt (both halves; the forward gather's sd_point_geo, same taps);
    // lane half h owns taps 2 h and 2 h + 1
    int key[2] = {-1, -1};
    float gw[2] = {0.f, 0.f};
    if (valid) {
        const int64_t b = pt / a.P;
        const PointGeo geo = sd_point_geo(a.cam_f + b * SD_CAM_WORDS, a.xyz[pt * 3],
                                          a.xyz[pt * 3 + 1], a.xyz[pt * 3 + 2], a.Wf, a.Hf);
        const int base = (int)b * a.Hf * a.Wf;
        const int i0 = h ? geo.t.i10 : geo.t.i00, i1 = h ? geo.t.i11 : geo.t.i01;
        gw[0] = h ? geo.t.w10 : geo.t.w00;
        gw[1] = h ? geo.t.w11 : geo.t.w01;
        key[0] = gw[0] != 0.f ? base + i0 : -1;  // a zero weight adds nothing: no row
        key[1] = gw[1] != 0.f ? base + i1 : -1;
    }
    // rows in order of first appearance: each pass takes the first unassigned key of the
    // wave and gives every equal key its row (passes = distinct texels)
    int row[2] = {-1, -1};
    int nrow = 0;
    ml_wave_sync();  // the previous tile's table reads are done
    for (;;) {
        const uint64_t m0 = __ballot(key[0] >= 0 && row[0] < 0);
        const uint64_t m1 = __ballot(key[1] >= 0 && row[1] < 0);
        if (!(m0 | m1)) break;
        const int kv = m0 ? __builtin_amdgcn_readlane(key[0], __builtin_ctzll(m0))
                          : __builtin_amdgcn_readlane(key[1], __builtin_ctzll(m1));
        if (key[0] == kv) row[0] = nrow;
        if (key[1] == kv) row[1] = nrow;
        if (lane == 0) soff[nrow] = kv * a.C;
        ++nrow;
    }
    *(float2 *)(sw + 4 * r + 2 * h) = make_float2(gw[0], gw[1]);
    srow[2 * r + h] = (uint16_t)((row[0] & 0xff) | (row[1] & 0xff) << 8);
    ml_wave_sync();
    return nrow;
}

// S fragments of row tile mt (A operand in the k order kappa of ml_frag: k-step s, lane
// half h, element j = point 16 s + 8 (j >> 2) + 4 h + (j & 3)); row 32 mt + r
template <int P>
__device__ __forceinline__ void ml_s_frags(const int *scr, int mt, int lane,
                                           typename T16<P>::Frag (&sh)[2],
                                           typename T16<P>::Frag (&sl)[2]) {
    typedef typename T16<P>::E E;
    const int h = lane >> 5, r = lane & 31;
    const float4 *sw = (const float4 *)scr;
    const uint32_t *srow = (const uint32_t *)(scr + 128);
    const uint32_t k = 32 * mt + r;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            // four elements' table reads at a time (all 16 hoisted: 80 live registers, spills)
            if ((j & 3) == 0) __builtin_amdgcn_sched_barrier(0);
            const int q = 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            const float4 w4 = sw[q];
            const uint32_t rq = srow[q];
            float w = (rq & 0xffu) == k ? w4.x : 0.f;
            w += ((rq >> 8) & 0xffu) == k ? w4.y : 0.f;
            w += ((rq >> 16) & 0xffu) == k ? w4.z : 0.f;
            w += (rq >> 24) == k ? w4.w : 0.f;
            const E hi = (E)w;
            sh[s][j] = hi;
            sl[s][j] = (E)(w - (float)hi);
        }
}

// G = S dX for one 32-channel column tile and row tile mt, and its atomics.  The G row of
// this lane's element i: 32 mt + 8 (i >> 2) + 4 h + (i & 3).
template <int P>
__device__ __forceinline__ void ml_s_emit(const int *scr, int mt, int nr, int lane,
                                          const typename T16<P>::Frag (&sh)[2],
                                          const typename T16<P>::Frag (&sl)[2],
                                          const typename T16<P>::Frag &b0,
                                          const typename T16<P>::Frag &b1, float *dg) {
    typedef T16<P> Tr;
    const int h = lane >> 5;
    const int *soff = scr + 160;
    f32x16 g;
#pragma unroll
    for (int i = 0; i < 16; ++i) g[i] = 0.f;
    g = Tr::mma32(sh[0], b0, g);
    g = Tr::mma32(sh[1], b1, g);
    g = Tr::mma32(sl[0], b0, g);
    g = Tr::mma32(sl[1], b1, g);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int kk = 32 * mt + 8 * (i >> 2) + 4 * h + (i & 3);
        if (kk < nr && g[i] != 0.f && !ML_DIAG_NO_ATOMICS) unsafeAtomicAdd(dg + soff[kk], g[i]);
    }
}

// dX = dH W_in, 32 channels at a time, each tile straight into ml_s_emit
template <int P>
__device__ __forceinline__ void ml_scatter(const sd_mlp_train_args &a,
                                           const typename T16<P>::Frag (&af)[8],
                                           const typename T16<P>::Frag *wx, const int *scr,
                                           int nr, int lane) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    const int r = lane & 31;
    Frag s0h[2], s0l[2];
    ml_s_frags<P>(scr, 0, lane, s0h, s0l);
    const int nmt = (nr + 31) >> 5;
    const int UC = a.C >> 5;
    for (int u = 0; u < UC; ++u) {
        f32x16 o;
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] = 0.f;
#pragma unroll
        for (int s = 0; s < 8; ++s) o = Tr::mma32(af[s], wx[(u * 8 + s) * 64 + lane], o);
        const Frag b0 = ml_frag<P>(o, 0), b1 = ml_frag<P>(o, 1);
        float *dg = a.dgrid + 32 * u + r;
        ml_s_emit<P>(scr, 0, nr, lane, s0h, s0l, b0, b1, dg);
        for (int mt = 1; mt < nmt; ++mt) {  // more than 32 texels: points off the encoder view
            Frag sh[2], sl[2];
            ml_s_frags<P>(scr, mt, lane, sh, sl);
            ml_s_emit<P>(scr, mt, nr, lane, sh, sl, b0, b1, dg);
        }
    }
}

template <int P, bool SCAT>
__global__ void __launch_bounds__(ML_WAVES * 64) k_mlp_bwd(const sd_mlp_train_args a) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    typedef typename Tr::E E;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int KO = (a.D + 1 + 15) >> 4;  // k-steps over the outputs (dino, then out_0)
    const int UC = a.C >> 5;             // 32-column tiles of dX
    const int n1 = 4 * KO * 64, n2 = UC * 8 * 64;
    {
        const uint4 *s1 = (const uint4 *)a.wtf, *s2 = (const uint4 *)a.wxf;
        uint4 *d = (uint4 *)lds;
        for (int i = threadIdx.x; i < n1; i += blockDim.x) d[i] = s1[i];
        for (int i = threadIdx.x; i < n2; i += blockDim.x) d[n1 + i] = s2[i];
        __syncthreads();
    }
    const Frag *wt = (const Frag *)lds;
    const Frag *wx = wt + n1;
    int *scr = (int *)(lds + (n1 + n2) * 16);  // per-wave scatter tables (ml_scatter)
    const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    const int wave = threadIdx.x >> 6;
    const int64_t ntile = (a.N + 31) >> 5;
    for (int64_t tile = (int64_t)blockIdx.x * ML_WAVES + wave; tile < ntile;
         tile += (int64_t)gridDim.x * ML_WAVES) {
        const int64_t p0 = tile * 32;
        const int64_t pt = p0 + r;
        const bool valid = pt < a.N;
        const int64_t pc = valid ? pt : a.N - 1;
        // dY^T as B operand: lane (point r, half h), k-step s: dY[point][16 s + 8 h + j]
        int *wscr = scr + wave * ML_SCR_WORDS;
        const int nr = SCAT ? ml_scatter_tables(a, wscr, pt, valid, lane) : 0;
        const float sg = a.sigma[pc];
        const float dsg = valid ? a.d_sigma[pc] * (1.f - expf(-sg)) : 0.f;  // softplus'
        E *dyr = (E *)a.dy + pt * ML_DYLD;
        f32x16 dh[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int i = 0; i < 16; ++i) dh[t][i] = 0.f;
        // the lane's dY pieces (8 consecutive dino values per k-step, 16-B loads) and its
        // saved H values, all issued before the first use
        float4 dd[2 * ML_MAXKO];
#pragma unroll
        for (int s = 0; s < ML_MAXKO; ++s)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int k = 16 * s + 8 * h + 4 * q;
                dd[2 * s + q] = (k + 4 <= a.D) ? *(const float4 *)(a.d_dino + pc * a.D + k)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        const E *hr = (const E *)a.h + pc * ML_HLD;
        uint2 hv[16];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) hv[4 * t + g] = *(const uint2 *)(hr + 32 * t + 8 * g + 4 * h);
#pragma unroll
        for (int s = 0; s < ML_MAXKO; ++s) {
            if (s >= KO) break;
            float v[8];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float4 d4 = dd[2 * s + q];
                v[4 * q] = d4.x; v[4 * q + 1] = d4.y; v[4 * q + 2] = d4.z; v[4 * q + 3] = d4.w;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 16 * s + 8 * h + j;
                if (k == a.D) v[j] = dsg;
                if (!valid) v[j] = 0.f;
            }
            Frag f;
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = (E)v[j];
            if (valid && 16 * s + 8 * h < ML_DYLD)
                *(uint4 *)(dyr + 16 * s + 8 * h) = __builtin_bit_cast(uint4, f);
#pragma unroll
            for (int t = 0; t < 4; ++t) dh[t] = Tr::mma32(wt[(t * KO + s) * 64 + lane], f, dh[t]);
        }
        // ReLU mask from the saved H (this lane's hidden 32 t + 8 g + 4 h + 0..3)
        E *dhr = (E *)a.dh + pt * ML_DH;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint2 hq = hv[4 * t + g];
                const float h0 = sd_unpack_lo<P>(hq.x), h1 = sd_unpack_hi<P>(hq.x);
                const float h2 = sd_unpack_lo<P>(hq.y), h3 = sd_unpack_hi<P>(hq.y);
                dh[t][4 * g] = h0 > 0.f ? dh[t][4 * g] : 0.f;
                dh[t][4 * g + 1] = h1 > 0.f ? dh[t][4 * g + 1] : 0.f;
                dh[t][4 * g + 2] = h2 > 0.f ? dh[t][4 * g + 2] : 0.f;
                dh[t][4 * g + 3] = h3 > 0.f ? dh[t][4 * g + 3] : 0.f;
                if (valid)
                    *(uint2 *)(dhr + 32 * t + 8 * g + 4 * h) =
                        uint2{sd_pack2<E>(dh[t][4 * g], dh[t][4 * g + 1]),
                              sd_pack2<E>(dh[t][4 * g + 2], dh[t][4 * g + 3])};
            }
        if constexpr (!SCAT) {
            if (!a.dx) continue;  // the caller needs no input gradient: dH / dY only
        }
        // dX = dH W_in[:, :C]: A = dH (rows = points) from the accumulators
        Frag af[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) af[s] = ml_frag<P>(dh[s >> 1], s & 1);
        if constexpr (SCAT) {  // fused grid_sample backward: no dX rows
            ml_scatter<P>(a, af, wx, wscr, nr, lane);
            continue;
        }
        for (int u = 0; u < UC; ++u) {
            f32x16 o;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] = 0.f;
#pragma unroll
            for (int s = 0; s < 8; ++s) o = Tr::mma32(af[s], wx[(u * 8 + s) * 64 + lane], o);
            const int col = 32 * u + r;
            if (a.dx_dtype == SD_F32) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t p = p0 + 8 * (i >> 2) + 4 * h + (i & 3);
                    if (p < a.N) ((float *)a.dx)[p * a.lddx + col] = o[i];
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t p = p0 + 8 * (i >> 2) + 4 * h + (i & 3);
                    if (p < a.N) ((E *)a.dx)[p * a.lddx + col] = (E)o[i];
                }
            }
        }
        // the code / ones columns of dX (if the caller's rows have them) carry no gradient
        for (int c = a.C + lane; c < a.lddx; c += 64)
            for (int i = 0; i < 32; ++i) {
                const int64_t p = p0 + i;
                if (p < a.N) {
                    if (a.dx_dtype == SD_F32) ((float *)a.dx)[p * a.lddx + c] = 0.f;
                    else ((E *)a.dx)[p * a.lddx + c] = (E)0.f;
                }
            }
    }
}

static int ml_check(const sd_mlp_train_args *a, bool bwd) {
    if (!a || a->N < 0 || (a->dtype != SD_F16 && a->dtype != SD_BF16) || a->kx <= 0 ||
        a->kx > a->ldx || a->kx > 16 * ML_MAXKS || a->ldx % 8 || a->D <= 0 || a->D > 64 || a->D % 8 || a->C <= 0 || a->C % 32 ||
        a->C > a->kx || a->N * a->ldx * 2 >= (1LL << 32))
        return 0;
    if (!bwd) return a->x && a->w1f && a->w2f && a->b_out && a->h && a->sigma && a->dino;
    if (!(a->wtf && a->wxf && a->h && a->sigma && a->d_sigma && a->d_dino && a->dy && a->dh))
        return 0;
    if (a->dgrid)  // fused scatter: the frame / grid geometry of the forward gather
        return a->xyz && a->cam_f && a->P > 0 && a->N % a->P == 0 && a->Hf > 0 && a->Wf > 0 &&
               (a->N / a->P) * a->Hf * a->Wf * (int64_t)a->C < (1LL << 31);
    if (!a->dx) return 1;  // no dX wanted (weight gradients only)
    return a->lddx >= a->C && a->lddx <= a->ldx &&
           (a->dx_dtype == SD_F32 || a->dx_dtype == a->dtype);
}

template <typename K>
static int ml_launch(K kern, const sd_mlp_train_args *a, int lds_bytes, hipStream_t s) {
    if (lds_bytes > 160 * 1024) {
        sd_set_error("sd_mlp_train: packed weights exceed the 160 KiB LDS");
        return -1;
    }
    sd_lds_attr((const void *)kern, 160 * 1024);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t tiles = (a->N + 31) / 32;
    int64_t nblk = (tiles + ML_WAVES - 1) / ML_WAVES;
    // weights are staged once per workgroup: persistent, one workgroup per CU
    if (nblk > (int64_t)cus) nblk = (int64_t)cus;
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(ML_WAVES * 64), lds_bytes, s, *a);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_mlp_train: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_mlp_train_fwd(const sd_mlp_train_args *a, void *stream) {
    if (!ml_check(a, false)) {
        sd_set_error("sd_mlp_train_fwd: invalid argument (16-bit dtype, D <= 64, D % 8 == 0, "
                     "C % 32 == 0, ldx % 8 == 0, kx <= 320)");
        return -1;
    }
    if (a->N == 0) return 0;
    const int KS = (a->kx + 15) / 16, U = (a->D + 1 + 31) / 32;
    const int lds = (4 * KS + U * 8) * 64 * 16;
    if (a->dtype == SD_F16) return ml_launch(k_mlp_fwd<SD_F16>, a, lds, (hipStream_t)stream);
    return ml_launch(k_mlp_fwd<SD_BF16>, a, lds, (hipStream_t)stream);
}

extern "C" int sd_mlp_train_bwd(const sd_mlp_train_args *a, void *stream) {
    if (!ml_check(a, true)) {
        sd_set_error("sd_mlp_train_bwd: invalid argument");
        return -1;
    }
    if (a->N == 0) return 0;
    const int KO = (a->D + 1 + 15) / 16;
    const int lds = (4 * KO + (a->C / 32) * 8) * 64 * 16 + ML_WAVES * ML_SCR_WORDS * 4;
    hipStream_t s = (hipStream_t)stream;
    if (a->dgrid)
        return a->dtype == SD_F16 ? ml_launch(k_mlp_bwd<SD_F16, true>, a, lds, s)
                                  : ml_launch(k_mlp_bwd<SD_BF16, true>, a, lds, s);
    return a->dtype == SD_F16 ? ml_launch(k_mlp_bwd<SD_F16, false>, a, lds, s)
                              : ml_launch(k_mlp_bwd<SD_BF16, false>, a, lds, s);
}

// ---------------------------------------------------------------------------
// weight gradients of the training MLP: C = A^T B over the N points, A (N, Ma) and B (N, Nb)
// 16-bit rows (dW1 = dH^T X, dW_o = dY^T [H | 1]).  A workgroup (4 waves) sums a contiguous
// range of points into a partial (Ma x Nb) f32 tile set; the partials are summed by the
// caller (deterministic).  Both operands have k = points, the slow axis of their rows: each
// 32-point chunk is staged row-major in LDS and read back transposed by
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, delivered column-major), so
// lane (row / column r, half h) gets the 8 points 8 h .. 8 h + 7 of its row / column.
// Wave w owns output row tile w (Ma <= 128) and every column tile (its A fragment re-used
// across the row).
// ---------------------------------------------------------------------------
#define WG_MAXT 10  // column tiles per wave (Nb <= 320)
#define WG_MAXLD 8  // 16-B staging loads per thread per 32-point chunk

typedef __attribute__((ext_vector_type(4))) short wg_s16x4;

__device__ __forceinline__ uint2 wg_tr(const void *lds_addr) {
    const wg_s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) wg_s16x4 *)(uintptr_t)lds_addr);
    return __builtin_bit_cast(uint2, v);
}

template <int P, int NT>
__global__ void __launch_bounds__(256) k_wgrad(const sd_wgrad_args g) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int MaP = (g.Ma + 31) & ~31, NbP = (g.Nb + 31) & ~31;
    // column split blockIdx.y: columns [nb0, nb0 + nbw) of B, NT tiles of 32
    const int nb0 = blockIdx.y * NT * 32;
    const int nbw = g.Nb - nb0 < NT * 32 ? g.Nb - nb0 : NT * 32;
    const int rsa = MaP + 8, rsb = NT * 32 + 8;  // LDS row strides (elements; 16-B multiples)
    uint16_t *sA = (uint16_t *)lds;
    uint16_t *sB = sA + 32 * rsa;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int mt = MaP >> 5;
    // zero the padding columns once (loads never write them)
    for (int i = tid; i < 32 * rsa; i += 256) sA[i] = 0;
    for (int i = tid; i < 32 * rsb; i += 256) sB[i] = 0;
    __syncthreads();
    // this workgroup's points [p_lo, p_hi)
    const int64_t per = (g.N + gridDim.x - 1) / gridDim.x;
    const int64_t p_lo = (int64_t)blockIdx.x * per;
    const int64_t p_hi = p_lo + per < g.N ? p_lo + per : g.N;
    // 16-B chunks of one 32-row chunk: A (32 x Ma), B (32 x Nb)
    const int ca = g.Ma / 8, cb = nbw / 8;  // chunks per row (Ma, Nb multiples of 8)
    const int nca = 32 * ca, ncb = 32 * cb;
    const int nld = (nca + ncb + 255) / 256;  // loads per thread
    // transposed-read lane address: group G = lane >> 4 (col base 16 (G & 1), k base
    // 8 (G >> 1)), lane 4 q + p of the group: row (k) kb + q, columns cb + 4 p .. + 3
    const int G = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int kb = 8 * (G >> 1), cbase = 16 * (G & 1) + 4 * pp;
    // wave w owns output row tile w (Ma <= 128) and all NT column tiles
    const bool own = wave < mt;
    f32x16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    // staged chunk pieces (nld <= WG_MAXLD), two sets: chunk k + 2 loads while chunk k is
    // multiplied (one set in flight left each chunk's MFMAs waiting on a memory round trip)
    uint4 st0[WG_MAXLD], st1[WG_MAXLD];
    uint32_t ok0 = 0, ok1 = 0;  // which pieces are real (the zeros are applied at the LDS store)
    // every load issued unconditionally (invalid lanes read the first row, dropped at the
    // LDS store), so the count in flight is static and the wait for one set leaves the
    // other in flight
    auto gload = [&](uint4 (&st)[WG_MAXLD], uint32_t &okm, int64_t p0) {
        okm = 0;
#pragma unroll
        for (int i = 0; i < WG_MAXLD; ++i) {
            const int c = tid + 256 * i;
            const bool isa = c < nca;
            const int cc = isa ? c : c - nca;
            const int row = isa ? c / ca : cc / cb;
            const int col = isa ? (c - row * ca) * 8 : nb0 + (cc - row * cb) * 8;
            const int64_t p = p0 + row;
            const bool ok = i < nld && c < nca + ncb && p < p_hi;
            const uint16_t *src = !ok ? (const uint16_t *)g.a
                                      : isa ? (const uint16_t *)g.a + p * g.lda + col
                                            : (const uint16_t *)g.b + p * g.ldb + col;
            st[i] = *(const uint4 *)src;
            okm |= ok ? 1u << i : 0u;
        }
    };
    auto lstore = [&](const uint4 (&st)[WG_MAXLD], uint32_t okm) {
#pragma unroll
        for (int i = 0; i < WG_MAXLD; ++i) {
            const int c = tid + 256 * i;
            if (i < nld && c < nca + ncb) {
                const uint4 v = (okm >> i) & 1u ? st[i] : uint4{0u, 0u, 0u, 0u};
                if (c < nca) {
                    const int row = c / ca, col = (c - row * ca) * 8;
                    *(uint4 *)(sA + row * rsa + col) = v;
                } else {
                    const int cc = c - nca, row = cc / cb, col = (cc - row * cb) * 8;
                    *(uint4 *)(sB + row * rsb + col) = v;
                }
            }
        }
    };
    auto compute = [&]() {
        if (own) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {  // two k-steps of 16 points
                const uint16_t *ra = sA + (16 * s + kb + q) * rsa + 32 * wave + cbase;
                const uint2 a0 = wg_tr(ra), a1 = wg_tr(ra + 4 * rsa);
                const Frag af = __builtin_bit_cast(Frag, uint4{a0.x, a0.y, a1.x, a1.y});
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const uint16_t *rb = sB + (16 * s + kb + q) * rsb + 32 * j + cbase;
                    const uint2 b0 = wg_tr(rb), b1 = wg_tr(rb + 4 * rsb);
                    const Frag bf = __builtin_bit_cast(Frag, uint4{b0.x, b0.y, b1.x, b1.y});
                    acc[j] = Tr::mma32(af, bf, acc[j]);
                }
            }
        }
    };
    if (p_lo < p_hi) gload(st0, ok0, p_lo);
    if (p_lo + 32 < p_hi) gload(st1, ok1, p_lo + 32);
    for (int64_t p0 = p_lo; p0 < p_hi; p0 += 64) {
        __syncthreads();  // the previous chunk's reads are done
        lstore(st0, ok0);
        __syncthreads();
        if (p0 + 64 < p_hi) gload(st0, ok0, p0 + 64);
        compute();
        if (p0 + 32 >= p_hi) break;  // workgroup-uniform
        __syncthreads();
        lstore(st1, ok1);
        __syncthreads();
        if (p0 + 96 < p_hi) gload(st1, ok1, p0 + 96);
        compute();
    }
    // partial tile: acc[i][j] register e = C[32 ti + 8 (e >> 2) + 4 h + (e & 3)][32 j + r]
    float *out = g.part + (int64_t)blockIdx.x * MaP * NbP;
    if (own) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e)
                if (32 * j < nbw)
                    out[(int64_t)(32 * wave + 8 * (e >> 2) + 4 * h + (e & 3)) * NbP + nb0 + 32 * j + r] =
                        acc[j][e];
    }
}

extern "C" int sd_wgrad(const sd_wgrad_args *g, void *stream) {
    if (!g || !g->a || !g->b || !g->part || g->N < 0 || g->Ma <= 0 || g->Nb <= 0 ||
        g->Ma % 8 || g->Nb % 8 || g->Ma > 128 || g->Nb > 32 * WG_MAXT || g->lda < g->Ma ||
        g->ldb < g->Nb || g->lda % 8 || g->ldb % 8 || g->nparts <= 0 ||
        (g->dtype != SD_F16 && g->dtype != SD_BF16) ||
        (32 * (g->Ma / 8) + 32 * (g->Nb / 8) + 255) / 256 > WG_MAXLD) {
        sd_set_error("sd_wgrad: invalid argument (16-bit rows, Ma <= 128, Nb <= 320, "
                     "multiples of 8)");
        return -1;
    }
    const int MaP = (g->Ma + 31) & ~31, NbP = (g->Nb + 31) & ~31;
    const int lds = 32 * (MaP + 8 + 5 * 32 + 8) * 2;
    if (g->N == 0) {
        if (hipMemsetAsync(g->part, 0, (size_t)g->nparts * MaP * NbP * 4, (hipStream_t)stream) !=
            hipSuccess) {
            sd_set_error("sd_wgrad: memset failed");
            return -2;
        }
        return 0;
    }
    // column tiles per workgroup: at most 5 (<= ~200 VGPRs: two waves per SIMD), the rest
    // of the columns split over gridDim.y
    const int nt_all = NbP / 32;
    const int ncs = (nt_all + 4) / 5;
    const int nt = (nt_all + ncs - 1) / ncs;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)g->nparts, (unsigned)ncs);
#define WG_CASE(NT_)                                                                             \
    case NT_:                                                                                    \
        if (g->dtype == SD_F16)                                                                  \
            hipLaunchKernelGGL((k_wgrad<SD_F16, NT_>), grid, dim3(256), lds, st, *g);            \
        else                                                                                     \
            hipLaunchKernelGGL((k_wgrad<SD_BF16, NT_>), grid, dim3(256), lds, st, *g);           \
        break;
    switch (nt) {
        WG_CASE(1) WG_CASE(2) WG_CASE(3) WG_CASE(4) WG_CASE(5)
    }
#undef WG_CASE
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_wgrad: launch failed");
        return -2;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Both weight gradients of the training MLP in one pass (sd_mlp_train_wgrad): dW1 = dH^T X
// (128 x kx) and dW_o = dY^T [H | 1] (72 x 136) read each point's four rows once -- two
// sd_wgrad launches re-read dH for their column split and left 73 MB of partials to a
// separate torch reduction.  A workgroup (8 waves, one per CU) sums every gridDim-th
// 32-point chunk.  A chunk's four row blocks (32 rows each, contiguous in HBM) go to LDS
// by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave instruction, no staging registers)
// into padded rows, in a ring of three stages: the DMAs of chunks c + 1 and c + 2 are
// in flight while chunk c is multiplied, one barrier per chunk.  Each wave multiplies its
// output tiles from LDS read transposed (ds_read_b64_tr_b16, as k_wgrad): wave w owns dW1
// row tile w & 3 and column tiles 5 (w >> 2) .. + 4, and dW_o tiles w and w + 8 of its
// 3 x 5.  Tiles reach past the used columns (X to 320, H to 160, dY to 96 rows) into the
// rows' zero pads: those output elements are dropped.  Rows past N: the dH / dY rows are
// zeroed (the stale X / H rows then add 0).  Partials (nparts x 56320 f32) are summed in
// MW_S splits (k_mw_split) and then across the splits into the parameter layout
// (k_mw_final).  Algorithmic bytes: N (2 ldx + 256 + 144 + 272) read.
// ---------------------------------------------------------------------------
#define MW_S 16                      // splits of the partial sum
#define MW_KXP 320                   // X columns of the partial (kx, ldx <= 320)
#define MW_P1 (128 * MW_KXP)         // dW1 partial
#define MW_P2 (96 * 160)             // dW_o partial (rows 72.. and columns 136.. dropped)
#define MW_PT (MW_P1 + MW_P2)
#define MW_RING 3
#ifndef MW_NT
#define MW_NT 1  // the chunk rows LDS-DMA'd with the non-temporal hint
#endif
#ifndef MW_DIAG
#define MW_DIAG 0  // diagnostic builds only (tools/build_variant.py): 1 no MFMA, 2 no DMA, 3 no partial stores
#endif
// LDS stage: X [32][ldx], dH [32][128], dY [32][72], H [32][136] 16-bit rows at row strides
// of 64 or 192 B mod 256 (X: 2 ldx rounded up to one, 704 B for ldx 296..320; dH 320, dY
// 192, H 320): the 4 rows x 64 B of a half-wave's ds_read_b64_tr_b16 fall in 4 disjoint
// 16-bank groups (rows of 256 / 272 B put all four in the same banks: 4-way conflicts).
// The pads are never written (zero from the start) and the tiles' reach past the used
// columns stays inside them.
__host__ __device__ constexpr int mw_xstride(int ldx) {
    int s = (2 * ldx + 63) & ~63;
    while (s % 256 != 64 && s % 256 != 192) s += 64;
    return s;
}
__host__ __device__ constexpr int mw_stage_bytes(int ldx) { return 32 * (mw_xstride(ldx) + 320 + 192 + 320); }

template <int P>
__global__ void __launch_bounds__(512) k_mlp_wgrad(const sd_mlp_wgrad_args g) {
    typedef T16<P> Tr;
    typedef typename Tr::Frag Frag;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: scalar tile choice
    const int h = lane >> 5;
    const int sbx = mw_xstride(g.ldx), SZ = mw_stage_bytes(g.ldx);
    const int oDH = 32 * sbx, oDY = oDH + 32 * 320, oH = oDY + 32 * 192;
    // zero the ring once (the pads are never written)
    for (int i = tid; i < MW_RING * SZ / 16; i += 512) ((uint4 *)lds)[i] = uint4{0u, 0u, 0u, 0u};
    __syncthreads();
    // this workgroup's chunks of 32 points: blockIdx.x + gridDim.x i, i < nch -- the
    // workgroups sweep the rows together (contiguous ranges per workgroup put 256 streams
    // at a 256 KiB stride in dH: the same HBM channels at once, 2.2 TB/s)
    const int64_t nchunk = (g.N + 31) >> 5;
    const int nch = blockIdx.x < nchunk ? (int)((nchunk - 1 - blockIdx.x) / gridDim.x + 1) : 0;
    auto chunk_p0 = [&](int ci) { return ((int64_t)blockIdx.x + (int64_t)gridDim.x * ci) * 32; };
    // DMA units of a chunk (1 KiB of an LDS block each: X sbx / 32, dH 10, dY 6, H 10); wave
    // w issues units w, w + 8, ...  Lane l of unit lu fills the block's 16-B granule
    // 64 lu + l: row gl / G, granule gl % G of the row (a pad past the row's bytes: no load).
    const int ux = sbx >> 5, nu = ux + 26;
    const int cw = (nu - wave + 7) >> 3;  // this wave's units per chunk (<= 6)
    int upk[6];  // per unit: source byte in the chunk's block << 5 | row, or -1
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int u = wave + 8 * i;
        int lu, G, rb;
        if (u < ux) { lu = u; G = sbx >> 4; rb = 2 * g.ldx; }
        else if (u < ux + 10) { lu = u - ux; G = 20; rb = 256; }
        else if (u < ux + 16) { lu = u - ux - 10; G = 12; rb = 144; }
        else { lu = u - ux - 16; G = 20; rb = 272; }
        const int gl = 64 * lu + lane, row = gl / G, cg = gl - row * G;
        upk[i] = (u < nu && 16 * cg < rb) ? (row * rb + 16 * cg) << 5 | row : -1;
    }
    // per unit (wave-uniform, resolved once: selected inside the loop, the compiler made the
    // four row pointers a scratch table and waited vmcnt(0) on its load before every DMA,
    // draining the ring): source rows, bytes per row, LDS destination in the stage
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    uint64_t ubase[6];
    int urb[6];
    uint32_t udst[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int u = wave + 8 * i;
        uint64_t b;
        int rb, lu, off;
        if (u < ux) { b = (uint64_t)g.x; rb = 2 * g.ldx; lu = u; off = 0; }
        else if (u < ux + 10) { b = (uint64_t)g.dh; rb = 256; lu = u - ux; off = oDH; }
        else if (u < ux + 16) { b = (uint64_t)g.dy; rb = 144; lu = u - ux - 10; off = oDY; }
        else { b = (uint64_t)g.h; rb = 272; lu = u - ux - 16; off = oH; }
        // (uint32_t first: a sign-extended low word set the high bits -- a faulting address)
        ubase[i] = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(b >> 32)) << 32;
        urb[i] = __builtin_amdgcn_readfirstlane(rb);
        udst[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + off + 1024 * lu));
    }
    auto dma = [&](int ci) {  // chunk ci (< nch) into stage ci % 3
        const int64_t p0 = chunk_p0(ci);
        const int nv = g.N - p0 < 32 ? (int)(g.N - p0) : 32;  // rows present
        const uint32_t st = (uint32_t)((ci % MW_RING) * SZ);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (i >= cw) break;
            if (upk[i] >= 0 && (upk[i] & 31) < nv && MW_DIAG != 2)
                if (MW_NT)  // X / dH / dY rows are read once: non-temporal stream
                    sd_dma16_nt((const uint8_t *)ubase[i] + p0 * urb[i] + (upk[i] >> 5), udst[i] + st);
                else
                    sd_dma16((const uint8_t *)ubase[i] + p0 * urb[i] + (upk[i] >> 5), udst[i] + st);
        }
    };
    // transposed-read lane address (k_wgrad): group G = lane >> 4, lane 4 q + pp of it
    const int G = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int kb = 8 * (G >> 1), cbase = 16 * (G & 1) + 4 * pp;
    const int rt1 = wave & 3, ct1 = 5 * (wave >> 2);
    const int t2a = wave, t2b = wave + 8;  // dW_o tiles (row t / 5, column t % 5)
    const bool has2b = t2b < 15;
    f32x16 acc1[5], acc2[2];
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc1[j][e] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc2[j][e] = 0.f;
    auto frag = [&](const uint16_t *p, int stride) {
        const uint2 a0 = wg_tr(p), a1 = wg_tr(p + 4 * stride);
        return __builtin_bit_cast(Frag, uint4{a0.x, a0.y, a1.x, a1.y});
    };
    auto compute = [&](const uint8_t *sb) {
        const uint16_t *sx = (const uint16_t *)sb, *sdh = (const uint16_t *)(sb + oDH);
        const uint16_t *sdy = (const uint16_t *)(sb + oDY), *sh = (const uint16_t *)(sb + oH);
        const int ex = sbx >> 1;  // X row stride (elements)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {  // two k-steps of 16 points
            __builtin_amdgcn_sched_barrier(0);  // one k-step's fragments live at a time
            const int kr = 16 * ks + kb + q;
            const Frag af = frag(sdh + kr * 160 + 32 * rt1 + cbase, 160);
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const Frag bf = frag(sx + kr * ex + 32 * (ct1 + j) + cbase, ex);
                acc1[j] = Tr::mma32(af, bf, acc1[j]);
            }
            {
                const Frag a2 = frag(sdy + kr * 96 + 32 * (t2a / 5) + cbase, 96);
                const Frag b2 = frag(sh + kr * 160 + 32 * (t2a % 5) + cbase, 160);
                acc2[0] = Tr::mma32(a2, b2, acc2[0]);
            }
            if (has2b) {
                const Frag a2 = frag(sdy + kr * 96 + 32 * (t2b / 5) + cbase, 96);
                const Frag b2 = frag(sh + kr * 160 + 32 * (t2b % 5) + cbase, 160);
                acc2[1] = Tr::mma32(a2, b2, acc2[1]);
            }
        }
    };
    if (nch > 0) dma(0);
    if (nch > 1) dma(1);
    for (int c = 0; c < nch; ++c) {
        // chunk c landed: the wave's cw DMAs of chunk c + 1 (a full chunk) may stay in flight
        const int64_t pn = chunk_p0(c + 1);
        if (c + 1 < nch && pn + 32 <= g.N) {  // exactly this wave's count of the next chunk
            if (cw >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if (cw == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else if (cw == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const int64_t p0 = chunk_p0(c);
        if (p0 + 32 > g.N) {  // the last chunk: zero its dH / dY rows past N
            uint8_t *sb = lds + (c % MW_RING) * SZ;
            const int nv = (int)(g.N - p0);
            for (int i = tid; i < (32 - nv) * 25; i += 512) {
                const int row = nv + i / 25, k = i % 25;
                uint4 *d = k < 16 ? (uint4 *)(sb + oDH + row * 320) + k : (uint4 *)(sb + oDY + row * 192) + (k - 16);
                *d = uint4{0u, 0u, 0u, 0u};
            }
        }
        __syncthreads();  // chunk c visible to all waves; chunk c - 1's stage reads are done
        if (c + 2 < nch) dma(c + 2);  // into the stage chunk c - 1 used
        if (MW_DIAG != 1) compute(lds + (c % MW_RING) * SZ);
    }
    if (MW_DIAG == 3 && acc1[0][0] != 12345.f) return;
    // partial tiles: register e of a tile = C[32 rt + 8 (e >> 2) + 4 h + (e & 3)][32 ct + r]
    float *out = g.work + (int64_t)blockIdx.x * MW_PT;
    const int r = lane & 31;
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e)
            out[(32 * rt1 + 8 * (e >> 2) + 4 * h + (e & 3)) * MW_KXP + 32 * (ct1 + j) + r] = acc1[j][e];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int t = j ? t2b : t2a;
        if (j && !has2b) break;
#pragma unroll
        for (int e = 0; e < 16; ++e)
            out[MW_P1 + (32 * (t / 5) + 8 * (e >> 2) + 4 * h + (e & 3)) * 160 + 32 * (t % 5) + r] =
                acc2[j][e];
    }
}

// partial sums: split s of the nparts partials, one float4 per thread
__global__ void __launch_bounds__(256) k_mw_split(float *work, int nparts) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= MW_PT / 4) return;
    const int ps = (nparts + MW_S - 1) / MW_S;
    const int p0 = blockIdx.y * ps, p1 = p0 + ps < nparts ? p0 + ps : nparts;
    const float4 *src = (const float4 *)work;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = p0; p < p1; ++p) {
        const float4 v = src[(int64_t)p * (MW_PT / 4) + e];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    ((float4 *)(work + (int64_t)nparts * MW_PT))[blockIdx.y * (MW_PT / 4) + e] = s;
}

// the MW_S split sums into the parameter layout (lin_in: [dw_in | db_in]; lin_out rows:
// out_0 first, then dino)
__global__ void __launch_bounds__(256) k_mw_final(const sd_mlp_wgrad_args g) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= MW_PT) return;
    const float *mid = g.work + (int64_t)g.nparts * MW_PT;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < MW_S; ++k) s += mid[k * MW_PT + e];
    const int din = g.kx - 1;
    if (e < MW_P1) {
        const int row = e / MW_KXP, col = e - row * MW_KXP;
        if (col < din) g.dw_in[row * din + col] = s;
        else if (col == din) g.db_in[row] = s;
        return;
    }
    const int e2 = e - MW_P1, row = e2 / 160, col = e2 - row * 160;
    if (row > g.D) return;
    const int orow = row == g.D ? 0 : row + 1;
    if (col < 128) g.dw_out[orow * 128 + col] = s;
    else if (col == 128) g.db_out[orow] = s;
}

extern "C" int64_t sd_mlp_train_wgrad_work(int32_t nparts) {
    return nparts > 0 ? (int64_t)(nparts + MW_S) * MW_PT : -1;
}

extern "C" int sd_mlp_train_wgrad(const sd_mlp_wgrad_args *g, void *stream) {
    if (!g || (g->N > 0 && (!g->x || !g->dh || !g->dy || !g->h)) || !g->work || !g->dw_in || !g->db_in ||
        !g->dw_out || !g->db_out || g->N < 0 || g->kx <= 8 || g->kx > MW_KXP || g->kx % 8 ||
        g->ldx < g->kx || g->ldx > MW_KXP || g->ldx % 8 || g->D <= 0 || g->D > 64 || g->D % 8 || g->nparts <= 0 ||
        (g->dtype != SD_F16 && g->dtype != SD_BF16)) {
        sd_set_error("sd_mlp_train_wgrad: invalid argument (kx <= 320, kx % 8 == 0, D <= 64, "
                     "D % 8 == 0, 16-bit rows)");
        return -1;
    }
    hipStream_t st = (hipStream_t)stream;
    if (g->N == 0) {  // empty: zero gradients
        const bool ok = hipMemsetAsync(g->dw_in, 0, (size_t)128 * (g->kx - 1) * 4, st) == hipSuccess &&
                        hipMemsetAsync(g->db_in, 0, 128 * 4, st) == hipSuccess &&
                        hipMemsetAsync(g->dw_out, 0, (size_t)(g->D + 1) * 128 * 4, st) == hipSuccess &&
                        hipMemsetAsync(g->db_out, 0, (size_t)(g->D + 1) * 4, st) == hipSuccess;
        if (!ok) sd_set_error("sd_mlp_train_wgrad: memset failed");
        return ok ? 0 : -2;
    }
    const int lds = MW_RING * mw_stage_bytes(g->ldx);
    if (g->dtype == SD_F16) {
        sd_lds_attr((const void *)k_mlp_wgrad<SD_F16>, lds);
        hipLaunchKernelGGL(k_mlp_wgrad<SD_F16>, dim3(g->nparts), dim3(512), lds, st, *g);
    } else {
        sd_lds_attr((const void *)k_mlp_wgrad<SD_BF16>, lds);
        hipLaunchKernelGGL(k_mlp_wgrad<SD_BF16>, dim3(g->nparts), dim3(512), lds, st, *g);
    }
    hipLaunchKernelGGL(k_mw_split, dim3((MW_PT / 4 + 255) / 256, MW_S), dim3(256), 0, st,
                       g->work, g->nparts);
    hipLaunchKernelGGL(k_mw_final, dim3((MW_PT + 255) / 256), dim3(256), 0, st, *g);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_mlp_train_wgrad: launch failed");
        return -2;
    }
    return 0;
}
