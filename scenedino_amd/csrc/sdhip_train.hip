// sdhip_train.hip -- gfx950 kernels of the differentiable (training) field path.
//
// The inference path fuses gather -> MLP -> compositing into one kernel and never
// materialises per-sample activations.  Training (train.py through the renderer,
// base_trainer.py:223,251) needs gradients w.r.t. the feature grid and the ResnetFC
// parameters, so the training path splits at the two places where autograd needs
// saved state:
//
//   k_field_gather      a8-a10 + a15: per point, projection, frustum mask, the bilinear
//                       border gather of the C grid channels and the 39-d positional code,
//                       written as the MLP input row X = [feat | code | 1] (bts.py:321-328;
//                       the trailing 1 folds the ResnetFC biases into its GEMMs),
//                       plus the colour samples / invalid masks (no gradient: images are
//                       data).  The ResnetFC layers are plain library GEMMs (autograd).
//   k_field_gather_bwd  grid_sample backward (bts.py:299-309): dX[:, :C] scattered into the
//                       NHWC grid gradient with the forward's bilinear weights (hardware
//                       f32 atomics; the border clamp duplicates a tap only with weight 0,
//                       as torch's within-bounds test drops it).
//   k_composite_bwd     alpha-compositing backward (nerf.py:376-405): reverse transmittance
//                       recurrence, division-free (below), d sigma and d per-sample
//                       features / colours.
//
// Composite backward.  w_k = a_k T_k, T_k = prod_{j<k} (1 - a_j + 1e-10).  With
// g_k = dL/dw_k (direct + depth z_k + <dL/dfeat, f_k> + <dL/drgb, c_k>):
//   dL/da_k = T_k (g_k - U_k) + dL/dalphas_k,
//   U_{K-1} = 0,  U_{k-1} = g_k a_k + (1 - a_k + 1e-10) U_k,
// which equals the textbook  T_k g_k - (sum_{m>k} g_m w_m) / (1 - a_k + 1e-10)  without
// dividing by a factor that is 1e-10 once a sample saturates.
// d sigma_k = dL/da_k * exp(-|delta_k| relu(sigma_k)) * |delta_k| * [sigma_k > 0]
// (hard_alpha_cap: the last alpha is the constant 1, no gradient).
#include "sdhip_point.h"

#define TR_WAVES 4
#define TR_MAXK 512

// LDS written by some lanes of a wave, read by others: complete the wave's LDS traffic
// and stop the compiler moving accesses across (waves of a block run different rays,
// so no block barrier)
__device__ __forceinline__ void sd_wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---------------------------------------------------------------------------
// forward gather: one wave per tile of 32 consecutive points (a ray's samples).  Lane r
// (and r + 32) computes point r's geometry; the tile splits into runs of consecutive
// points with the same frame and tap quad -- a ray's samples straddle one texel quad
// through rounding when the render view is the encoder view (3.5 runs per 32 samples on
// the bench's rays) and walk along an epipolar line otherwise.  Each run's four texel
// rows are loaded ONCE (every lane 4 channels, f32x4 of the NHWC grid; the next run's
// loads issued before this run's blends) and blended for each of its points: a quad per
// point re-read 1 KiB x 4 from L2 for every sample (1 GB per bench step, 137 us).
// ---------------------------------------------------------------------------
#define TR_TILE 32

// row element types of X / dX: f32, or the autocast dtype (f16 / bf16) of the MLP GEMMs
template <int DT> struct TrE { typedef float T; };
template <> struct TrE<SD_F16> { typedef _Float16 T; };
template <> struct TrE<SD_BF16> { typedef __bf16 T; };

template <int DT>
__device__ __forceinline__ void tr_store4(typename TrE<DT>::T *dst, const f32x4 &o) {
    if constexpr (DT == SD_F32) {
        *(f32x4 *)dst = o;
    } else {
        typedef typename TrE<DT>::T E;
        typedef __attribute__((ext_vector_type(4))) E e4;
        *(e4 *)dst = e4{(E)o[0], (E)o[1], (E)o[2], (E)o[3]};
    }
}

// positional code entry s (< 39) of v = [x, y, z~] (positional_encoding.py:68-80): v, then
// sin(f_j v + phi) with rows (freq j, phase) and the 3 coordinates innermost; 39: the 1
__device__ __forceinline__ float tr_code(const float v[3], int s) {
    if (s < 3) return s == 0 ? v[0] : s == 1 ? v[1] : v[2];
    if (s >= 39) return 1.f;
    const int t = s - 3, fi = t / 6, cs = (t % 6) / 3, co = t % 3;
    const float f = 1.5f * (float)(1 << fi);
    const float vv = co == 0 ? v[0] : co == 1 ? v[1] : v[2];
    return sinf(fmaf(vv, f, cs ? 1.5707963705062866f : 0.f));
}

template <int DT>
__global__ void __launch_bounds__(TR_WAVES * 64)
k_field_gather(const float *__restrict__ xyz, int64_t B, int64_t P,
               const float *__restrict__ grid, int C, int Hf, int Wf,
               const float *__restrict__ cam_f, const float *__restrict__ img, int nv, int Hc,
               int Wc, const float *__restrict__ cam_c, typename TrE<DT>::T *__restrict__ x_out,
               uint8_t *__restrict__ invalid_f, float *__restrict__ rgb,
               float *__restrict__ invalid) {
    typedef typename TrE<DT>::T E;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int64_t NP = B * P;
    const int ld = C + 40;  // [feat (C) | code (39) | 1]: the 1 carries the bias through the GEMM
    const int64_t plane = (int64_t)Hf * Wf * C;
    const int64_t cplane = (int64_t)Hc * Wc * 4;
    const int64_t ntile = (NP + TR_TILE - 1) / TR_TILE;
    for (int64_t tile = (int64_t)blockIdx.x * TR_WAVES + (threadIdx.x >> 6); tile < ntile;
         tile += (int64_t)gridDim.x * TR_WAVES) {
        const int64_t p0 = tile * TR_TILE;
        const int64_t pt = p0 + r;
        const bool valid = pt < NP;
        float px = 0.f, py = 0.f, pz = 0.f;
        int gi[4] = {0, 0, 0, 0}, gb = -1;
        float gw[4] = {0.f, 0.f, 0.f, 0.f}, gv[3] = {0.f, 0.f, 0.f};
        bool invf = false;
        if (valid) {
            px = xyz[pt * 3]; py = xyz[pt * 3 + 1]; pz = xyz[pt * 3 + 2];
            const int64_t b = pt / P;
            const PointGeo geo = sd_point_geo(cam_f + b * SD_CAM_WORDS, px, py, pz, Wf, Hf);
            gi[0] = geo.t.i00; gi[1] = geo.t.i01; gi[2] = geo.t.i10; gi[3] = geo.t.i11;
            gw[0] = geo.t.w00; gw[1] = geo.t.w01; gw[2] = geo.t.w10; gw[3] = geo.t.w11;
            gv[0] = geo.v[0]; gv[1] = geo.v[1]; gv[2] = geo.v[2];
            gb = (int)b;
            invf = geo.inv_f;
        }
        // runs: a point opens one unless it has the previous point's frame and taps
        const int src = ((lane - 1) & 63) * 4;
        const bool same = __builtin_amdgcn_ds_bpermute(src, gb) == gb &&
                          __builtin_amdgcn_ds_bpermute(src, gi[0]) == gi[0] &&
                          __builtin_amdgcn_ds_bpermute(src, gi[1]) == gi[1] &&
                          __builtin_amdgcn_ds_bpermute(src, gi[2]) == gi[2] &&
                          __builtin_amdgcn_ds_bpermute(src, gi[3]) == gi[3];
        const uint32_t om = (uint32_t)__ballot(valid && (r == 0 || !same));
        const int nvp = __builtin_popcountll(__ballot(valid) & 0xffffffffull);
        // features: per channel pass (64 lanes x 4 channels), the runs in order
        for (int c = lane * 4; c - lane * 4 < C; c += 256) {
            const bool cin = c < C;
            const int cc = cin ? c : 0;
            auto issue = [&](int j, f32x4 (&t)[4]) {
                const float *g = grid + (int64_t)__builtin_amdgcn_readlane(gb, j) * plane + cc;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    t[q] = *(const f32x4 *)(g + (int64_t)__builtin_amdgcn_readlane(gi[q], j) * C);
            };
            uint32_t rem = om;
            f32x4 t[4], tn[4];
            if (rem) issue(__builtin_ctz(rem), t);
            while (rem) {
                const int s0 = __builtin_ctz(rem);
                rem &= rem - 1;
                const int e0 = rem ? __builtin_ctz(rem) : nvp;
                if (rem) issue(__builtin_ctz(rem), tn);  // the next run's texels in flight
                for (int j = s0; j < e0; ++j) {
                    float w[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        w[q] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                             __builtin_bit_cast(int, gw[q]), j));
                    f32x4 o;
#pragma unroll
                    for (int i = 0; i < 4; ++i)  // grid_sampler_2d's nw, ne, sw, se order
                        o[i] = ((t[0][i] * w[0] + t[1][i] * w[1]) + t[2][i] * w[2]) + t[3][i] * w[3];
                    if (cin) tr_store4<DT>(x_out + (p0 + j) * ld + c, o);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) t[q] = tn[q];
            }
        }
        // positional code and the bias 1: lane half h writes entries 20 h .. 20 h + 19 of
        // its point's 40
        if (valid) {
            E *xr = x_out + pt * ld + C;
#pragma unroll 1
            for (int k = 0; k < 20; k += 2) {  // (one sinf body: unrolled, 169 VGPRs)
                const int s = 20 * h + k;
                const float a0 = tr_code(gv, s), a1 = tr_code(gv, s + 1);
                if constexpr (DT == SD_F32) {
                    *(float2 *)(xr + s) = make_float2(a0, a1);
                } else {
                    typedef __attribute__((ext_vector_type(2))) E e2;
                    *(e2 *)(xr + s) = e2{(E)a0, (E)a1};
                }
            }
        }
        // colour samples / masks: lane = (point, view) pairs, 64 per pass
        if (nv > 0 && (rgb || invalid)) {
            for (int q0 = 0; q0 < nvp * nv; q0 += 64) {
                const int q = q0 + lane;
                const bool cdo = q < nvp * nv;
                const int cj = cdo ? q / nv : 0, v = cdo ? q - cj * nv : 0;
                const float cx = __shfl(px, cj), cy = __shfl(py, cj), cz = __shfl(pz, cj);
                if (cdo) {
                    const int64_t p = p0 + cj;
                    const int64_t b = p / P;
                    float col[3] = {0.f, 0.f, 0.f};
                    const bool ic = sd_color_view(cam_c + (b * nv + v) * SD_CAM_WORDS,
                                                  img + (b * nv + v) * cplane, Wc, Hc, cx, cy, cz, col);
                    if (rgb) {
                        rgb[(p * nv + v) * 3] = col[0];
                        rgb[(p * nv + v) * 3 + 1] = col[1];
                        rgb[(p * nv + v) * 3 + 2] = col[2];
                    }
                    if (invalid) {
                        float x, y, zc;  // the encoder-frustum test of sd_point_geo, same arithmetic
                        sd_project(cam_f + b * SD_CAM_WORDS, cx, cy, cz, x, y, zc);
                        invalid[p * nv + v] = (ic | sd_outside(x, y, zc)) ? 1.f : 0.f;
                    }
                }
            }
        }
        if (h == 0 && valid && invalid_f) invalid_f[pt] = invf ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// gather backward: dG (B, Hf, Wf, C) += bilinear scatter of dX[:, :C]
// One wave per run of TR_RUN consecutive points (a ray's samples are consecutive, and
// they often project onto the same 2x2 texels -- always when the render view is the
// encoder view): contributions are summed in registers while a point's four tap indices
// equal the previous point's, and only flushed to HBM (f32 atomics in L2) when they change.
// ---------------------------------------------------------------------------
#define TR_RUN 16

// lane's channels c + 64 i (i < 4): every atomic instruction covers 64 consecutive floats
// (atomics are not merged across lanes; 16-B-strided lanes would move 4x the sectors)
__device__ __forceinline__ void tr_flush(float *g, const int idx[4], const f32x4 acc[4], int C,
                                         int c) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        float *dst = g + (int64_t)idx[t] * C + c;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (c + 64 * i < C && acc[t][i] != 0.f) unsafeAtomicAdd(dst + 64 * i, acc[t][i]);
    }
}

template <int DT>
__global__ void __launch_bounds__(TR_WAVES * 64)
k_field_gather_bwd(const float *__restrict__ xyz, int64_t B, int64_t P,
                   const typename TrE<DT>::T *__restrict__ dx, int64_t ldx, int C, int Hf, int Wf,
                   const float *__restrict__ cam_f, float *__restrict__ dgrid) {
    const int lane = threadIdx.x & 63;
    const int64_t NP = B * P;
    const int64_t nruns = (NP + TR_RUN - 1) / TR_RUN;
    const int64_t plane = (int64_t)Hf * Wf * C;
    for (int64_t run = (int64_t)blockIdx.x * TR_WAVES + (threadIdx.x >> 6); run < nruns;
         run += (int64_t)gridDim.x * TR_WAVES) {
        const int64_t p0 = run * TR_RUN;
        const int n = (int)(p0 + TR_RUN < NP ? TR_RUN : NP - p0);
        // geometry of the run's points, lane j < n = point p0 + j (broadcast below)
        int gi[4] = {0, 0, 0, 0}, gb = 0;
        float gw[4] = {0.f, 0.f, 0.f, 0.f};
        if (lane < n) {
            const int64_t p = p0 + lane;
            const int64_t b = p / P;
            const PointGeo geo = sd_point_geo(cam_f + b * SD_CAM_WORDS, xyz[p * 3], xyz[p * 3 + 1],
                                              xyz[p * 3 + 2], Wf, Hf);
            gi[0] = geo.t.i00; gi[1] = geo.t.i01; gi[2] = geo.t.i10; gi[3] = geo.t.i11;
            gw[0] = geo.t.w00; gw[1] = geo.t.w01; gw[2] = geo.t.w10; gw[3] = geo.t.w11;
            gb = (int)b;
        }
        for (int c = lane; c < C; c += 256) {
            // all rows of the run in flight at once (16 x 4 coalesced words per lane)
            f32x4 v[TR_RUN];
#pragma unroll
            for (int j = 0; j < TR_RUN; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    v[j][i] = (j < n && c + 64 * i < C) ? (float)dx[(p0 + j) * ldx + c + 64 * i] : 0.f;
            int idx[4] = {-1, -1, -1, -1}, bcur = -1;
            f32x4 acc[4] = {};
#pragma unroll
            for (int j = 0; j < TR_RUN; ++j) {
                if (j < n) {
                    int ni[4];
                    float wt[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        ni[t] = __builtin_amdgcn_readlane(gi[t], j);
                        wt[t] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                                                              __builtin_bit_cast(int, gw[t]), j));
                    }
                    const int b = __builtin_amdgcn_readlane(gb, j);
                    if (b != bcur || ni[0] != idx[0] || ni[1] != idx[1] || ni[2] != idx[2] ||
                        ni[3] != idx[3]) {  // wave-uniform branch
                        if (bcur >= 0) tr_flush(dgrid + bcur * plane, idx, acc, C, c);
                        bcur = b;
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            idx[t] = ni[t];
                            acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
                        }
                    }
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int i = 0; i < 4; ++i) acc[t][i] += v[j][i] * wt[t];
                }
            }
            if (bcur >= 0) tr_flush(dgrid + bcur * plane, idx, acc, C, c);
        }
    }
}

// ---------------------------------------------------------------------------
// composite backward: one wave per ray
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(TR_WAVES * 64)
k_composite_bwd(const float *__restrict__ z, const float *__restrict__ sigma,
                const float *__restrict__ feat, int F, const float *__restrict__ rgb, int Cc,
                int64_t R, int K, int hard_cap, const float *__restrict__ g_depth,
                const float *__restrict__ g_feat, const float *__restrict__ g_rgb,
                const float *__restrict__ g_w, const float *__restrict__ g_a,
                float *__restrict__ d_sigma, float *__restrict__ d_feat,
                float *__restrict__ d_rgb) {
    __shared__ float s_a[TR_WAVES][TR_MAXK], s_g[TR_WAVES][TR_MAXK], s_t[TR_WAVES][TR_MAXK];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float *sa = s_a[wv], *sg = s_g[wv], *st = s_t[wv];
    for (int64_t ray = (int64_t)blockIdx.x * TR_WAVES + wv; ray < R;
         ray += (int64_t)gridDim.x * TR_WAVES) {
        const float *zr = z + ray * K, *sr = sigma + ray * K;
        const float gd = g_depth ? g_depth[ray] : 0.f;
        // phase 0 (F % 4 == 0): <dL/dfeat, f_k> with coalesced 16-B row reads, 4 samples per
        // instruction (16 lanes per row), reduced over the row's lanes -> st[k]
        const bool vec = feat && g_feat && (F % 4) == 0;
        if (vec) {
            const int rr = lane >> 4, c4 = (lane & 15) * 4;
            const float *gf = g_feat + ray * F;
#pragma unroll 4
            for (int k0 = 0; k0 < K; k0 += 4) {
                const int k = k0 + rr;
                float s = 0.f;
                if (k < K) {
                    const float *fr = feat + (ray * K + k) * (int64_t)F;
                    for (int c = c4; c < F; c += 64) {
                        const f32x4 a = *(const f32x4 *)(fr + c), b = *(const f32x4 *)(gf + c);
                        s += ((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3];
                    }
                }
                s += __shfl_xor(s, 8);
                s += __shfl_xor(s, 4);
                s += __shfl_xor(s, 2);
                s += __shfl_xor(s, 1);
                if ((lane & 15) == 0 && k < K) st[k] = s;
            }
            sd_wave_lds_sync();
        }
        // phase 1 (lane = sample): alpha and g_k = dL/dw_k
        for (int k = lane; k < K; k += 64) {
            const float zk = zr[k];
            const float delta = (k + 1 < K) ? zr[k + 1] - zk : 1e10f;
            float alpha = 1.f - expf(-fabsf(delta) * fmaxf(sr[k], 0.f));
            if (hard_cap && k == K - 1) alpha = 1.f;
            float g = gd * zk;
            if (g_w) g += g_w[ray * K + k];
            if (vec) {
                g += st[k];
            } else if (feat && g_feat) {
                const float *fr = feat + (ray * K + k) * (int64_t)F;
                const float *gf = g_feat + ray * F;
                float s = 0.f;
                for (int c = 0; c < F; ++c) s += gf[c] * fr[c];
                g += s;
            }
            if (rgb && g_rgb) {
                const float *cr = rgb + (ray * K + k) * (int64_t)Cc;
                const float *gc = g_rgb + ray * Cc;
                float s = 0.f;
                for (int c = 0; c < Cc; ++c) s += gc[c] * cr[c];
                g += s;
            }
            sa[k] = alpha;
            sg[k] = g;
        }
        sd_wave_lds_sync();
        // phase 2: T_k forward, U_k backward; sa <- w_k, sg <- dL/da_k.  K <= 64: the
        // recurrences over readlane broadcasts of the lanes' (alpha, g) (the same products
        // in the same order as the one-lane LDS loop below, without its LDS round trips)
        if (K <= 64) {
            const float al = lane < K ? sa[lane] : 0.f, gl = lane < K ? sg[lane] : 0.f;
            float T = 1.f, tl = 0.f;
            for (int k = 0; k < K; ++k) {
                if (lane == k) tl = T;
                const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, al), k));
                T = T * ((1.f - a) + 1e-10f);
            }
            float U = 0.f, dal = 0.f, wl = 0.f;
            for (int k = K - 1; k >= 0; --k) {
                const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, al), k));
                const float g = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, gl), k));
                const float tk = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tl), k));
                const float da = tk * (g - U);
                U = g * a + ((1.f - a) + 1e-10f) * U;
                if (lane == k) {
                    dal = da;
                    wl = a * tk;
                }
            }
            sd_wave_lds_sync();  // every lane has read its (alpha, g)
            if (lane < K) {
                sg[lane] = dal;
                sa[lane] = wl;
            }
        } else if (lane == 0) {
            float T = 1.f;
            for (int k = 0; k < K; ++k) {
                st[k] = T;
                T = T * ((1.f - sa[k]) + 1e-10f);
            }
            float U = 0.f;
            for (int k = K - 1; k >= 0; --k) {
                const float a = sa[k], g = sg[k];
                const float tk = st[k];
                float da = tk * (g - U);
                U = g * a + ((1.f - a) + 1e-10f) * U;
                sg[k] = da;
                sa[k] = a * tk;  // w_k
            }
        }
        sd_wave_lds_sync();
        // phase 3 (lane = sample): d sigma
        for (int k = lane; k < K; k += 64) {
            const float zk = zr[k];
            const float delta = (k + 1 < K) ? zr[k + 1] - zk : 1e10f;
            const float s = sr[k];
            float da = sg[k];
            if (g_a) da += g_a[ray * K + k];
            float ds = 0.f;
            if (!(hard_cap && k == K - 1) && s > 0.f) {
                const float ad = fabsf(delta);
                ds = da * expf(-ad * s) * ad;
            }
            d_sigma[ray * K + k] = ds;
        }
        // phase 4 (lane = channel): d feat_k = w_k dL/dfeat, d rgb_k = w_k dL/drgb
        if (d_feat && g_feat && F <= 64) {  // the lane's dL/dfeat loaded once, not after every store
            const float gfl = lane < F ? g_feat[ray * F + lane] : 0.f;
            for (int k = 0; k < K; ++k) {
                const float w = sa[k];
                if (lane < F) d_feat[(ray * K + k) * (int64_t)F + lane] = w * gfl;
            }
        } else if (d_feat && g_feat) {
            for (int k = 0; k < K; ++k) {
                const float w = sa[k];
                for (int c = lane; c < F; c += 64)
                    d_feat[(ray * K + k) * (int64_t)F + c] = w * g_feat[ray * F + c];
            }
        }
        if (d_rgb && g_rgb) {
            for (int k = 0; k < K; ++k) {
                const float w = sa[k];
                for (int c = lane; c < Cc; c += 64)
                    d_rgb[(ray * K + k) * (int64_t)Cc + c] = w * g_rgb[ray * Cc + c];
            }
        }
        sd_wave_lds_sync();
    }
}

// ---------------------------------------------------------------------------
// NHWC f32 -> NCHW f32 (the grid gradient back in the encoder's layout) through a
// 32x33 LDS tile; grid (W/32, C/32, B*H); inverse of sdhip_rays.hip's k_pack_grid
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_unpack_grid(const float *__restrict__ in, int64_t C,
                                                     int64_t H, int64_t W,
                                                     float *__restrict__ out) {
    __shared__ float tile[32][33];
    const int64_t bh = blockIdx.z;
    const int64_t b = bh / H, y = bh - b * H;
    const int64_t x0 = (int64_t)blockIdx.x * 32, c0 = (int64_t)blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int j = ty; j < 32; j += 8) {  // rows = pixels x, columns = channels c (contiguous)
        const int64_t x = x0 + j, c = c0 + tx;
        tile[j][tx] = (c < C && x < W) ? in[((b * H + y) * W + x) * C + c] : 0.f;
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        const int64_t c = c0 + j, x = x0 + tx;
        if (c < C && x < W) out[((b * C + c) * H + y) * W + x] = tile[tx][j];
    }
}

// vector variant (C % 4 == 0, W % 4 == 0): 64 x 64 tile, 16-byte loads along c and
// stores along x; grid (W/64, C/64, B*H)
__global__ void __launch_bounds__(256) k_unpack_grid4(const float *__restrict__ in, int64_t C,
                                                      int64_t H, int64_t W,
                                                      float *__restrict__ out) {
    __shared__ float tile[64][65];
    const int64_t bh = blockIdx.z;
    const int64_t b = bh / H, y = bh - b * H;
    const int64_t x0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + 256 * k, px = i >> 4, ch = (i & 15) * 4;
        const int64_t x = x0 + px, c = c0 + ch;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (x < W && c < C) v = *(const f32x4 *)(in + ((b * H + y) * W + x) * C + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[ch + j][px] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = threadIdx.x + 256 * k, ch = i >> 4, px = (i & 15) * 4;
        const int64_t c = c0 + ch, x = x0 + px;
        if (c < C && x < W)
            *(f32x4 *)(out + ((b * C + c) * H + y) * W + x) =
                f32x4{tile[ch][px], tile[ch][px + 1], tile[ch][px + 2], tile[ch][px + 3]};
    }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int tr_blocks(int64_t units) {
    const int64_t want = (units + TR_WAVES - 1) / TR_WAVES;
    const int64_t cap = (int64_t)sd_num_cus() * 32;
    return (int)(want < cap ? want : cap);
}

extern "C" int sd_field_gather(const float *xyz, int64_t B, int64_t P, const float *grid_nhwc,
                               int32_t C, int32_t Hf, int32_t Wf, const float *cam_f,
                               const float *img, int32_t nv, int32_t Hc, int32_t Wc,
                               const float *cam_c, void *x_out, int32_t x_dtype,
                               uint8_t *invalid_f, float *rgb, float *invalid, void *stream) {
    if (B <= 0 || P < 0 || !xyz || !grid_nhwc || !cam_f || !x_out || C <= 0 || (C % 4) ||
        (x_dtype != SD_F32 && x_dtype != SD_F16 && x_dtype != SD_BF16) ||
        Hf <= 0 || Wf <= 0 || nv < 0 || nv > 64 ||
        (nv > 0 && (rgb || invalid) && (!img || !cam_c || Hc <= 0 || Wc <= 0))) {
        sd_set_error("sd_field_gather: invalid argument (C % 4 == 0, nv <= 64)");
        return -1;
    }
    if (P == 0) return 0;
    const dim3 grid(tr_blocks((B * P + TR_TILE - 1) / TR_TILE)), blk(TR_WAVES * 64);
    hipStream_t s = (hipStream_t)stream;
    if (x_dtype == SD_F16)
        hipLaunchKernelGGL(k_field_gather<SD_F16>, grid, blk, 0, s, xyz, B, P, grid_nhwc, C, Hf,
                           Wf, cam_f, img, nv, Hc, Wc, cam_c, (_Float16 *)x_out, invalid_f, rgb,
                           invalid);
    else if (x_dtype == SD_BF16)
        hipLaunchKernelGGL(k_field_gather<SD_BF16>, grid, blk, 0, s, xyz, B, P, grid_nhwc, C, Hf,
                           Wf, cam_f, img, nv, Hc, Wc, cam_c, (__bf16 *)x_out, invalid_f, rgb,
                           invalid);
    else
        hipLaunchKernelGGL(k_field_gather<SD_F32>, grid, blk, 0, s, xyz, B, P, grid_nhwc, C, Hf,
                           Wf, cam_f, img, nv, Hc, Wc, cam_c, (float *)x_out, invalid_f, rgb,
                           invalid);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_field_gather: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_field_gather_bwd(const float *xyz, int64_t B, int64_t P, const void *dx,
                                   int32_t dx_dtype, int64_t ldx, int32_t C, int32_t Hf,
                                   int32_t Wf, const float *cam_f, float *dgrid_nhwc,
                                   void *stream) {
    if (B <= 0 || P < 0 || !xyz || !dx || !cam_f || !dgrid_nhwc || C <= 0 || (C % 4) ||
        (dx_dtype != SD_F32 && dx_dtype != SD_F16 && dx_dtype != SD_BF16) ||
        ldx < C || Hf <= 0 || Wf <= 0) {
        sd_set_error("sd_field_gather_bwd: invalid argument (C % 4 == 0, ldx >= C)");
        return -1;
    }
    if (P == 0) return 0;
    const dim3 grid(tr_blocks((B * P + TR_RUN - 1) / TR_RUN)), blk(TR_WAVES * 64);
    hipStream_t s = (hipStream_t)stream;
    if (dx_dtype == SD_F16)
        hipLaunchKernelGGL(k_field_gather_bwd<SD_F16>, grid, blk, 0, s, xyz, B, P,
                           (const _Float16 *)dx, ldx, C, Hf, Wf, cam_f, dgrid_nhwc);
    else if (dx_dtype == SD_BF16)
        hipLaunchKernelGGL(k_field_gather_bwd<SD_BF16>, grid, blk, 0, s, xyz, B, P,
                           (const __bf16 *)dx, ldx, C, Hf, Wf, cam_f, dgrid_nhwc);
    else
        hipLaunchKernelGGL(k_field_gather_bwd<SD_F32>, grid, blk, 0, s, xyz, B, P,
                           (const float *)dx, ldx, C, Hf, Wf, cam_f, dgrid_nhwc);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_field_gather_bwd: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_composite_bwd(const float *z, const float *sigma, const float *feat, int64_t F,
                                const float *rgb, int64_t Cc, int64_t R, int32_t K,
                                int32_t hard_alpha_cap, const float *g_depth, const float *g_feat,
                                const float *g_rgb, const float *g_weights, const float *g_alphas,
                                float *d_sigma, float *d_feat, float *d_rgb, void *stream) {
    if (R < 0 || K <= 0 || K > TR_MAXK || !z || !sigma || !d_sigma || F < 0 || Cc < 0 ||
        (d_feat && (!feat || !g_feat)) || (d_rgb && (!rgb || !g_rgb)) ||
        (g_feat && !feat) || (g_rgb && !rgb) || F >= (1 << 30) || Cc >= (1 << 30)) {
        sd_set_error("sd_composite_bwd: invalid argument (0 < K <= 512; feature / colour "
                     "gradients need their forward inputs)");
        return -1;
    }
    if (R == 0) return 0;
    hipLaunchKernelGGL(k_composite_bwd, dim3(tr_blocks(R)), dim3(TR_WAVES * 64), 0,
                       (hipStream_t)stream, z, sigma, feat, (int)F, rgb, (int)Cc, R, K,
                       hard_alpha_cap, g_depth, g_feat, g_rgb, g_weights, g_alphas, d_sigma,
                       d_feat, d_rgb);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_composite_bwd: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_unpack_grid(const float *grid_nhwc, int64_t B, int64_t C, int64_t H, int64_t W,
                              float *grid_nchw, void *stream) {
    if (B < 0 || C <= 0 || H <= 0 || W <= 0 || !grid_nhwc || !grid_nchw ||
        B * H >= (1LL << 31)) {
        sd_set_error("sd_unpack_grid: invalid argument");
        return -1;
    }
    if (B == 0) return 0;
    if (C % 4 == 0 && W % 4 == 0 && ((uintptr_t)grid_nhwc & 15) == 0 &&
        ((uintptr_t)grid_nchw & 15) == 0) {
        dim3 g4((unsigned)((W + 63) / 64), (unsigned)((C + 63) / 64), (unsigned)(B * H));
        hipLaunchKernelGGL(k_unpack_grid4, g4, dim3(256), 0, (hipStream_t)stream, grid_nhwc, C, H,
                           W, grid_nchw);
        if (hipGetLastError() != hipSuccess) {
            sd_set_error("sd_unpack_grid: launch failed");
            return -2;
        }
        return 0;
    }
    dim3 g((unsigned)((W + 31) / 32), (unsigned)((C + 31) / 32), (unsigned)(B * H));
    hipLaunchKernelGGL(k_unpack_grid, g, dim3(256), 0, (hipStream_t)stream, grid_nhwc, C, H, W,
                       grid_nchw);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_unpack_grid: launch failed");
        return -2;
    }
    return 0;
}
