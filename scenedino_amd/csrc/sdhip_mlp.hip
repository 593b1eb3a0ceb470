// sdhip_mlp.hip -- the ResnetFC field MLP of the training path (resnetfc.py:135-203 with
// n_blocks = 0, under the reference's with_amp autocast: base_trainer.py:223,251) as two
// fused MFMA kernels on the gather rows x = [feat (C) | code (39) | 1]:
//
//   k_mlp_fwd : H^T = relu(W1 X^T) (W1 = [W_in | b_in]: the ones column carries the bias),
//               out = H W_o^T + b_o, sigma = softplus(out_0) (bts.py:516-541, threshold 20),
//               dino = out_1..D; H is kept (16-bit, + a ones column) for the backward.
//   k_mlp_bwd : dY = [d dino | d sigma . sigmoid(out_0)], dH^T = (W_o^T dY^T) * [H > 0],
//               dX = dH W_in[:, :C] (f32 rows for sd_field_gather_bwd); dY and dH rows are
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
        for (int u = 0; u < U; ++u) {
            f32x16 o;
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] = 0.f;
#pragma unroll
            for (int s = 0; s < 8; ++s) o = Tr::mma32(af[s], w2[(u * 8 + s) * 64 + lane], o);
            // o: row = point p0 + 8 (i >> 2) + 4 h + (i & 3), column = output 32 u + r
            // (outputs 0 .. D-1 = dino, D = sigma)
            const int col = 32 * u + r;
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

template <int P>
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
        // dX = dH W_in[:, :C]: A = dH (rows = points) from the accumulators
        Frag af[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) af[s] = ml_frag<P>(dh[s >> 1], s & 1);
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
    return a->lddx >= a->C && a->lddx <= a->ldx && (a->dx_dtype == SD_F32 || a->dx_dtype == a->dtype) && a->wtf && a->wxf && a->h && a->sigma && a->d_sigma && a->d_dino && a->dy && a->dh &&
           a->dx;
}

template <typename K>
static int ml_launch(K kern, const sd_mlp_train_args *a, int lds_bytes, hipStream_t s) {
    if (lds_bytes > 160 * 1024) {
        sd_set_error("sd_mlp_train: packed weights exceed the 160 KiB LDS");
        return -1;
    }
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
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
    const int lds = (4 * KO + (a->C / 32) * 8) * 64 * 16;
    if (a->dtype == SD_F16) return ml_launch(k_mlp_bwd<SD_F16>, a, lds, (hipStream_t)stream);
    return ml_launch(k_mlp_bwd<SD_BF16>, a, lds, (hipStream_t)stream);
}
