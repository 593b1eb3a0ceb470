// sdhip_seg.hip -- SSCBench voxel-query path on gfx950 (CDNA4).
//
//   k_voxel_points : voxel-centre grid in the velodyne frame, rigidly moved into the
//                    camera frame.  fp64 arithmetic, one rounding to f32,
//                    bit-exact with the reference's numba + numpy pipeline
//                    (sscbench/point_utils.py:17-82, sscbench/fusion.py:203-219,407-411,
//                    evaluate_model_sscbench.py:270-278).
//   k_seg_head     : per-point DINO code (D_r = 64) -> MlpDimReduction.transform_expand
//                    (64 -> 128 ReLU -> 768, L2 normalise; dim_reduction.py:22-25) ->
//                    SemanticHead "stego_kmeans" (semantic_head.py:107-111: StegoClusterHead
//                    768 -> 64 linear + 768 -> 768 ReLU -> 64, L2 normalise; cosine k-means
//                    argmax over the cluster centres, pseudo_assignment lookup,
//                    semantic_head.py:285-373) -> optionally the SSCBench alpha-weighted
//                    class pick (evaluate_model_sscbench.py:727-742 at factor 1).
//
// Folding (all exact algebra; only the rounding order differs from the reference):
//   f = e / n,  e = W2 h + b2,  n = max(|e|, 1e-12),  h = relu(W1 x + b1)   (transform_expand)
//   SemanticHead re-normalises f (|f| = 1: the identity up to rounding).
//   stego = Wl f + bl + Wn2 relu(Wn1 f + bn1) + bn2
//         = (L h + Wl b2) / n + bl + bn2 + Wn2 relu((M h + Wn1 b2) / n + bn1)
//   with L = Wl W2 (64 x 128) and M = Wn1 W2 (768 x 128) folded once on the host: the
//   768 x 768 product of the reference becomes a 768 x 128 one.  The class is
//   argmax_k <stego / |stego|, c_k / |c_k|> = argmax_k <n stego, c_k / |c_k|> (a positive
//   scale does not move an argmax), so the kernel forms n stego (n u = relu(M h + Wn1 b2 +
//   n bn1): the biases enter as accumulator inits, no per-element rescale) and scores it
//   on the matrix cores with hi + lo bf16 operands (fp32-grade).
//
// The norm: |e|^2 = h^T G h + 2 (W2^T b2).h + |b2|^2 with G = W2^T W2 (d_latent x
// d_latent, folded on the host, bf16 hi + lo fragments): 64 MFMAs per 32 points instead of
// the 768 x 128 product (the fp8 record keeps that product on fp8 MFMA).
//
// Work unit: one wave = SG_NT x 32 points (lane = point, as the accumulator columns of
// v_mfma_f32_32x32x16_bf16); weights are the MFMA A operands (rows = output features),
// 1-KiB fragments (each feeds SG_NT MFMAs).  The big products (Gram, M + Wn2) stream their
// weight tiles through LDS, in a ring of slots shared by the workgroup's 4 waves
// (one per SIMD, two workgroups per CU); the small ones (W1, L) read their fragments from L2.  Hidden vectors
// never leave the registers: an accumulator tile is converted in place into the B operand
// of the next product (k order permuted; the host packs the A operands to match, see
// scenedino_amd/seg_pack.py).
#include "sdhip_common.h"

extern "C" void sd_set_error(const char *msg);

#ifndef SG_NT
#define SG_NT 2        // 32-point column tiles per wave (2: 2 waves per SIMD, measured -11 % vs 4)
#endif
#ifndef SG_EXP
#define SG_EXP 0       // timing experiments only, wrong results: 1 no waits, 2 no vmcnt, 3 no DMA, 4 no barrier
#endif
#ifndef SG_WAVES
#define SG_WAVES 4     // waves per workgroup sharing the LDS weight stream (two workgroups per
                       // CU drift apart: one's HBM input phase overlaps the other's MFMAs; -6 %)
#endif
#define SG_DR 64       // reduced DINO dims (MlpDimReduction reduced_channels)
#define SG_DL 128      // latent dims (MlpDimReduction latent_channels)
#define SG_DC 64       // stego code dims

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

// ---------------------------------------------------------------------------
// voxel-centre grid
// ---------------------------------------------------------------------------
struct VoxConst {
    double o[3];   // origin, already rounded to f32 (vox2world casts vol_origin to float32)
    double t[12];  // rows 0..2 of the 4x4 rigid transform
};

__global__ void __launch_bounds__(256) k_voxel_points(VoxConst c, double vox, int64_t nx,
                                                      int64_t ny, int64_t nz,
                                                      float *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nx * ny * nz) return;
    const int64_t iz = i % nz;
    const int64_t q = i / nz;
    const int64_t iy = q % ny;
    const int64_t ix = q / ny;
    // vox2world (numba, fusion.py:212-218): f32 coords, f64 arithmetic, f32 store
    const double ci[3] = {(double)(float)ix, (double)(float)iy, (double)(float)iz};
    double p[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double v = c.o[j] + vox * ci[j];
        v = v + vox * 0.5;
        p[j] = (double)(float)v;
    }
    // rigid_transform (fusion.py:407-411) in f64, then .float() (evaluate_model_sscbench.py:278)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double acc = c.t[4 * j] * p[0];
        acc = acc + c.t[4 * j + 1] * p[1];
        acc = acc + c.t[4 * j + 2] * p[2];
        acc = acc + c.t[4 * j + 3];
        out[i * 3 + j] = (float)acc;
    }
}

// ---------------------------------------------------------------------------
// grow: 3x3x3 max filter of the density grid (F.max_pool3d(kernel 3, stride 1, padding 1),
// evaluate_model_sscbench.py:755-756), separable: a thread takes the max over its voxel's
// 3 x 3 (x, y) neighbourhood at its own z (9 loads, coalesced along z), the z step reads
// the neighbours' partial maxima from LDS (a block edge recomputes its outside
// neighbour).  NaN propagates and the padding never wins, as torch's max pooling.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sg_nanmax(float m, float v) { return (v > m || v != v) ? v : m; }

__device__ __forceinline__ float sg_max9(const float *__restrict__ in, int x, int y, int z,
                                         int nx, int ny, int nz) {
    float m = -INFINITY;
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
            const int xx = x + dx, yy = y + dy;
            if (xx >= 0 && xx < nx && yy >= 0 && yy < ny)
                m = sg_nanmax(m, in[((int64_t)xx * ny + yy) * nz + z]);
        }
    return m;
}

__global__ void __launch_bounds__(256) k_grow3(const float *__restrict__ in, int nx, int ny,
                                               int nz, float *__restrict__ out) {
    __shared__ float sm[256];
    const int n = nx * ny * nz;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int ic = i < n ? i : n - 1;
    const int z = ic % nz, q = ic / nz, y = q % ny, x = q / ny;
    const float m9 = sg_max9(in, x, y, z, nx, ny, nz);
    sm[threadIdx.x] = m9;
    __syncthreads();
    if (i >= n) return;
    float m = m9;
    if (z > 0) m = sg_nanmax(m, threadIdx.x > 0 ? sm[threadIdx.x - 1] : sg_max9(in, x, y, z - 1, nx, ny, nz));
    if (z + 1 < nz)
        m = sg_nanmax(m, threadIdx.x < 255 ? sm[threadIdx.x + 1] : sg_max9(in, x, y, z + 1, nx, ny, nz));
    out[i] = m;
}

// ---------------------------------------------------------------------------
// folded transform_expand + stego + k-means head
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x16 sg_zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

// 16 floats stored in accumulator-row order for lane half h: vec + (t * 2 + h) * 16
__device__ __forceinline__ f32x16 sg_rows(const float *__restrict__ vec, int t, int h) {
    const f32x4_t *p = (const f32x4_t *)(vec + (t * 2 + h) * 16);
    f32x16 r;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        f32x4_t v = p[g];
        r[4 * g] = v[0]; r[4 * g + 1] = v[1]; r[4 * g + 2] = v[2]; r[4 * g + 3] = v[3];
    }
    return r;
}

#define SG_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
// OCP e4m3 x e4m3 -> f32, 32x32x64, unit scales (E8M0 127): lane l holds A[l & 31][32 (l >> 5)
// + j] / B[32 (l >> 5) + j][l & 31] in byte j (tools/probe/mfma_f8.hip)
#define SG_MFMA8(a, b, c) \
    __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4((a), (b), (c), 0, 0, 0, 127, 0, 127)

__device__ __forceinline__ uint32_t sg_bf16_bits(__bf16 v) { return (uint32_t)__builtin_bit_cast(unsigned short, v); }

// element e of a bf16x8 register quad as f32; volatile so that the unpacking stays in the
// Gram epilogue (hoisted, h's 128 unpacked values would spill)
__device__ __forceinline__ float sg_bf16_at(bf16x8 v, int e) {
    typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
    const uint32_t w = __builtin_bit_cast(u32x4_t, v)[e >> 1];
    float r;
    if (e & 1) asm volatile("v_and_b32 %0, 0xffff0000, %1" : "=v"(r) : "v"(w));
    else asm volatile("v_lshlrev_b32 %0, 16, %1" : "=v"(r) : "v"(w));
    return r;
}

// relu(acc[8 s .. 8 s + 7]) as a bf16 B operand: round to bf16 (RNE), then max with +0 on
// the 16-bit patterns (a negative bf16 is a negative int16): one v_pk_max_i16 per pair
__device__ __forceinline__ bf16x8 sg_relu_b(const f32x16 &acc, int s) {
    typedef __attribute__((ext_vector_type(8))) short s16x8_t;
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
    s16x8_t v = __builtin_bit_cast(s16x8_t, r);
    v = __builtin_elementwise_max(v, (s16x8_t)0);
    return __builtin_bit_cast(bf16x8, v);
}

// Weight tiles are streamed through LDS, shared by the workgroup's 4 waves (each wave used
// to read every fragment from L2 itself): 1-KiB pieces by LDS-DMA, issued as inline asm so
// that the compiler does not fence every LDS read behind the DMA (m0 = LDS destination).
#define SG_SLOT (16 * 1024)  // one tile: 16 Gram fragments, 8 M + 4 Wn2 fragments or 4 KiB fp8
#define SG_NSLOT 3          // LDS slots (the M loop runs three deep)
#ifndef SG_NT_IN
#define SG_NT_IN 1          // the input codes (read once) with the non-temporal hint
#endif
__device__ __forceinline__ void sg_dma1k(const uint8_t *src, uint32_t lds_dst, int lane) {
    lds_dst = __builtin_amdgcn_readfirstlane(lds_dst);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src + lane * 16), "s"(lds_dst) : "memory");
}

// diagnostic build only (SG_PROF=1): per-phase s_memtime cycles summed over all waves
#ifndef SG_PROF
#define SG_PROF 0
#endif
#if SG_PROF
__device__ unsigned long long sg_prof[16];
#define SG_T(i)                                            \
    {                                                      \
        const uint64_t _t = __builtin_amdgcn_s_memtime();  \
        pacc[i] += (uint32_t)(_t - tlast);                 \
        tlast = _t;                                        \
    }
extern "C" int sd_seg_prof(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sg_prof), sizeof(sg_prof)) != hipSuccess) return -2;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sg_prof), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#else
#define SG_T(i)
#endif

// MODE bit 0: write dino_full (transform_expand output); bit 1: segmentation head.
// F8 (labels / seg only): the norm product |W2 h + b2| on fp8 MFMA -- h quantised to e4m3
// with a per-point power-of-two scale (its largest value lands in [128, 256)), W2 with the
// per-tensor one of the packed record; the scales leave in the f32 epilogue (exact).
template <int MODE, bool F8>
#ifndef SG_WPE
#define SG_WPE 1  // waves per SIMD the register budget must allow
#endif
__global__ void __launch_bounds__(SG_WAVES * 64) __attribute__((amdgpu_waves_per_eu(SG_WPE)))
k_seg_head(const void *__restrict__ dino_in,
                                                            int32_t x16, int64_t P, int32_t DF,
                                                            const float *__restrict__ sigma,
                                                            float neg_vox, sd_seg_head h,
                                                            int32_t *__restrict__ labels,
                                                            uint8_t *__restrict__ seg,
                                                            float *__restrict__ full) {
    constexpr bool FULL = MODE & 1;
    constexpr bool SEG = MODE & 2;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r = lane & 31, hh = lane >> 5;
    const int64_t base = ((int64_t)blockIdx.x * SG_WAVES + wave) * (32 * SG_NT);
    // workgroup-uniform exit only: the weight stream below has barriers (waves past P run
    // on zero inputs and store nothing)
    if ((int64_t)blockIdx.x * SG_WAVES * (32 * SG_NT) >= P) return;
    const int T2 = DF / 32;
#if SG_PROF
    uint32_t pacc[10] = {};
    uint64_t tlast = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ __attribute__((aligned(16))) uint8_t sg_lds[];
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)sg_lds;
    // stage tile pieces [0, n) (1 KiB each, piece i from src(i)) into slot; wave w issues w, w + 4, ...
    auto stage = [&](int slot, int n, auto src) {
#if SG_EXP != 3
        // every wave issues the same count (no branch: the loops stay one basic block);
        // a wave past the last piece re-copies an earlier one (the same bytes)
#pragma unroll
        for (int k = 0; k < (n + SG_WAVES - 1) / SG_WAVES; ++k) {
            const int i = (wave + k * SG_WAVES) % n;
            sg_dma1k(src(i), lds0 + slot * SG_SLOT + i * 1024, lane);
        }
#endif
    };
    auto landed = [&]() {  // this wave's DMA done, then every wave's (and the previous slot free)
#if SG_EXP != 1 && SG_EXP != 2
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#if SG_EXP != 1 && SG_EXP != 4
        __syncthreads();
#endif
    };
    // Gram tile t: 16 fragments at t * 16 KiB
    auto gsrc = [&](int t) { return [=](int i) { return (const uint8_t *)h.wg + (int64_t)t * 16384 + i * 1024; }; };
    // M tile t: M fragments (t, 0..7) at t * 8 KiB, then Wn2 fragments (rt, 2 t + s)
    const int KS = DF / 16;
    auto msrc = [&](int t) {
        return [=](int i) {
            return i < 8 ? (const uint8_t *)h.wm + (int64_t)t * 8192 + i * 1024
                         : (const uint8_t *)h.wn2 + ((int64_t)((i - 8) >> 1) * KS + 2 * t + ((i - 8) & 1)) * 1024;
        };
    };
    // W1 into slot 1 and L into slot 2 (read from LDS by layer 1 / the L path, both done
    // before those slots take Gram / M tiles), the first Gram tile into slot 0: one wait
    // for all of it (and the input codes) instead of a chain of L2 round trips
    stage(1, 16, [&](int i) { return (const uint8_t *)h.w1 + i * 1024; });
    if (SEG) stage(2, 16, [&](int i) { return (const uint8_t *)h.wl + i * 1024; });
    if (!F8) stage(0, 16, gsrc(0));
    // the M loop's bias rows (Wn1 b2, bn1; accumulator-row order) in LDS after the slots
    const float *lds_b = (const float *)(sg_lds + SG_NSLOT * SG_SLOT);
    if (SEG) {
        f32x4_t *d = (f32x4_t *)(sg_lds + SG_NSLOT * SG_SLOT);
        for (int i = threadIdx.x; i < DF / 2; i += SG_WAVES * 64)
            d[i] = i < DF / 4 ? ((const f32x4_t *)h.bm)[i] : ((const f32x4_t *)h.bn1)[i - DF / 4];
    }

    // ---- layer 1: h = relu(W1 x + b1) -> B operands hb[ct][k-step 0..7] ----
    bf16x8 hb[SG_NT][SG_DL / 16];
    {
        bf16x8 xb[SG_NT][SG_DR / 16];
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) {
            const int64_t p = base + 32 * ct + r;
            if (p < P && x16) {  // bf16 codes (sd_field_query dino_dtype SD_BF16): as loaded
                const bf16x8 *src = (const bf16x8 *)dino_in + p * (SG_DR / 8);
#pragma unroll
                for (int s = 0; s < SG_DR / 16; ++s)
                    xb[ct][s] = SG_NT_IN ? __builtin_nontemporal_load(&src[2 * s + hh]) : src[2 * s + hh];
            } else if (p < P) {
                const f32x4_t *src = (const f32x4_t *)((const float *)dino_in + p * SG_DR);
#pragma unroll
                for (int s = 0; s < SG_DR / 16; ++s) {
                    f32x4_t a = src[4 * s + 2 * hh], b = src[4 * s + 2 * hh + 1];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        xb[ct][s][j] = (__bf16)a[j];
                        xb[ct][s][4 + j] = (__bf16)b[j];
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < SG_DR / 16; ++s)
#pragma unroll
                    for (int j = 0; j < 8; ++j) xb[ct][s][j] = (__bf16)0.f;
            }
        }
        landed();  // W1 (and L, Gram tile 0) in LDS
        const bf16x8 *w1 = (const bf16x8 *)(sg_lds + 1 * SG_SLOT);
#pragma unroll
        for (int t = 0; t < SG_DL / 32; ++t) {
            const f32x16 bb = sg_rows(h.b1, t, hh);  // the bias rides in as the accumulator
            f32x16 acc[SG_NT];
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = bb;
#pragma unroll
            for (int s = 0; s < SG_DR / 16; ++s) {
                const bf16x8 a = w1[(t * (SG_DR / 16) + s) * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = SG_MFMA(a, xb[ct][s], acc[ct]);
            }
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) {
                hb[ct][2 * t] = sg_relu_b(acc[ct], 0);
                hb[ct][2 * t + 1] = sg_relu_b(acc[ct], 1);
            }
        }
    }

    SG_T(0);
    // ---- n = max(|W2 h + b2|, 1e-12)  (F.normalize, dim_reduction.py:25) ----
    float den[SG_NT];
    if (F8) {
        // h as fp8 B operands: k-step s (64 hidden), byte j of lane half hh = hidden
        // 32 (2 s + (j >> 4)) + (jj & 3) + 8 (jj >> 2) + 4 hh, jj = j & 15 -- the rows this
        // lane holds of layer-1 tiles 2 s and 2 s + 1 (register jj = hb[2 tile + (jj >> 3)][jj & 7])
        i32x8_t h8[SG_NT][2];
        float scp[SG_NT];
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) {
            uint32_t mx = 0;  // h >= 0: the largest bf16 bit pattern is the largest value
#pragma unroll
            for (int q = 0; q < SG_DL / 16; ++q)
#pragma unroll
                for (int e = 0; e < 8; ++e) mx = max(mx, sg_bf16_bits(hb[ct][q][e]));
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, 32));
            const int eb = max((int)((mx >> 7) & 0xffu), 8);  // biased exponent of max h
            const float mul = __uint_as_float((uint32_t)(261 - eb) << 23);  // 2^(134 - eb)
            scp[ct] = __uint_as_float((uint32_t)(eb - 7) << 23) * h.w2_f8_scale;
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int w = 0; w < 8; ++w) {
                    const int tile = 2 * st + (w >> 2), q = 2 * tile + ((w & 3) >> 1), e0 = 4 * (w & 1);
                    float v[4];
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        v[b] = __uint_as_float(sg_bf16_bits(hb[ct][q][e0 + b]) << 16) * mul;
                    int word = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
                    word = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], word, true);
                    h8[ct][st][w] = word;
                }
        }
        float ss[SG_NT];
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) ss[ct] = 0.f;
        const uint8_t *w2 = (const uint8_t *)h.w2_f8;  // tile t: 4 KiB at t * 4096
        auto src = [&](int t) { return [=](int i) { return w2 + (int64_t)t * 4096 + i * 1024; }; };
        stage(0, 4, src(0));
        f32x16 bb = sg_rows(h.b2, 0, hh);
        for (int t = 0; t < T2; ++t) {
            landed();
            if (t + 1 < T2) stage((t + 1) & 1, 4, src(t + 1));
            const int tn = t + 1 < T2 ? t + 1 : t;
            i32x8_t cur[2];
            const i32x8_t *sl = (const i32x8_t *)(sg_lds + (t & 1) * SG_SLOT);
#pragma unroll
            for (int st = 0; st < 2; ++st) cur[st] = sl[st * 64 + lane];
            const f32x16 bbn = sg_rows(h.b2, tn, hh);
            f32x16 acc[SG_NT];
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = sg_zero16();
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = SG_MFMA8(cur[st], h8[ct][st], acc[ct]);
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float e = fmaf(acc[ct][i], scp[ct], bb[i]);
                    ss[ct] = fmaf(e, e, ss[ct]);
                }
            bb = bbn;
        }
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) {
            const float tot = ss[ct] + __shfl_xor(ss[ct], 32);
            den[ct] = fmaxf(sqrtf(tot), 1e-12f);
        }
    } else {
        // Gram form: |e|^2 = sum_i h_i ((G h)_i + g2_i) + |b2|^2, G = W2^T W2 as bf16 hi + lo
        // fragments (64 MFMAs per 32 points in place of the d_full x d_latent product's
        // 192); the rows of G h land in the registers that hold the same rows of h
        float ss[SG_NT];
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) ss[ct] = 0.f;
        // software-pipelined over the 4 tiles (two slots): tile t + 1's product is issued
        // before tile t's epilogue; tile 0 landed with the layer-1 wait
        auto g_issue = [&](int slot, f32x16 *acc) {
            const bf16x8 *sl = (const bf16x8 *)(sg_lds + slot * SG_SLOT);
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = sg_zero16();
#pragma unroll
            for (int q = 0; q < 2 * (SG_DL / 16); ++q) {
                const bf16x8 a = sl[q * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = SG_MFMA(a, hb[ct][q & 7], acc[ct]);
            }
        };
        f32x16 acc[SG_NT];
        landed();  // every wave is done with W1 (slot 1)
        stage(1, 16, gsrc(1));
        g_issue(0, acc);
#pragma unroll  // (h's registers are indexed by t)
        for (int t = 0; t < SG_DL / 32; ++t) {
            f32x16 accn[SG_NT];
            if (t + 1 < SG_DL / 32) {
                landed();  // tile t + 1 landed; every wave has issued tile t (its slot is free)
                if (t + 2 < SG_DL / 32) stage(t & 1, 16, gsrc(t + 2));
                else if (t + 2 == SG_DL / 32 && SEG) stage(0, 12, msrc(0));  // the M loop's first tile
                g_issue((t + 1) & 1, accn);
            }
            const f32x16 gg = sg_rows(h.g2, t, hh);
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    ss[ct] = fmaf(sg_bf16_at(hb[ct][2 * t + (i >> 3)], i & 7), acc[ct][i] + gg[i], ss[ct]);
            if (t + 1 < SG_DL / 32) {
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = accn[ct];
            }
        }
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) {
            const float tot = fmaxf(ss[ct] + __shfl_xor(ss[ct], 32) + h.b2sq, 0.f);
            den[ct] = fmaxf(sqrtf(tot), 1e-12f);
        }
    }

    SG_T(1);
    if (FULL) {  // dino_full = e / n, recomputed with n known (one store per element)
        const bf16x8 *w2 = (const bf16x8 *)h.w2;
        for (int t = 0; t < T2; ++t) {
            f32x16 acc[SG_NT];
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = sg_zero16();
#pragma unroll
            for (int q = 0; q < SG_DL / 16; ++q) {
                const bf16x8 a = w2[(t * (SG_DL / 16) + q) * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = SG_MFMA(a, hb[ct][q], acc[ct]);
            }
            const f32x16 bb = sg_rows(h.b2, t, hh);
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) {
                const int64_t p = base + 32 * ct + r;
                if (p < P) {
                    float *dst = full + p * DF + 32 * t + 4 * hh;
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        f32x4_t v;
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = (acc[ct][4 * g + e] + bb[4 * g + e]) / den[ct];
                        *(f32x4_t *)(dst + 8 * g) = v;
                    }
                }
            }
        }
    }
    if (!SEG) return;

    // ---- the stego code times n (a positive scale the k-means argmax ignores):
    //      n stego = L h + Wl b2 + n (bl + bn2) + Wn2 relu(M h + Wn1 b2 + n bn1),
    //      every bias entering as an MFMA accumulator init ----
    // linear path folded to L (64 x 128)
    f32x16 sacc[SG_NT][SG_DC / 32];
    {
        const bf16x8 *wl = (const bf16x8 *)(sg_lds + 2 * SG_SLOT);  // (staged at the start)
#pragma unroll
        for (int rt = 0; rt < SG_DC / 32; ++rt) {
            const f32x16 lb = sg_rows(h.bl, rt, hh);
            const f32x16 ob = sg_rows(h.bo, rt, hh);
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct)
#pragma unroll
                for (int i = 0; i < 16; ++i) sacc[ct][rt][i] = fmaf(den[ct], ob[i], lb[i]);
#pragma unroll
            for (int q = 0; q < SG_DL / 16; ++q) {
                const bf16x8 a = wl[(rt * (SG_DL / 16) + q) * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) sacc[ct][rt] = SG_MFMA(a, hb[ct][q], sacc[ct][rt]);
            }
        }
    }
    SG_T(2);
    // nonlinear path, n u = relu(M h + Wn1 b2 + n bn1) per 32-row tile, consumed at once by
    // Wn2 (64 x 768).  Software-pipelined: tile t + 1's M product is issued before tile
    // t's ReLU epilogue and Wn2 product, so the matrix cores stay fed while the epilogue
    // runs; three LDS slots (tile t + 2 streams into the slot tile t - 1 left)
    {
        if (F8) {  // (the Gram loop staged tile 0 already)
            landed();  // the norm loop's last slot is free
            stage(0, 12, msrc(0));
        }
        auto m_issue = [&](int t, f32x16 *acc) {  // tile t (slot t mod 3) into acc
            const f32x16 mbv = sg_rows(lds_b, t, hh), nbv = sg_rows(lds_b + DF, t, hh);
            const bf16x8 *sl = (const bf16x8 *)(sg_lds + (t % 3) * SG_SLOT);
            bf16x8 cur[SG_DL / 16];
#pragma unroll
            for (int q = 0; q < SG_DL / 16; ++q) cur[q] = sl[q * 64 + lane];
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[ct][i] = fmaf(den[ct], nbv[i], mbv[i]);
#pragma unroll
            for (int q = 0; q < SG_DL / 16; ++q)
#pragma unroll
                for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = SG_MFMA(cur[q], hb[ct][q], acc[ct]);
        };
        auto m_finish = [&](int t, const f32x16 *acc) {  // relu + Wn2 of tile t
            const bf16x8 *sl = (const bf16x8 *)(sg_lds + (t % 3) * SG_SLOT);
            bf16x8 ub[SG_NT][2];
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) {
                ub[ct][0] = sg_relu_b(acc[ct], 0);
                ub[ct][1] = sg_relu_b(acc[ct], 1);
            }
#pragma unroll
            for (int rt = 0; rt < SG_DC / 32; ++rt)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const bf16x8 cw = sl[(8 + 2 * rt + s) * 64 + lane];
#pragma unroll
                    for (int ct = 0; ct < SG_NT; ++ct) sacc[ct][rt] = SG_MFMA(cw, ub[ct][s], sacc[ct][rt]);
                }
        };
        f32x16 acc[SG_NT];
        landed();  // tile 0 in slot 0; every wave is past the norm loop
        stage(1 % T2, 12, msrc(1 % T2));
        m_issue(0, acc);
        for (int t = 0; t + 1 < T2; ++t) {  // (branch-free body; the last tile is peeled)
            SG_T(3);
            landed();  // tile t + 1 landed; every wave is done with tile t - 1's slot
            SG_T(4);
            // tile t + 2 (past the end: tile T2 - 1 again, into the spare slot)
            const int t2 = t + 2 < T2 ? t + 2 : T2 - 1;
            stage((t + 2) % 3, 12, msrc(t2));
            f32x16 accn[SG_NT];
            m_issue(t + 1, accn);
            SG_T(5);
            m_finish(t, acc);
            SG_T(6);
#pragma unroll
            for (int ct = 0; ct < SG_NT; ++ct) acc[ct] = accn[ct];
        }
        m_finish(T2 - 1, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the spare slot's DMA (LDS lives on)
    }
    SG_T(3);

    // ---- cosine k-means: argmax_k <n stego, c_k/|c_k|> (first maximum wins, as
    //      torch.argmax) -> pseudo_assignment.  The scores as one MFMA tile per 32
    //      clusters (rows) x 32 points: stego and the centres as bf16 hi + lo operands
    //      (hi hi + hi lo + lo hi: fp32-grade scores) ----
    bf16x8 shi[SG_NT][SG_DC / 16], slo[SG_NT][SG_DC / 16];
#pragma unroll
    for (int ct = 0; ct < SG_NT; ++ct)
#pragma unroll
        for (int q = 0; q < SG_DC / 16; ++q)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = sacc[ct][q >> 1][8 * (q & 1) + j];
                const __bf16 hi = (__bf16)v;
                shi[ct][q][j] = hi;
                slo[ct][q][j] = (__bf16)(v - (float)hi);
            }
    float best[SG_NT];
    int bi[SG_NT];
#pragma unroll
    for (int ct = 0; ct < SG_NT; ++ct) {
        best[ct] = -INFINITY;
        bi[ct] = 0;
    }
    const bf16x8 *wc = (const bf16x8 *)h.centres;  // [tile][hi, lo][k-step][64][8]
    const int nct = (h.n_clusters + 31) >> 5;
    for (int c = 0; c < nct; ++c) {
        bf16x8 ah[SG_DC / 16], al[SG_DC / 16];
#pragma unroll
        for (int q = 0; q < SG_DC / 16; ++q) {
            ah[q] = wc[((2 * c) * (SG_DC / 16) + q) * 64 + lane];
            al[q] = wc[((2 * c + 1) * (SG_DC / 16) + q) * 64 + lane];
        }
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) {
            f32x16 acc = sg_zero16();
#pragma unroll
            for (int q = 0; q < SG_DC / 16; ++q) {
                acc = SG_MFMA(ah[q], shi[ct][q], acc);
                acc = SG_MFMA(ah[q], slo[ct][q], acc);
                acc = SG_MFMA(al[q], shi[ct][q], acc);
            }
            // this lane's rows in increasing cluster order; padding rows never win
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int k = 32 * c + 8 * (i >> 2) + 4 * hh + (i & 3);
                if (k < h.n_clusters && acc[i] > best[ct]) {
                    best[ct] = acc[i];
                    bi[ct] = k;
                }
            }
        }
    }
#pragma unroll
    for (int ct = 0; ct < SG_NT; ++ct) {  // the two lane halves: larger score, then lower index
        const float ob = __shfl_xor(best[ct], 32);
        const int oi = __shfl_xor(bi[ct], 32);
        if (ob > best[ct] || (ob == best[ct] && oi < bi[ct])) bi[ct] = oi;
    }
    SG_T(7);
#if SG_PROF
    if (lane < 10) atomicAdd(&sg_prof[lane], (unsigned long long)pacc[lane]);
    if (lane == 0) atomicAdd(&sg_prof[15], 1ull);
#endif
    if (hh == 0) {
#pragma unroll
        for (int ct = 0; ct < SG_NT; ++ct) {
            const int64_t p = base + 32 * ct + r;
            if (p >= P) continue;
            const int lab = h.assign[bi[ct]];
            if (labels) labels[p] = lab;
            if (seg) {
                // alphas = 1 - exp(-VOXEL_SIZE * sigma); argmax over the 19 classes of
                // alpha * one_hot(label) = label if alpha > 0 else 0
                const float alpha = 1.f - expf(neg_vox * sigma[p]);
                seg[p] = (uint8_t)(alpha > 0.f ? lab : 0);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// the same head on v_mfma_f32_16x16x32_bf16 (records with frag_layout SD_SEG_FRAG16)
// ---------------------------------------------------------------------------
// Same products, same k order within every dot product's 32-deep step, same LDS weight
// stream and workgroup shape; the fragments are 16-row tiles with 32-deep k-steps (lane
// l: row / column l & 15, k = 8 (l >> 4) + j; accumulator register i of lane group
// g = l >> 4 holds row 4 g + i).  A wave takes 4 column tiles of 16 points (64 points, as
// k_seg_head's 2 x 32).  An accumulator pair (row tiles 2 q, 2 q + 1) is the B operand of
// the next product's k-step q: element j <- row 32 q + 16 (j >> 2) + 4 g + (j & 3), the
// order seg_pack.py packs the A operands in (perm16).  Why: the 16x16x32 form does the
// same FLOPs per cycle as 32x32x16, and the chip holds a higher clock on it under load
// (MI355X_MICROARCH.md, DVFS item 7); a timing probe of this kernel's MFMA mix measured
// 0.75 -> 0.69 ms (profiles/r6_c5).
#ifndef SG16_NCT
#define SG16_NCT 4  // 16-point column tiles per wave
#endif
#define SG_MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ f32x4_t sg_rows4(const float *__restrict__ vec, int t, int g) {
    return ((const f32x4_t *)vec)[t * 4 + g];
}
__device__ __forceinline__ f32x4_t sg_zero4() { return f32x4_t{0.f, 0.f, 0.f, 0.f}; }

// relu of the accumulator pair (a: row tile 2 q, b: 2 q + 1) as the bf16 B operand of k-step q
__device__ __forceinline__ bf16x8 sg_relu_b16(const f32x4_t &a, const f32x4_t &b) {
    typedef __attribute__((ext_vector_type(8))) short s16x8_t;
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        r[j] = (__bf16)a[j];
        r[4 + j] = (__bf16)b[j];
    }
    s16x8_t v = __builtin_bit_cast(s16x8_t, r);
    v = __builtin_elementwise_max(v, (s16x8_t)0);
    return __builtin_bit_cast(bf16x8, v);
}

template <int MODE>
__global__ void __launch_bounds__(SG_WAVES * 64) __attribute__((amdgpu_waves_per_eu(SG_WPE)))
k_seg_head16(const void *__restrict__ dino_in, int32_t x16, int64_t P, int32_t DF,
             const float *__restrict__ sigma, float neg_vox, sd_seg_head h,
             int32_t *__restrict__ labels, uint8_t *__restrict__ seg, float *__restrict__ full) {
    constexpr bool FULL = MODE & 1;
    constexpr bool SEG = MODE & 2;
    constexpr int NCT = SG16_NCT;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pc = lane & 15, g = lane >> 4;
    const int64_t base = ((int64_t)blockIdx.x * SG_WAVES + wave) * (16 * NCT);
    if ((int64_t)blockIdx.x * SG_WAVES * (16 * NCT) >= P) return;  // workgroup-uniform only
    const int T2 = DF / 32;
    extern __shared__ __attribute__((aligned(16))) uint8_t sg_lds[];
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)sg_lds;
    auto stage = [&](int slot, int n, auto src) {
#pragma unroll
        for (int k = 0; k < (n + SG_WAVES - 1) / SG_WAVES; ++k) {
            const int i = (wave + k * SG_WAVES) % n;
            sg_dma1k(src(i), lds0 + slot * SG_SLOT + i * 1024, lane);
        }
    };
    auto landed = [&]() {
#ifndef SG16_EXP
#define SG16_EXP 0  // timing probes only (wrong results): 1 no waits, 2 no barrier
#endif
        if (SG16_EXP != 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (SG16_EXP == 0) __syncthreads();
    };
    auto gsrc = [&](int t) { return [=](int i) { return (const uint8_t *)h.wg + (int64_t)t * 16384 + i * 1024; }; };
    const int KS = DF / 32;  // Wn2 k-steps
    // M tile t (32 rows): fragments (row tile 2 t + (i >> 2), k-step i & 3) at t * 8 KiB,
    // then the Wn2 fragments (code row tile i - 8, k-step t)
    auto msrc = [&](int t) {
        return [=](int i) {
            return i < 8 ? (const uint8_t *)h.wm + (int64_t)t * 8192 + i * 1024
                         : (const uint8_t *)h.wn2 + ((int64_t)(i - 8) * KS + t) * 1024;
        };
    };
    stage(1, 16, [&](int i) { return (const uint8_t *)h.w1 + i * 1024; });
    if (SEG) stage(2, 16, [&](int i) { return (const uint8_t *)h.wl + i * 1024; });
    stage(0, 16, gsrc(0));
    const float *lds_b = (const float *)(sg_lds + SG_NSLOT * SG_SLOT);
    if (SEG) {
        f32x4_t *d = (f32x4_t *)(sg_lds + SG_NSLOT * SG_SLOT);
        for (int i = threadIdx.x; i < DF / 2; i += SG_WAVES * 64)
            d[i] = i < DF / 4 ? ((const f32x4_t *)h.bm)[i] : ((const f32x4_t *)h.bn1)[i - DF / 4];
    }

    // ---- layer 1: h = relu(W1 x + b1) -> B operands hb[ct][k-step 0..3] ----
    bf16x8 hb[NCT][SG_DL / 32];
    {
        bf16x8 xb[NCT][SG_DR / 32];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            const int64_t p = base + 16 * ct + pc;
            if (p < P && x16) {  // point p's dims 32 s + 8 g .. + 7
                const bf16x8 *src = (const bf16x8 *)dino_in + p * (SG_DR / 8);
#pragma unroll
                for (int s = 0; s < SG_DR / 32; ++s)
                    xb[ct][s] = SG_NT_IN ? __builtin_nontemporal_load(&src[4 * s + g]) : src[4 * s + g];
            } else if (p < P) {
                const f32x4_t *src = (const f32x4_t *)((const float *)dino_in + p * SG_DR);
#pragma unroll
                for (int s = 0; s < SG_DR / 32; ++s) {
                    f32x4_t a = src[8 * s + 2 * g], b = src[8 * s + 2 * g + 1];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        xb[ct][s][j] = (__bf16)a[j];
                        xb[ct][s][4 + j] = (__bf16)b[j];
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < SG_DR / 32; ++s)
#pragma unroll
                    for (int j = 0; j < 8; ++j) xb[ct][s][j] = (__bf16)0.f;
            }
        }
        landed();  // W1 (and L, Gram tile 0) in LDS
        const bf16x8 *w1 = (const bf16x8 *)(sg_lds + 1 * SG_SLOT);
#pragma unroll
        for (int q = 0; q < SG_DL / 32; ++q) {
            f32x4_t acc[NCT][2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f32x4_t bb = sg_rows4(h.b1, 2 * q + u, g);
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) acc[ct][u] = bb;
#pragma unroll
                for (int s = 0; s < SG_DR / 32; ++s) {
                    const bf16x8 a = w1[((2 * q + u) * (SG_DR / 32) + s) * 64 + lane];
#pragma unroll
                    for (int ct = 0; ct < NCT; ++ct) acc[ct][u] = SG_MFMA16(a, xb[ct][s], acc[ct][u]);
                }
            }
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) hb[ct][q] = sg_relu_b16(acc[ct][0], acc[ct][1]);
        }
    }

    // ---- n = max(|W2 h + b2|, 1e-12) by the Gram form (hi + lo G, two slots) ----
    float den[NCT];
    {
        float ss[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) ss[ct] = 0.f;
        auto g_issue = [&](int slot, f32x4_t (*acc)[2]) {
            const bf16x8 *sl = (const bf16x8 *)(sg_lds + slot * SG_SLOT);
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) acc[ct][0] = acc[ct][1] = sg_zero4();
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const bf16x8 a = sl[i * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) acc[ct][i >> 3] = SG_MFMA16(a, hb[ct][i & 3], acc[ct][i >> 3]);
            }
        };
        f32x4_t acc[NCT][2];
        landed();  // every wave is done with W1 (slot 1)
        stage(1, 16, gsrc(1));
        g_issue(0, acc);
#pragma unroll
        for (int t = 0; t < SG_DL / 32; ++t) {
            f32x4_t accn[NCT][2];
            if (t + 1 < SG_DL / 32) {
                landed();
                if (t + 2 < SG_DL / 32) stage(t & 1, 16, gsrc(t + 2));
                else if (t + 2 == SG_DL / 32 && SEG) stage(0, 12, msrc(0));
                g_issue((t + 1) & 1, accn);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f32x4_t gg = sg_rows4(h.g2, 2 * t + u, g);
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        ss[ct] = fmaf(sg_bf16_at(hb[ct][t], 4 * u + e), acc[ct][u][e] + gg[e], ss[ct]);
            }
            if (t + 1 < SG_DL / 32) {
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) acc[ct][0] = accn[ct][0], acc[ct][1] = accn[ct][1];
            }
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            float tot = ss[ct] + __shfl_xor(ss[ct], 16);
            tot += __shfl_xor(tot, 32);
            den[ct] = fmaxf(sqrtf(fmaxf(tot + h.b2sq, 0.f)), 1e-12f);
        }
    }

    if (FULL) {  // dino_full = e / n: lane (point, g) holds dims 16 t + 4 g .. + 3
        const bf16x8 *w2 = (const bf16x8 *)h.w2;
        for (int t = 0; t < DF / 16; ++t) {
            f32x4_t acc[NCT];
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) acc[ct] = sg_zero4();
#pragma unroll
            for (int q = 0; q < SG_DL / 32; ++q) {
                const bf16x8 a = w2[(t * (SG_DL / 32) + q) * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) acc[ct] = SG_MFMA16(a, hb[ct][q], acc[ct]);
            }
            const f32x4_t bb = sg_rows4(h.b2, t, g);
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) {
                const int64_t p = base + 16 * ct + pc;
                if (p < P) {
                    f32x4_t v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = (acc[ct][e] + bb[e]) / den[ct];
                    *(f32x4_t *)(full + p * DF + 16 * t + 4 * g) = v;
                }
            }
        }
    }
    if (!SEG) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no DMA left in flight at exit)
        return;
    }

    // ---- n stego = L h + Wl b2 + n (bl + bn2) + Wn2 relu(M h + Wn1 b2 + n bn1) ----
    f32x4_t sacc[NCT][SG_DC / 16];
    {
        const bf16x8 *wl = (const bf16x8 *)(sg_lds + 2 * SG_SLOT);
#pragma unroll
        for (int rt = 0; rt < SG_DC / 16; ++rt) {
            const f32x4_t lb = sg_rows4(h.bl, rt, g), ob = sg_rows4(h.bo, rt, g);
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
                for (int e = 0; e < 4; ++e) sacc[ct][rt][e] = fmaf(den[ct], ob[e], lb[e]);
#pragma unroll
            for (int q = 0; q < SG_DL / 32; ++q) {
                const bf16x8 a = wl[(rt * (SG_DL / 32) + q) * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) sacc[ct][rt] = SG_MFMA16(a, hb[ct][q], sacc[ct][rt]);
            }
        }
    }
    {
        auto m_issue = [&](int t, f32x4_t (*acc)[2]) {
            const bf16x8 *sl = (const bf16x8 *)(sg_lds + (t % 3) * SG_SLOT);
            bf16x8 cur[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) cur[i] = sl[i * 64 + lane];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const f32x4_t mbv = sg_rows4(lds_b, 2 * t + u, g), nbv = sg_rows4(lds_b + DF, 2 * t + u, g);
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[ct][u][e] = fmaf(den[ct], nbv[e], mbv[e]);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) acc[ct][i >> 2] = SG_MFMA16(cur[i], hb[ct][i & 3], acc[ct][i >> 2]);
        };
        auto m_finish = [&](int t, f32x4_t (*acc)[2]) {
            const bf16x8 *sl = (const bf16x8 *)(sg_lds + (t % 3) * SG_SLOT);
            bf16x8 ub[NCT];
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) ub[ct] = sg_relu_b16(acc[ct][0], acc[ct][1]);
#pragma unroll
            for (int rt = 0; rt < SG_DC / 16; ++rt) {
                const bf16x8 cw = sl[(8 + rt) * 64 + lane];
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) sacc[ct][rt] = SG_MFMA16(cw, ub[ct], sacc[ct][rt]);
            }
        };
        f32x4_t acc[NCT][2];
        landed();  // tile 0 in slot 0; every wave is past the norm loop
        stage(1 % T2, 12, msrc(1 % T2));
        m_issue(0, acc);
        for (int t = 0; t + 1 < T2; ++t) {
            landed();
            const int t2 = t + 2 < T2 ? t + 2 : T2 - 1;
            stage((t + 2) % 3, 12, msrc(t2));
            f32x4_t accn[NCT][2];
            m_issue(t + 1, accn);
            m_finish(t, acc);
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) acc[ct][0] = accn[ct][0], acc[ct][1] = accn[ct][1];
        }
        m_finish(T2 - 1, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }

    // ---- cosine k-means on MFMA (hi + lo operands), 16 clusters per tile ----
    bf16x8 shi[NCT][SG_DC / 32], slo[NCT][SG_DC / 32];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
        for (int q = 0; q < SG_DC / 32; ++q)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = sacc[ct][2 * q + (j >> 2)][j & 3];
                const __bf16 hi = (__bf16)v;
                shi[ct][q][j] = hi;
                slo[ct][q][j] = (__bf16)(v - (float)hi);
            }
    float best[NCT];
    int bi[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
        best[ct] = -INFINITY;
        bi[ct] = 0;
    }
    const bf16x8 *wc = (const bf16x8 *)h.centres;  // [tile][hi, lo][k-step][64][8]
    const int nct = (h.n_clusters + 15) >> 4;
    for (int c = 0; c < nct; ++c) {
        bf16x8 ah[SG_DC / 32], al[SG_DC / 32];
#pragma unroll
        for (int q = 0; q < SG_DC / 32; ++q) {
            ah[q] = wc[((2 * c) * (SG_DC / 32) + q) * 64 + lane];
            al[q] = wc[((2 * c + 1) * (SG_DC / 32) + q) * 64 + lane];
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            f32x4_t acc = sg_zero4();
#pragma unroll
            for (int q = 0; q < SG_DC / 32; ++q) {
                acc = SG_MFMA16(ah[q], shi[ct][q], acc);
                acc = SG_MFMA16(ah[q], slo[ct][q], acc);
                acc = SG_MFMA16(al[q], shi[ct][q], acc);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // this lane's clusters in increasing order
                const int k = 16 * c + 4 * g + e;
                if (k < h.n_clusters && acc[e] > best[ct]) {
                    best[ct] = acc[e];
                    bi[ct] = k;
                }
            }
        }
    }
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)  // the 4 lane groups: larger score, then lower index
#pragma unroll
        for (int m = 16; m <= 32; m <<= 1) {
            const float ob = __shfl_xor(best[ct], m);
            const int oi = __shfl_xor(bi[ct], m);
            if (ob > best[ct] || (ob == best[ct] && oi < bi[ct])) {
                best[ct] = ob;
                bi[ct] = oi;
            }
        }
    if (g == 0) {
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            const int64_t p = base + 16 * ct + pc;
            if (p >= P) continue;
            const int lab = h.assign[bi[ct]];
            if (labels) labels[p] = lab;
            if (seg) {
                const float alpha = 1.f - expf(neg_vox * sigma[p]);
                seg[p] = (uint8_t)(alpha > 0.f ? lab : 0);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int sd_voxel_points(const double *origin, double vox, int64_t nx, int64_t ny,
                               int64_t nz, const double *T, float *pts_out, void *stream) {
    if (!origin || !T || !pts_out || nx <= 0 || ny <= 0 || nz <= 0 || !(vox > 0.0) ||
        nx * ny * nz > ((int64_t)1 << 40)) {
        sd_set_error("sd_voxel_points: invalid argument");
        return -1;
    }
    VoxConst c;
    for (int j = 0; j < 3; ++j) c.o[j] = (double)(float)origin[j];
    for (int j = 0; j < 12; ++j) c.t[j] = T[j];
    const int64_t n = nx * ny * nz;
    hipLaunchKernelGGL(k_voxel_points, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, c, vox, nx, ny, nz, pts_out);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_voxel_points: launch failed");
        return -2;
    }
    return 0;
}

extern "C" int sd_grow3(const float *in, int64_t nx, int64_t ny, int64_t nz, float *out,
                        void *stream) {
    if (!in || !out || in == out || nx <= 0 || ny <= 0 || nz <= 0 || nx * ny * nz > 0x7fffff00LL) {
        sd_set_error("sd_grow3: invalid argument (distinct in / out, positive dims)");
        return -1;
    }
    const int64_t n = nx * ny * nz;
    hipLaunchKernelGGL(k_grow3, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, in, (int)nx, (int)ny, (int)nz, out);
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_grow3: launch failed");
        return -2;
    }
    return 0;
}

static int sg_valid(const sd_seg_head *h, int need_seg) {
    if (!h || !h->w1 || !h->b1 || !h->w2 || !h->b2 || !h->wg || !h->g2) return 0;
    if (h->d_in != SG_DR || h->d_latent != SG_DL || h->d_full <= 0 || h->d_full % 32 ||
        h->d_full > 4096)
        return 0;
    if (need_seg) {
        if (!h->wl || !h->bl || !h->bo || !h->wm || !h->bm || !h->bn1 || !h->wn2 ||
            !h->centres || !h->assign)
            return 0;
        if (h->d_code != SG_DC || h->n_clusters <= 0 || h->n_clusters > 256) return 0;
    }
    return 1;
}

extern "C" int sd_seg_query(const void *dino, int32_t dino_dtype, int64_t P,
                            const sd_seg_head *h, const float *sigma, float voxel_size,
                            int32_t *labels, uint8_t *seg, float *dino_full, void *stream) {
    const int want_seg = labels != nullptr || seg != nullptr;
    if (h && (h->frag_layout != SD_SEG_FRAG32 && h->frag_layout != SD_SEG_FRAG16)) {
        sd_set_error("sd_seg_query: frag_layout must be SD_SEG_FRAG32 or SD_SEG_FRAG16");
        return -1;
    }
    if (h && h->frag_layout == SD_SEG_FRAG16 && h->w2_f8) {
        sd_set_error("sd_seg_query: the fp8 norm (w2_f8) needs frag_layout SD_SEG_FRAG32");
        return -1;
    }
    if (!dino || P < 0 || !sg_valid(h, want_seg) || (seg && !sigma) ||
        (!want_seg && !dino_full) || (dino_dtype != SD_F32 && dino_dtype != SD_BF16) ||
        ((uintptr_t)dino & 15)) {
        sd_set_error("sd_seg_query: invalid argument (d_in 64, d_latent 128, d_full % 32 == 0, "
                     "d_code 64, 1..256 clusters; seg needs sigma; at least one output; dino "
                     "f32 or bf16, 16-B aligned)");
        return -1;
    }
    if (P == 0) return 0;
    const int64_t per_wg = (int64_t)SG_WAVES * (h->frag_layout == SD_SEG_FRAG16 ? 16 * SG16_NCT : 32 * SG_NT);
    const int64_t nblk = (P + per_wg - 1) / per_wg;
    if (nblk > 0x7fffffffLL) {
        sd_set_error("sd_seg_query: too many points");
        return -1;
    }
    const float neg_vox = -voxel_size;
    hipStream_t s = (hipStream_t)stream;
    const size_t lds_bytes = (size_t)SG_NSLOT * SG_SLOT + (want_seg ? 8 * (size_t)h->d_full : 0);
    const int mode = (dino_full ? 1 : 0) | (want_seg ? 2 : 0);
    // fp8 norm only for the labels / seg outputs (dino_full is the bf16 expansion)
    const bool f8 = h->w2_f8 != nullptr && mode == 2;
#define SG_LAUNCH(M, F)                                                                            \
    hipLaunchKernelGGL((k_seg_head<M, F>), dim3((unsigned)nblk), dim3(SG_WAVES * 64), lds_bytes, s, dino, \
                       (int32_t)(dino_dtype == SD_BF16), P, \
                       h->d_full, sigma, neg_vox, *h, labels, seg, dino_full)
#define SG_LAUNCH16(M)                                                                              \
    hipLaunchKernelGGL((k_seg_head16<M>), dim3((unsigned)nblk), dim3(SG_WAVES * 64), lds_bytes, s, dino, \
                       (int32_t)(dino_dtype == SD_BF16), P, h->d_full, sigma, neg_vox, *h, labels, seg, \
                       dino_full)
    if (h->frag_layout == SD_SEG_FRAG16) {
        if (mode == 1) SG_LAUNCH16(1);
        else if (mode == 2) SG_LAUNCH16(2);
        else SG_LAUNCH16(3);
    } else switch (mode) {
    case 1: SG_LAUNCH(1, false); break;
    case 2:
        if (f8) SG_LAUNCH(2, true); else SG_LAUNCH(2, false);
        break;
    default: SG_LAUNCH(3, false); break;
    }
#undef SG_LAUNCH
#undef SG_LAUNCH16
    if (hipGetLastError() != hipSuccess) {
        sd_set_error("sd_seg_query: launch failed");
        return -2;
    }
    return 0;
}
