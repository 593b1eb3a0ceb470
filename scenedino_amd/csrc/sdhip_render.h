// sdhip_render.h -- device helpers shared by the gfx950 projected-grid render kernels
// (sdhip_proj.hip: per-ray global gather; sdhip_tile.hip: LDS-staged tap tiles).
#pragma once
#include "sdhip_point.h"

// 16-bit element traits.  Blend of the pair-interleaved projected grid (k_project):
// every dword of a row holds (P[x0][c], P[x1][c]) of one channel c, so a bilinear
// sample is two v_dot2 per channel, row y0 . (w00, w01) + row y1 . (w10, w11), in f32
// with one rounding to the 16-bit operand type.
template <int P> struct T16;
template <> struct T16<SD_F16> {
    typedef f16x8 Frag;
    typedef _Float16 E;
    static __device__ __forceinline__ f32x4 mma(const Frag &a, const Frag &b, const f32x4 &c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x16 mma32(const Frag &a, const Frag &b, const f32x16 &c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint16_t bits(float f) {
        return __builtin_bit_cast(uint16_t, (_Float16)f);
    }
    // x . w with a zero accumulator (VOP3P form: no v_mov of the zero)
    static __device__ __forceinline__ float dot2z(uint32_t x, uint32_t w) {
        float r;
        asm("v_dot2_f32_f16 %0, %1, %2, 0" : "=v"(r) : "v"(x), "v"(w));
        return r;
    }
    static __device__ __forceinline__ float dot2(uint32_t x, uint32_t w, float c) {
        return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, x), __builtin_bit_cast(f16x2, w), c, false);
    }
};
template <> struct T16<SD_BF16> {
    typedef bf16x8 Frag;
    typedef __bf16 E;
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    static __device__ __forceinline__ f32x4 mma(const Frag &a, const Frag &b, const f32x4 &c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ f32x16 mma32(const Frag &a, const Frag &b, const f32x16 &c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint16_t bits(float f) {
        return __builtin_bit_cast(uint16_t, (__bf16)f);
    }
    static __device__ __forceinline__ float dot2z(uint32_t x, uint32_t w) {
        float r;
        asm("v_dot2_f32_bf16 %0, %1, %2, 0" : "=v"(r) : "v"(x), "v"(w));
        return r;
    }
    static __device__ __forceinline__ float dot2(uint32_t x, uint32_t w, float c) {
        return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, x), __builtin_bit_cast(bf16x2, w), c, false);
    }
};

// two floats -> one packed 16-bit pair (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32, RNE)
template <typename E>
__device__ __forceinline__ uint32_t sd_pack2(float a, float b) {
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    typedef __attribute__((ext_vector_type(2))) E e2;
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, e2));
}

// 16-bit halves of a packed pair -> f32
template <int P> __device__ __forceinline__ float sd_unpack_lo(uint32_t d) {
    if (P == SD_BF16) return bf16lo(d);
    return (float)__builtin_bit_cast(f16x2, d)[0];
}
template <int P> __device__ __forceinline__ float sd_unpack_hi(uint32_t d) {
    if (P == SD_BF16) return bf16hi(d);
    return (float)__builtin_bit_cast(f16x2, d)[1];
}

// blend weights as the ray pass stores them: (w00, w01), (w10, w11) packed in E
template <int P>
__device__ __forceinline__ uint4 sd_pack_w(float w00, float w01, float w10, float w11) {
    typedef typename T16<P>::E E;
    return uint4{sd_pack2<E>(w00, w01), sd_pack2<E>(w10, w11), 0u, 0u};
}

// 8 channels of one sample from its four plain taps (16 B = 8 channels each): a = (x0, y0),
// b = (x0 + 1, y0), c = (x0, y0 + 1), d = (x0 + 1, y0 + 1).  v_perm pairs the two
// horizontal taps of a channel into one dword, then per channel
//   row y0 . (w00, w01) + row y1 . (w10, w11)
// as two v_dot2 in f32 with one rounding to the 16-bit operand type.
template <int P>
__device__ __forceinline__ typename T16<P>::Frag sd_blend_plain(const uint4 &a, const uint4 &b,
                                                               const uint4 &c, const uint4 &d,
                                                               const uint4 &wp) {
    typedef T16<P> Tr;
    const uint32_t A[4] = {a.x, a.y, a.z, a.w}, B[4] = {b.x, b.y, b.z, b.w};
    const uint32_t C[4] = {c.x, c.y, c.z, c.w}, D[4] = {d.x, d.y, d.z, d.w};
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t p0 = __builtin_amdgcn_perm(B[i], A[i], 0x05040100u);
        const uint32_t p1 = __builtin_amdgcn_perm(B[i], A[i], 0x07060302u);
        const uint32_t q0 = __builtin_amdgcn_perm(D[i], C[i], 0x05040100u);
        const uint32_t q1 = __builtin_amdgcn_perm(D[i], C[i], 0x07060302u);
        const float lo = Tr::dot2(p0, wp.x, Tr::dot2z(q0, wp.y));
        const float hi = Tr::dot2(p1, wp.x, Tr::dot2z(q1, wp.y));
        o[i] = sd_pack2<typename Tr::E>(lo, hi);
    }
    return __builtin_bit_cast(typename Tr::Frag, uint4{o[0], o[1], o[2], o[3]});
}

// DPP with "old" = 1.0 for lanes whose source is outside the row (bound_ctrl off)
#define SD_DPP1(x, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, 1.f), \
                                                          __builtin_bit_cast(int, (x)), (ctrl), 0xf, 0xf, false))
#define SD_DPP0(x, ctrl) \
    __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, (x)), (ctrl), 0xf, 0xf, true))

// inclusive product scan over the 16 lanes of every row (row_shr 1, 2, 4, 8)
__device__ __forceinline__ float sd_scan_mul16(float x) {
    x *= SD_DPP1(x, 0x111);
    x *= SD_DPP1(x, 0x112);
    x *= SD_DPP1(x, 0x114);
    x *= SD_DPP1(x, 0x118);
    return x;
}
// sum over the 16 lanes of every row, result in every lane (row_ror 8, 4, 2, 1)
__device__ __forceinline__ float sd_rowsum16(float x) {
    x += SD_DPP0(x, 0x128);
    x += SD_DPP0(x, 0x124);
    x += SD_DPP0(x, 0x122);
    x += SD_DPP0(x, 0x121);
    return x;
}

// sin of an angle given in revolutions (x / 2 pi): one range reduction + v_sin_f32
__device__ __forceinline__ float sd_sin_rev(float r) {
    return __builtin_amdgcn_sinf(__builtin_amdgcn_fractf(r));
}

// Positional-code fragment of chunk pc for lane group g (element e):
//   G = 2 pc + (g >> 1), phase = g & 1 (0: sin, 1: cos = sin(x + pi/2))
//   G < 3, e < 6 : sin(v[e % 3] * 1.5 * 2^(2G + (e >= 3)) + phase * pi/2)
//   G = 0, e >= 6: raw inputs (g = 0: x, y; g = 1: z~, 0)
//   otherwise don't-care: the packed code weights of those slots are zero
//   (scenedino_amd/mlp_pack.py: proj_pe_col gives the W_in column of every slot).
// The angle is formed in revolutions, fmaf(v * 4^(g >> 1), 1.5 * 2^k / 2 pi, phase / 4).
template <typename Frag, typename E>
__device__ __forceinline__ Frag sd_code_frag(const float v[3], int pc, int g) {
    const float ph = (g & 1) ? 0.25f : 0.f;
    const float ls = (g >> 1) ? 4.f : 1.f;
    const float u[3] = {v[0] * ls, v[1] * ls, v[2] * ls};
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (e < 6) {
            const float f = 1.5f * (float)(1 << (4 * pc + (e >= 3 ? 1 : 0))) * 0.15915494309189535f;
            r[e] = sd_sin_rev(fmaf(u[e % 3], f, ph));
        } else if (pc == 0) {
            r[e] = (g >> 1) ? 0.f : (g == 0 ? v[e - 6] : (e == 6 ? v[2] : 0.f));
        } else {
            r[e] = 0.f;
        }
    }
    const uint4 u4 = {sd_pack2<E>(r[0], r[1]), sd_pack2<E>(r[2], r[3]), sd_pack2<E>(r[4], r[5]),
                      sd_pack2<E>(r[6], r[7])};
    return __builtin_bit_cast(Frag, u4);
}

// ReLU of two packed 16-bit values (bf16 or f16): a negative value has the sign bit
// set, i.e. is a negative int16, so max_i16(x, 0) clamps it to +0.
__device__ __forceinline__ uint32_t sd_relu2(uint32_t x) {
    typedef __attribute__((ext_vector_type(2))) short s16x2;
    const s16x2 v = __builtin_bit_cast(s16x2, x);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, (s16x2){0, 0}));
}
