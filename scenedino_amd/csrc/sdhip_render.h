// sdhip_render.h -- device helpers shared by the gfx950 projected-grid render kernels
// (sdhip_proj.hip: per-ray global gather; sdhip_tile.hip: LDS-staged tap tiles).
#pragma once
#ifndef SD_PE_DIRECT
#define SD_PE_DIRECT 0
#endif
// overflow list of the tile kernel: entries are blocks of SD_LIST_BLK consecutive rays
// (a group of 8 or 12 rays lists 2 or 3 blocks); the fallback kernels render the blocks
#define SD_LIST_BLK 4
#include "sdhip_point.h"
// The lists live in sd_render_proj's work: one per tile workgroup (slot = blockIdx.x; the
// tile grid is one workgroup per CU), [slots] counts, then [slots][cap] block indices.  Every
// tile workgroup writes its count, so nothing is reset before the launch (a 4-byte memset
// was a 5 us fill kernel per frame), and fallback workgroup b renders list b.  cap bounds a
// tile workgroup's rays: its XCD share of the groups over its nwg = slots / 8 workgroups,
// < R / slots + 3 GR <= R / slots + 48.
__host__ __device__ inline int64_t sd_ovf_cap(int64_t R, int64_t slots) {
    return ((R + slots - 1) / slots + 64) / SD_LIST_BLK + 1;
}
__host__ __device__ inline int64_t sd_ovf_words(int64_t R, int64_t slots) {
    return slots + slots * sd_ovf_cap(R, slots);
}

// LDS-DMA of 16 B per active lane (global_load_lds_dwordx4) into lds_addr + 16 * lane, as
// inline asm: issued through the builtin, the compiler treats every later LDS read as a
// possible alias of the in-flight DMA and waits for it (s_waitcnt vmcnt(0)) at the first
// one; the kernels order these DMAs themselves (s_waitcnt vmcnt + barrier before the staged
// data is read).  m0 = LDS destination of lane 0, one wait state after the SALU write.
__device__ __forceinline__ void sd_dma16(const void *src, uint32_t lds_addr) {
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);  // wave-uniform by construction
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src), "s"(lds_addr) : "memory");
}
// the same with the non-temporal hint (a stream read once: the projection's grid sweep)
__device__ __forceinline__ void sd_dma16_nt(const void *src, uint32_t lds_addr) {
    lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt"
                 :: "v"(src), "s"(lds_addr) : "memory");
}

// 16-bit element traits.  Blend of the pair-interleaved projected grid (k_project):
// every dword of a row holds (P[x0][c], P[x1][c]) of one channel c, so a bilinear
// sample is two v_dot2 per channel, row y0 . (w00, w01) + row y1 . (w10, w11), in f32
// with one rounding to the 16-bit operand type.
template <int P> struct T16;
typedef __attribute__((ext_vector_type(4))) short sd_s16x4;
typedef __attribute__((ext_vector_type(4))) _Float16 sd_f16x4;

template <> struct T16<SD_F16> {
    typedef f16x8 Frag;
    typedef sd_f16x4 Frag4;  // 16x16x16 operand (4 elements per lane)
    typedef _Float16 E;
    static __device__ __forceinline__ f32x4 mma16(const Frag4 &a, const Frag4 &b, const f32x4 &c) {
        return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
    }
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
    typedef sd_s16x4 Frag4;  // 16x16x16 operand (4 elements per lane)
    typedef __bf16 E;
    static __device__ __forceinline__ f32x4 mma16(const Frag4 &a, const Frag4 &b, const f32x4 &c) {
        return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
    }
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

// Operand types of the two 16-bit render modes.  F: every operand upstream
// of sigma -- the projected grid P (or the NHWC grid G), the bilinear tap weights, the
// positional-code fragments and their W_in columns, relu(h) and W_sigma.  H: the DINO output
// layer (W_dino x hidden vectors / hidden sums).
//   fp16 mode: F = H = f16.
//   bf16 mode (BASELINE configs[1]): F = f16, H = bf16.  An 8-bit mantissa on any operand
//   upstream of sigma moves the composited depth past the 1e-2 m contract (1.3-3.4 cm with
//   every operand bf16; 0.98 cm with only the code columns bf16 -- the replay of the kernels'
//   arithmetic in tools/lowp_depth_emul.py, profiles/r5_lowp_depth_emul.txt), so bf16 is
//   kept where it costs no depth: the DINO head.  Same MFMA rate either way.
template <int P> struct RMode {
    typedef T16<SD_F16> F;
    typedef T16<P> H;
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
// (P = SD_F16 for both render modes, RMode)
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

// inclusive product scan over the 16 lanes of every row (row_shr 1, 2, 4, 8): one
// v_mul_f32_dpp per step, x = x[l - s] * x in place; a lane whose source lies before its
// row start is not written (bound_ctrl off) and so keeps x, the product with 1.  The
// s_nop 1 covers the VALU-write -> DPP-read hazard of every step.
#ifndef SD_SCAN_ASM
#define SD_SCAN_ASM 1
#endif
__device__ __forceinline__ float sd_scan_mul16(float x) {
#if !SD_SCAN_ASM
    x *= SD_DPP1(x, 0x111);
    x *= SD_DPP1(x, 0x112);
    x *= SD_DPP1(x, 0x114);
    x *= SD_DPP1(x, 0x118);
    return x;
#endif
    asm("s_nop 1\n\tv_mul_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_mul_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_mul_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_mul_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf"
        : "+v"(x));
    return x;
}

// torch softplus (beta 1, threshold 20) on the hardware exp2 / log2 (16-bit render
// modes: ~1e-7 relative, far below the operand rounding)
#ifndef SD_SP_FAST
#define SD_SP_FAST 0  // 1: raw exp2 / log2 softplus (fewer VALU, measured slower in k_render_tile)
#endif
__device__ __forceinline__ float sd_softplus_fast(float x) {
    if (!SD_SP_FAST) return x > 20.f ? x : __logf(1.f + __expf(x));
    const float l = __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(x * 1.4426950408889634f));
    return x > 20.f ? x : l * 0.6931471805599453f;
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

// Positional code (encoding_mode._z + PositionalEncoding, positional_encoding.py:13-80:
// [x, y, z~, sin / cos(1.5 * 2^f * coord), f = 0..5]) of one sample, spread over its 4
// lane groups: group c < 3 holds coordinate c's 12 sinusoids, group 3 the raw inputs.
//   f0 (16x16x32 operand): c < 3: slot 2 f + ph = sin (ph 0) / cos (ph 1) at f = 0..3;
//                          c = 3: x, y, z~, then zeros
//   f1 (16x16x16 operand): c < 3: slot 2 (f - 4) + ph at f = 4, 5;  c = 3: zeros
// (scenedino_amd/mlp_pack.py: proj_pe_col gives the W_in column of every slot).  f = 0 and
// f = 3 are evaluated directly (angle in revolutions, one range reduction + v_sin_f32);
// f = 1, 2, 4, 5 by double-angle steps sin 2a = 2 sin a cos a, cos 2a = 1 - 2 sin^2 a.
template <typename Frag, typename Frag4, typename E>
__device__ __forceinline__ void sd_code_frags(const float v[3], int g, Frag &f0, Frag4 &f1) {
    const float u = g == 0 ? v[0] : (g == 1 ? v[1] : v[2]);
    const float r0 = u * (float)(1.5 / 6.283185307179586);
    const float r3 = u * (float)(12.0 / 6.283185307179586);
    float s[6], c[6];
    s[0] = sd_sin_rev(r0);
    c[0] = sd_sin_rev(r0 + 0.25f);
    s[3] = sd_sin_rev(r3);
    c[3] = sd_sin_rev(r3 + 0.25f);
#if SD_PE_DIRECT
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        const float rf = u * (float)(1.5 / 6.283185307179586) * (float)(1 << f);
        s[f] = sd_sin_rev(rf);
        c[f] = sd_sin_rev(rf + 0.25f);
    }
#else
#pragma unroll
    for (int f = 0; f < 5; ++f) {
        if (f == 2) continue;
        s[f + 1] = (s[f] + s[f]) * c[f];
        c[f + 1] = fmaf(-2.f * s[f], s[f], 1.f);
    }
#endif
    const bool raw = g == 3;
    const uint4 u4 = {raw ? sd_pack2<E>(v[0], v[1]) : sd_pack2<E>(s[0], c[0]),
                      raw ? sd_pack2<E>(v[2], 0.f) : sd_pack2<E>(s[1], c[1]),
                      raw ? 0u : sd_pack2<E>(s[2], c[2]),
                      raw ? 0u : sd_pack2<E>(s[3], c[3])};
    f0 = __builtin_bit_cast(Frag, u4);
    const uint2 u2 = {raw ? 0u : sd_pack2<E>(s[4], c[4]), raw ? 0u : sd_pack2<E>(s[5], c[5])};
    f1 = __builtin_bit_cast(Frag4, u2);
}

// ReLU of two packed 16-bit values (bf16 or f16): a negative value has the sign bit
// set, i.e. is a negative int16, so max_i16(x, 0) clamps it to +0.
__device__ __forceinline__ uint32_t sd_relu2(uint32_t x) {
    typedef __attribute__((ext_vector_type(2))) short s16x2;
    const s16x2 v = __builtin_bit_cast(s16x2, x);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, (s16x2){0, 0}));
}
