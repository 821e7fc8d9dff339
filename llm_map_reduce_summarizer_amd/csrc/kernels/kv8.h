// FP8 paged KV cache (engine --kv-dtype fp8): layout and the row quantiser shared by the writers
// (rope_kv.hip; attn_decode.hip's fused RoPE + KV write) and the readers (attn_decode.hip,
// attn_prefill.hip paged path).
//
// One layer's K (or V) cache is a byte array [num_pages, Hkv, SLAB], SLAB = P * D + 4 * P: the slab
// of (page, kv head) holds the P rows of D OCP e4m3fn bytes, then the P fp32 row scales -- one
// contiguous 8.25 KiB block per (page, head) at P = 64, D = 128, half the bytes of the bf16 page
// plus 3 % for the scales.  x[row][d] = scale[row] * e4m3(q[row][d]).
//
// A row (one token of one kv head) is quantised as a whole when it is written: scale = the power of
// two >= max|x| / 448 (so every element fits e4m3's range), q = RNE e4m3(x / scale).  Power-of-two
// scales make dequantisation exact in bf16 (e4m3's 3 mantissa bits x 2^e), so the readers convert a
// staged row to bf16 with v_cvt_scalef32_pk_bf16_fp8 and the attention math downstream is the bf16
// kernel's, unchanged.
#pragma once
#include "common.h"

namespace kv8 {
constexpr int P = 64, D = 128;
constexpr int SLAB = P * D + 4 * P;  // bytes per (page, kv head)

__device__ __forceinline__ size_t slab_off(int page, int Hkv, int head) {
    return ((size_t)page * Hkv + head) * SLAB;
}

// the power of two >= amax / 448 (1 for an all-zero row), never below 2^-126: a subnormal scale would make
// 1 / scale overflow to inf and a zero element of the row 0 * inf = NaN, poisoning every later attention
// step over the sequence.  Rows with 0 < amax < 448 * 2^-126 quantise against 2^-126 (their elements
// round towards zero, as bf16 would flush them anyway).
constexpr int MIN_SCALE_EXP = -126;
__device__ __forceinline__ float row_scale(float amax) {
    if (!(amax > 0.f)) return 1.f;
    int e;
    const float m = frexpf(amax * (1.f / 448.f), &e);  // amax / 448 = m 2^e, m in [0.5, 1)
    e = m == 0.5f ? e - 1 : e;
    return ldexpf(1.f, e < MIN_SCALE_EXP ? MIN_SCALE_EXP : e);
}

__device__ __forceinline__ unsigned pack4(float a, float b, float c, float d) {
    unsigned w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// 16 consecutive-in-group values of one cache row, held by one lane of an aligned group of
// LANES = D / 16 lanes that together hold the whole row: dims c0 .. c0+7 <- f[0..7], c1 .. c1+7 <- f[8..15].
// The group reduces max|x| with xor shuffles (every lane of the group must call this), then each
// lane stores its 16 bytes; the lane holding dim 0 stores the scale.  ``write`` false: reduce only.
template <int LANES = D / 16>
__device__ __forceinline__ void put_row16(void* cache, int page, int Hkv, int head, int row, int P_, int D_, int c0,
                                          int c1, const float* f, bool write) {
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(f[j]));
#pragma unroll
    for (int o = 1; o < LANES; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
    if (!write) return;
    const float sc = row_scale(amax), inv = 1.f / sc;
    char* base = reinterpret_cast<char*>(cache) + slab_off(page, Hkv, head);
    uint2 lo = make_uint2(pack4(f[0] * inv, f[1] * inv, f[2] * inv, f[3] * inv),
                          pack4(f[4] * inv, f[5] * inv, f[6] * inv, f[7] * inv));
    uint2 hi = make_uint2(pack4(f[8] * inv, f[9] * inv, f[10] * inv, f[11] * inv),
                          pack4(f[12] * inv, f[13] * inv, f[14] * inv, f[15] * inv));
    *reinterpret_cast<uint2*>(base + (size_t)row * D_ + c0) = lo;
    *reinterpret_cast<uint2*>(base + (size_t)row * D_ + c1) = hi;
    if (c0 == 0) *reinterpret_cast<float*>(base + (size_t)P_ * D_ + 4 * row) = sc;
}

// 16 e4m3 bytes (one 16-B chunk of a row) x scale -> 16 bf16 (two 16-B vectors), exact for a power-of-two scale
__device__ __forceinline__ void dequant16(const u32x4 q, float sc, u32x4& lo, u32x4& hi) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    unsigned o[8];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(q[w], sc, false);
        const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(q[w], sc, true);
        o[2 * w] = __builtin_bit_cast(unsigned, a);
        o[2 * w + 1] = __builtin_bit_cast(unsigned, b);
    }
    lo = u32x4{o[0], o[1], o[2], o[3]};
    hi = u32x4{o[4], o[5], o[6], o[7]};
}
}  // namespace kv8
