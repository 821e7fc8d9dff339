// Shared helpers for the gfx950 (CDNA4) kernels of mrsum.
//
// Conventions (all kernels):
//   * bf16 tensors are moved as 16-byte vectors (8 x bf16 per lane); scalar
//     bf16 traffic is never used on a hot path (cdna_hip_programming.md G13).
//   * math is fp32; fp32 -> bf16 is a plain cast, which hipcc lowers to
//     v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
//   * wavefront = 64 lanes; every block size is a multiple of 64.
//   * every extern "C" launcher takes raw device pointers + a hipStream_t,
//     never allocates or synchronises (legal inside hipGraph capture) and
//     returns hipGetLastError() as an int.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <math.h>

#define MRSUM_API extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // 16-B staging register (SROA-friendly, unlike HIP's uint4 struct)

static constexpr int WAVE = 64;

__device__ __forceinline__ float bf16_bits_to_f32(uint32_t bits16) {
    return __uint_as_float(bits16 << 16);
}

// 8 packed bf16 (one uint4) -> 8 floats
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    bf16 x = (bf16)a, y = (bf16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide sum for blockDim.x <= 1024 (uses 16 floats of LDS).
__device__ __forceinline__ float block_sum(float v, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    v = wave_sum(v);
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float t = lane < nw ? red[lane] : 0.f;
    t = wave_sum(t);
    __syncthreads();
    return t;
}

// Loads that bypass this CU's L1 (buffer_load ... sc1, aux 16): they read the XCD's L2 / memory copy, so
// a split-K last arriver can read other workgroups' write-through (sc1) stores of THIS launch without an
// agent-scope acquire (buffer_inv sc1 + wait, ~1.7 us) -- the hand-off form of MI355X_MICROARCH.md
// "Valid forms" row 1 / cdna_hip_programming.md Guideline 16: every payload store sc1 and drained before
// the ticket add, the last adder loads after its add returned, the other waves after a barrier, EVERY
// load of the payload such a load.  ``base`` must be wave-uniform (one buffer resource), ``off`` bytes.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sc1_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, int off) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
__device__ __forceinline__ float2 ld_sc1_f2(__amdgpu_buffer_rsrc_t r, int off) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16);
    return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}

static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
