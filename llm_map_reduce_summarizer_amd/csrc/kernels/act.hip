// SwiGLU activation (K7) and token-embedding gather (K9).
//
// swiglu:  gu [T, 2F] bf16, the fused gate+up GEMM output with its columns in
//          blocks of 16 = [8 gate | 8 up] (the weight layout the decode GEMM's
//          fused SwiGLU epilogue needs); out [T, F] = silu(gate) * up,
//          16-B vectors, grid-stride.
// embed:   ids [T] int32 -> out [T, D] = table[ids]; one block per token,
//          16-B vectors (a row is D*2 bytes = 8 KiB at D=4096).  Ids are
//          clamped to [0, V) so a bad id can never read out of bounds.
#include "common.h"

// grid (F/8/256 column blocks, T rows): no 64-bit div/mod per element (a size_t i / fv here cost
// ~20 us per call at T=48, more than the memory traffic).
__global__ __launch_bounds__(256) void swiglu_kernel(const bf16* __restrict__ gu, bf16* __restrict__ out, int T,
                                                     int F) {
    const int fv = F >> 3;
    const int r = blockIdx.y;
    for (int c = blockIdx.x * 256 + threadIdx.x; c < fv; c += gridDim.x * 256) {  // output features [8c, 8c+8)
        const uint4* row = reinterpret_cast<const uint4*>(gu + r * 2 * (size_t)F);
        float g[8], u[8];  // 16-B vector 2c = gate features [8c, 8c+8), 2c+1 = the matching up
        unpack8(row[2 * c], g);
        unpack8(row[2 * c + 1], u);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
        reinterpret_cast<uint4*>(out + r * (size_t)F)[c] = pack8(g);
    }
}

MRSUM_API int mrsum_swiglu(const void* gu, void* out, int T, int F, hipStream_t s) {
    if (T <= 0) return 0;
    if (F % 8) return (int)hipErrorInvalidValue;
    const int cb = std::min(ceil_div(F / 8, 256), 64);
    for (int t0 = 0; t0 < T; t0 += 65535) {  // grid.y limit
        const int tn = std::min(T - t0, 65535);
        swiglu_kernel<<<dim3(cb, tn), 256, 0, s>>>((const bf16*)gu + (size_t)t0 * 2 * F, (bf16*)out + (size_t)t0 * F,
                                                   tn, F);
    }
    return (int)hipGetLastError();
}

__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ ids, const bf16* __restrict__ table,
                                                    bf16* __restrict__ out, int D, int V) {
    int id = ids[blockIdx.x];
    id = id < 0 ? 0 : (id >= V ? V - 1 : id);
    const uint4* src = reinterpret_cast<const uint4*>(table + (size_t)id * D);
    uint4* dst = reinterpret_cast<uint4*>(out + (size_t)blockIdx.x * D);
    for (int c = threadIdx.x; c < (D >> 3); c += blockDim.x) dst[c] = src[c];
}

MRSUM_API int mrsum_embed(const int* ids, const void* table, void* out, int T, int D, int V, hipStream_t s) {
    if (T <= 0) return 0;
    if (D % 8) return (int)hipErrorInvalidValue;
    embed_kernel<<<T, 256, 0, s>>>(ids, (const bf16*)table, (bf16*)out, D, V);
    return (int)hipGetLastError();
}
