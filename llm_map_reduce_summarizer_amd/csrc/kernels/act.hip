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

__global__ __launch_bounds__(256) void swiglu_kernel(const bf16* __restrict__ gu, bf16* __restrict__ out, int T,
                                                     int F) {
    const int fv = F >> 3;
    const size_t n = (size_t)T * fv;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / fv, c = i % fv;  // output features [8c, 8c+8)
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
    const size_t n = (size_t)T * (F / 8);
    const int blocks = (int)std::min<size_t>((n + 255) / 256, 256 * 16);
    swiglu_kernel<<<blocks, 256, 0, s>>>((const bf16*)gu, (bf16*)out, T, F);
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
