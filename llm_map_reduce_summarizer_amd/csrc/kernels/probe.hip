// HBM streaming probe (calibration tool, tools/bench_kernels.py): reads
// `bytes` with 16-B loads, UNROLL loads in flight per lane, grid-stride, and
// writes one word per workgroup so the loads cannot be eliminated.  Gives the
// floor for "a kernel that streams X MB" on this chip, boundary included,
// against which the decode GEMMs are judged.
#include "common.h"

template <int UNROLL>
__global__ __launch_bounds__(256) void stream_probe_kernel(const uint4* __restrict__ src, size_t n16,
                                                           unsigned* __restrict__ sink) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * UNROLL;
    for (size_t base = (size_t)blockIdx.x * 256 * UNROLL + threadIdx.x; base < n16; base += stride) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t i = base + (size_t)u * 256;
            v[u] = i < n16 ? src[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

MRSUM_API int mrsum_stream_probe(const void* src, size_t bytes, void* sink, int blocks, int unroll, hipStream_t s) {
    const size_t n16 = bytes / 16;
    if (unroll == 4) stream_probe_kernel<4><<<blocks, 256, 0, s>>>((const uint4*)src, n16, (unsigned*)sink);
    else if (unroll == 8) stream_probe_kernel<8><<<blocks, 256, 0, s>>>((const uint4*)src, n16, (unsigned*)sink);
    else stream_probe_kernel<16><<<blocks, 256, 0, s>>>((const uint4*)src, n16, (unsigned*)sink);
    return (int)hipGetLastError();
}

// Access-pattern probe (tools/exp_row_pattern.py): one workgroup per block of R consecutive rows of
// row_bytes each (the decode GEMM's weight tile), the block read slot by slot -- slot j = bytes
// [j C, (j + 1) C) of every row of the block, rows in order -- with UNROLL 16-B loads in flight per lane.
// C = 256 is the stream GEMM's k-block (128 bf16) per row per ring slot; C = row_bytes streams the block
// as one contiguous range.  Measures what the DRAM side pays for the tile's 256-B-per-row order.
template <int UNROLL>
__global__ __launch_bounds__(512) void stream_probe_rows_kernel(const char* __restrict__ src, int row_bytes, int R,
                                                                int C, unsigned* __restrict__ sink) {
    const int per_row = C / 16, per_slot = R * per_row;
    const int n = (row_bytes / C) * per_slot;
    const char* blk = src + (size_t)blockIdx.x * R * row_bytes;
    unsigned acc = 0;
    for (int base = threadIdx.x; base < n; base += blockDim.x * UNROLL) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const int q = base + u * blockDim.x;
            const int j = q / per_slot, w = q - j * per_slot;
            const int r = w / per_row, c = w - r * per_row;
            v[u] = q < n ? *reinterpret_cast<const uint4*>(blk + (size_t)r * row_bytes + (size_t)j * C + c * 16)
                         : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

MRSUM_API int mrsum_stream_probe_rows(const void* src, int rows, int row_bytes, int R, int C, int threads,
                                      void* sink, hipStream_t s) {
    if (R <= 0 || rows % R || C % 16 || row_bytes % C || (threads != 256 && threads != 512)) return (int)hipErrorInvalidValue;
    stream_probe_rows_kernel<16><<<rows / R, threads, 0, s>>>((const char*)src, row_bytes, R, C, (unsigned*)sink);
    return (int)hipGetLastError();
}
