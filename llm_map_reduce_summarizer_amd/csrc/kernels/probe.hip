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
