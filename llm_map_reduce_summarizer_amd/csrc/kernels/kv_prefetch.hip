// KV-cache prefetch into the Infinity Cache for small-batch decode (round 5 experiment, ops.hip.kv_prefetch).
//
// At B = 1 the decode attention of a 13.5k-token context reads 55 MB of K/V per layer in ~16.8 us, 5-6 us
// above a streaming probe of the same bytes (docs/decode_latency.md, round-4 table): its 256 workgroups
// start only after the QKV GEMM (the query is its output) and pay the HBM latency of their first pages on
// the critical path.  The K/V of the OLD positions does not depend on this step, so this kernel -- launched
// on a side stream of the captured decode graph, concurrently with the layer's QKV GEMM -- loads every
// cached page of every sequence once with the default cache policy: the lines land in the 256 MiB Infinity
// Cache (MI355X_MICROARCH.md "Infinity Cache": a table stays resident while it plus everything loaded in
// between fits), and the attention that follows reads them on-die.  Same bytes from HBM, moved earlier and
// beside a weight stream that leaves HBM headroom at B = 1.
//
// Geometry: a page of all kv heads is contiguous in both cache formats (bf16 [pages, Hkv, P, D]: Hkv x P x D x
// 2 bytes; fp8 slabs [pages, Hkv, SLAB]: Hkv x SLAB bytes) -- ``page_bytes`` per cache.  grid (B, WPS): the
// WPS workgroups of sequence b split its ceil(ctx / P) pages; each lane loads 16-B vectors, 8 in flight,
// and folds them into a value that is stored only when ``sink_flag`` is set (never, in the engine: the
// store keeps the loads alive).  Positions are read on the device (a captured graph replays every step).
#include "common.h"

__global__ __launch_bounds__(256) void kv_prefetch_kernel(const u32x4* __restrict__ kc, const u32x4* __restrict__ vc,
                                                          const int* __restrict__ block_tables, int bt_stride,
                                                          const int* __restrict__ positions, int P, int kvec,
                                                          int vvec, unsigned* __restrict__ sink, int sink_flag) {
    const int b = blockIdx.x, wps = gridDim.y, part = blockIdx.y;
    const int ctx = positions[b] + 1;
    const int npages = (ctx + P - 1) / P;
    const int* bt = block_tables + (size_t)b * bt_stride;
    unsigned acc = 0;
    // pages part, part + wps, ...: both caches of one page back to back
    for (int p = part; p < npages; p += wps) {
        const size_t pg = (size_t)bt[p];
        const u32x4* ks = kc + pg * kvec;
        const u32x4* vs = vc + pg * vvec;
        for (int i0 = threadIdx.x; i0 < kvec + vvec; i0 += 256 * 8) {
            u32x4 r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = min(i0 + 256 * u, kvec + vvec - 1);
                r[u] = i < kvec ? ks[i] : vs[i - kvec];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc ^= r[u].x ^ r[u].w;
        }
    }
    if (sink_flag) sink[(size_t)b * wps * 256 + part * 256 + threadIdx.x] = acc;
}

// kc / vc: one layer's caches; kpage_bytes / vpage_bytes: bytes of one page over all kv heads in each
// (multiples of 16); wps: workgroups per sequence.  sink: >= B * wps * 256 uints (written only with
// sink_flag, a test hook that proves the loads happen).
MRSUM_API int mrsum_kv_prefetch(const void* kc, const void* vc, const int* block_tables, int bt_stride,
                                const int* positions, int B, int P, int kpage_bytes, int vpage_bytes, int wps,
                                unsigned* sink, int sink_flag, hipStream_t s) {
    if (B <= 0) return 0;
    if (!kc || !vc || !block_tables || !positions || P <= 0 || wps <= 0 || kpage_bytes <= 0 || vpage_bytes <= 0 ||
        kpage_bytes % 16 || vpage_bytes % 16 || (sink_flag && !sink))
        return (int)hipErrorInvalidValue;
    dim3 grid(B, wps);
    kv_prefetch_kernel<<<grid, 256, 0, s>>>((const u32x4*)kc, (const u32x4*)vc, block_tables, bt_stride, positions, P,
                                            kpage_bytes / 16, vpage_bytes / 16, sink, sink_flag);
    return (int)hipGetLastError();
}
