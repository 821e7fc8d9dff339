// Diagnostic (tools/exp_stream_dma.py, not part of the package): what the chip's LDS-DMA path delivers for
// the decode stream GEMM's weight pattern with NO compute, to split the stream kernel's time into "the
// DMA stream" and "everything else" (sync, fragment reads, MFMA, epilogue).
//
// One workgroup of WPB waves per 16 * WPB weight rows (the stream GEMM's column tile, grid N / (16 WPB)),
// K-blocks of 128 bf16 per row per slot, D slots in ONE __shared__ array; every wave issues 4 x 1 KiB
// pieces per slot (8 rows x 128 B each, the GEMM's exact source addresses and swizzle), policy nt.
//   MODE 0: the GEMM's loop -- counted vmcnt leaving D - 2 slots in flight, raw s_barrier, refill
//   MODE 1: the same without the barrier (each wave runs its own ring)
//   MODE 2: no barrier, the refill issued before the wait: D - 1 slots in flight while slot j is read
// The landed data is folded into one word per lane (a ds_read per slot) so nothing is dead.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

typedef __hip_bfloat16 bf16;

namespace {
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void glds16(const void* g, char* lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, 2);
}

template <int WPB, int D, int MODE>
__global__ __launch_bounds__(64 * WPB, 1) void dma_probe_kernel(const bf16* __restrict__ W, int K, int kper,
                                                                unsigned* __restrict__ sink) {
    constexpr int R = 16 * WPB, SLOT = R * 256;
    __shared__ __attribute__((aligned(1024))) char lds[D * SLOT];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * R;
    const int nkb = kper / 128;  // split-K: workgroup (x, y) streams k [y kper, (y + 1) kper)
    const int prow = lane >> 3, pslot = lane & 7;
    const bf16* wsrc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int q = 4 * w + p;
        const int row = 8 * (q >> 1) + prow;
        wsrc[p] = W + (size_t)(n0 + row) * K + blockIdx.y * kper + 8 * (8 * (q & 1) + (pslot ^ prow));
    }
#define ISSUE(slot, kb)                                                                                 \
    {                                                                                                   \
        char* base = lds + (slot) * SLOT;                                                               \
        _Pragma("unroll") for (int p = 0; p < 4; ++p) glds16(wsrc[p] + (kb), base + (4 * w + p) * 1024); \
    }
    unsigned acc = 0;
#pragma unroll
    for (int s = 0; s < D - 1; ++s) ISSUE(s, min(s, nkb - 1) * 128);
    for (int j = 0; j < nkb; ++j) {
        const int nxt = j + D - 1;
        if (MODE == 2) {
            // refill first (own region: this wave's read of that buffer retired below), then wait for slot j
            // with D - 1 slots still in flight
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (nxt < nkb) ISSUE(nxt % D, nxt * 128);
            if (nxt < nkb) wait_vmcnt<4 * (D - 1)>();
            else wait_vmcnt<0>();
        } else {
            if (j + D - 2 < nkb) wait_vmcnt<4 * (D - 2)>();
            else wait_vmcnt<0>();
            if (MODE == 0) {
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
            if (nxt < nkb) ISSUE(nxt % D, nxt * 128);
        }
        acc ^= *reinterpret_cast<const unsigned*>(lds + (j % D) * SLOT + (4 * w) * 1024 + 16 * lane);
    }
#undef ISSUE
    if (acc == 0x9e3779b9u) sink[(blockIdx.y * gridDim.x + blockIdx.x) * 64 * WPB + tid] = acc;
}
}  // namespace

extern "C" int diag_dma_probe(const void* W, int N, int K, int splits, int wpb, int depth, int mode, void* sink,
                              hipStream_t s) {
    if (splits < 1 || K % (128 * splits) || N % (16 * wpb)) return (int)hipErrorInvalidValue;
    dim3 grid(N / (16 * wpb), splits), block(64 * wpb);
    const int kper = K / splits;
#define L(WPB_, D_, M_) \
    dma_probe_kernel<WPB_, D_, M_><<<grid, block, 0, s>>>((const bf16*)W, K, kper, (unsigned*)sink)
#define BY_MODE(WPB_, D_)                  \
    if (mode == 0) L(WPB_, D_, 0);         \
    else if (mode == 1) L(WPB_, D_, 1);    \
    else L(WPB_, D_, 2);
    if (wpb == 7) {
        if (depth == 3) { BY_MODE(7, 3) }
        else if (depth == 4) { BY_MODE(7, 4) }
        else { BY_MODE(7, 5) }
    } else if (wpb == 4) {
        if (depth == 4) { BY_MODE(4, 4) }
        else if (depth == 6) { BY_MODE(4, 6) }
        else { BY_MODE(4, 8) }
    } else {
        return (int)hipErrorInvalidValue;
    }
#undef BY_MODE
#undef L
    return (int)hipGetLastError();
}
