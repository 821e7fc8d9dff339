// One-shot peer-to-peer all-reduce over IPC-mapped buffers (the decode
// all-reduces of tensor-parallel Llama layers are B x 16 KiB, latency-bound, and 2 per layer).
//
// Every rank owns one uncached (hipDeviceMallocUncached) device allocation
//     [ flags: MAX_BLOCKS x MAX_RANKS u32 | pad | slot 0 | slot 1 ]    slot = max_bytes
// whose IPC handle is exchanged once; each rank maps all peers' allocations (xGMI on a node).
// A call (fp32 sum or u64 max over n bytes <= 1 MiB) runs ceil(n / 16 KiB) workgroups; block b owns
// bytes [16 KiB b, 16 KiB (b+1)):
//   1. copy my slice of `in` into MY slot (epoch & 1)            -- local uncached stores
//   2. system-scope release store of `epoch` into flags[b][me] of EVERY rank (remote over xGMI)
//   3. spin (system-scope acquire, s_sleep, bounded) until my flags[b][r] >= epoch for all r
//   4. out[slice] = sum_r slot_r[slice]                            -- remote uncached loads
// The epoch is a per-block counter in device memory advanced by the block itself, so the kernel
// is replay-safe inside a hipGraph (no host-side arguments change between calls).  Reuse of a slot
// two calls later is safe: passing call e+1's flag wait for block b means every peer's block b
// started e+1, i.e. (stream order) finished reading slot e & 1 in call e.
// Uncached memory keeps remote data and flags out of every L2 (no stale lines across GPUs); the
// release store orders the slot stores before the flag (buffer_wbl2 + s_waitcnt before it).
// A wait that exceeds its bound sets an error word (read by the host) instead of hanging the GPU.
#include "common.h"

#include <cstring>
#include <new>

namespace {
constexpr int MAX_RANKS = 8;
constexpr int MAX_BLOCKS = 64;
constexpr size_t HDR = 64 * 1024;  // flags region, slot 0 starts here
constexpr size_t CH = 16 * 1024;   // bytes per block (fixed: see ar_oneshot_kernel)

struct Peers {
    char* base[MAX_RANKS];  // every rank's allocation (mine included)
};

struct ArHandle {
    int rank, world;
    size_t max_bytes;
    char* mine;          // my uncached allocation
    void* opened[MAX_RANKS];
    Peers peers;
    unsigned* epochs;    // [MAX_BLOCKS] local device counters (regular memory)
    unsigned* error;     // [1] set on a timed-out wait
};

__device__ __forceinline__ void st_release_sys(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

enum { OP_SUM_F32 = 0, OP_MAX_U64 = 1 };

// Block b always owns bytes [b * CH, (b + 1) * CH) of a message, whatever the op and size, so the
// slot-reuse argument above holds per block across calls of different kinds.
template <int OP>
__global__ __launch_bounds__(256) void ar_oneshot_kernel(Peers peers, int rank, int world, size_t slot_bytes,
                                                         const char* __restrict__ in, char* __restrict__ out,
                                                         size_t nbytes, unsigned* __restrict__ epochs,
                                                         unsigned* __restrict__ error) {
    constexpr int VB = OP == OP_SUM_F32 ? 16 : 8;  // vector bytes
    __shared__ unsigned s_epoch;
    const int b = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) s_epoch = epochs[b] + 1;
    __syncthreads();
    const unsigned epoch = s_epoch;
    const size_t off = HDR + (size_t)(epoch & 1) * slot_bytes;
    const size_t b0 = (size_t)b * CH, b1 = b0 + CH < nbytes ? b0 + CH : nbytes;

    // 1. my slice -> my slot
    char* mine = peers.base[rank] + off;
    for (size_t i = b0 + (size_t)tid * VB; i < b1; i += 256 * VB) {
        if constexpr (VB == 16) *reinterpret_cast<float4*>(mine + i) = *reinterpret_cast<const float4*>(in + i);
        else *reinterpret_cast<unsigned long long*>(mine + i) = *reinterpret_cast<const unsigned long long*>(in + i);
    }
    // every wave retires its own slot stores at system scope before the flag can be published
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // 2. announce to every rank
    if (tid < world) {
        unsigned* f = reinterpret_cast<unsigned*>(peers.base[tid]) + b * MAX_RANKS + rank;
        st_release_sys(f, epoch);
    }
    // 3. wait for every rank's slice b (relaxed polling, one acquire after: the invalidate it
    //    implies runs once, and covers the whole block's later reads through the barrier)
    if (tid < world) {
        const unsigned* f = reinterpret_cast<const unsigned*>(peers.base[rank]) + b * MAX_RANKS + tid;
        // sticky error: once a wait has timed out, later calls do not wait again (the host sees the
        // error word at its next check and stops using this path)
        long spins = __hip_atomic_load(error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? (1L << 22) : 0;
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1L << 22)) {  // ~ a second: a peer is gone or late; flag it and fall through
                atomicOr(error, 1u);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // 4. combine every rank's copy of the slice
    for (size_t i = b0 + (size_t)tid * VB; i < b1; i += 256 * VB) {
        if constexpr (OP == OP_SUM_F32) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int r = 0; r < world; ++r) {
                const float4 v = *reinterpret_cast<const float4*>(peers.base[r] + off + i);
                acc.x += v.x;
                acc.y += v.y;
                acc.z += v.z;
                acc.w += v.w;
            }
            *reinterpret_cast<float4*>(out + i) = acc;
        } else {
            unsigned long long m = 0;
            for (int r = 0; r < world; ++r) {
                const unsigned long long v = *reinterpret_cast<const unsigned long long*>(peers.base[r] + off + i);
                m = v > m ? v : m;
            }
            *reinterpret_cast<unsigned long long*>(out + i) = m;
        }
    }
    if (tid == 0) epochs[b] = epoch;
}

static int launch_ar(ArHandle* h, int op, const void* in, void* out, size_t nbytes, hipStream_t s) {
    if (nbytes == 0) return 0;
    if (nbytes > h->max_bytes || nbytes > (size_t)MAX_BLOCKS * CH) return (int)hipErrorInvalidValue;
    for (int r = 0; r < h->world; ++r)
        if (!h->peers.base[r]) return (int)hipErrorInvalidValue;
    const int nblk = (int)((nbytes + CH - 1) / CH);
    if (op == OP_SUM_F32)
        ar_oneshot_kernel<OP_SUM_F32><<<nblk, 256, 0, s>>>(h->peers, h->rank, h->world, h->max_bytes,
                                                           (const char*)in, (char*)out, nbytes, h->epochs, h->error);
    else
        ar_oneshot_kernel<OP_MAX_U64><<<nblk, 256, 0, s>>>(h->peers, h->rank, h->world, h->max_bytes,
                                                           (const char*)in, (char*)out, nbytes, h->epochs, h->error);
    return (int)hipGetLastError();
}

MRSUM_API void* mrsum_ar_create(int rank, int world, size_t max_bytes) {
    if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world || max_bytes % 16) return nullptr;
    ArHandle* h = new (std::nothrow) ArHandle();
    if (!h) return nullptr;
    h->rank = rank;
    h->world = world;
    h->max_bytes = max_bytes;
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, HDR + 2 * max_bytes, hipDeviceMallocUncached) != hipSuccess) {
        delete h;
        return nullptr;
    }
    h->mine = (char*)p;
    if (hipMemset(p, 0, HDR) != hipSuccess || hipMalloc((void**)&h->epochs, MAX_BLOCKS * sizeof(unsigned) + 64)) {
        (void)hipFree(p);
        delete h;
        return nullptr;
    }
    (void)hipMemset(h->epochs, 0, MAX_BLOCKS * sizeof(unsigned) + 64);
    h->error = h->epochs + MAX_BLOCKS;
    for (int r = 0; r < MAX_RANKS; ++r) {
        h->peers.base[r] = nullptr;
        h->opened[r] = nullptr;
    }
    h->peers.base[rank] = h->mine;
    (void)hipDeviceSynchronize();
    return h;
}

// 64-byte IPC handle of this rank's allocation
MRSUM_API int mrsum_ar_ipc_handle(void* hv, void* out64) {
    auto h = (ArHandle*)hv;
    hipIpcMemHandle_t ih;
    hipError_t e = hipIpcGetMemHandle(&ih, h->mine);
    if (e != hipSuccess) return (int)e;
    std::memcpy(out64, &ih, sizeof(ih));
    return 0;
}

// handles: world x 64 bytes (this rank's own entry is ignored)
MRSUM_API int mrsum_ar_open(void* hv, const void* handles) {
    auto h = (ArHandle*)hv;
    for (int r = 0; r < h->world; ++r) {
        if (r == h->rank) continue;
        hipIpcMemHandle_t ih;
        std::memcpy(&ih, (const char*)handles + 64 * r, sizeof(ih));
        void* p = nullptr;
        hipError_t e = hipIpcOpenMemHandle(&p, ih, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return (int)e;
        h->opened[r] = p;
        h->peers.base[r] = (char*)p;
    }
    return 0;
}

// in-place allowed; n fp32 elements, n % 4 == 0, 4 n <= min(max_bytes, 1 MiB)
MRSUM_API int mrsum_ar_allreduce_f32(void* hv, const void* in, void* out, size_t n, hipStream_t s) {
    if (n % 4) return (int)hipErrorInvalidValue;
    return launch_ar((ArHandle*)hv, OP_SUM_F32, in, out, n * sizeof(float), s);
}

// element-wise max of n u64 (sampler keys), in-place allowed
MRSUM_API int mrsum_ar_allreduce_max_u64(void* hv, const void* in, void* out, size_t n, hipStream_t s) {
    return launch_ar((ArHandle*)hv, OP_MAX_U64, in, out, n * sizeof(unsigned long long), s);
}

MRSUM_API int mrsum_ar_error(void* hv) {
    auto h = (ArHandle*)hv;
    unsigned v = 0;
    if (hipMemcpy(&v, h->error, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int)v;
}

MRSUM_API void mrsum_ar_destroy(void* hv) {
    auto h = (ArHandle*)hv;
    if (!h) return;
    (void)hipDeviceSynchronize();
    for (int r = 0; r < MAX_RANKS; ++r)
        if (h->opened[r]) (void)hipIpcCloseMemHandle(h->opened[r]);
    (void)hipFree(h->mine);
    (void)hipFree(h->epochs);
    delete h;
}
