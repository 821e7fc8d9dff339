// Peer-to-peer hand-off primitives shared by the custom all-reduce (custom_ar.hip) and the decode GEMMs
// whose split-K last arriver all-reduces its column tile across the tensor-parallel group in its own
// epilogue (stream_gemm.hip "TP push").
//
// Every rank owns one uncached (hipDeviceMallocUncached) allocation, mapped by every peer over xGMI:
//     [ header HDR: one-shot flags | push-row flags ] [ one-shot slots ] [ push-row slots ]
//     [ granule-push slots: 2 parities x world ranks x slot bytes of tagged words (no flags) ]
// Uncached memory keeps remote payloads and flags out of every L2 (no stale lines across GPUs).
#pragma once
#include "common.h"

namespace mrsum_ar {
constexpr int MAX_RANKS = 8;
constexpr int MAX_BLOCKS = 64;
constexpr size_t HDR = 64 * 1024;         // flags header; slot 0 of the one-shot kernel starts here
constexpr size_t CH = 16 * 1024;          // one-shot bytes per block
constexpr int MAX_ROWS = 256;             // push-row kernel (ar_add_rmsnorm) rows
constexpr size_t PUSH_FLAGS = 16 * 1024;  // [MAX_ROWS][MAX_RANKS] u32
// GEMM-epilogue push: one epoch counter per 16 output columns (granule)
constexpr int GRAN = 16;
constexpr int MAX_GRAN = 8192 / GRAN;
static_assert(PUSH_FLAGS >= (size_t)MAX_BLOCKS * MAX_RANKS * 4, "flag regions overlap");
static_assert(PUSH_FLAGS + (size_t)MAX_ROWS * MAX_RANKS * 4 <= HDR, "push flags exceed header");

struct Peers {
    char* base[MAX_RANKS];  // every rank's allocation (mine included)
};

struct ArHandle {
    int rank, world;
    size_t max_bytes;
    char* mine;             // my uncached allocation
    void* opened[MAX_RANKS];
    Peers peers;
    unsigned* epochs;       // [MAX_BLOCKS] local device counters (regular memory)
    unsigned* error;        // [1] set on a timed-out wait
    unsigned* push_epochs;  // [MAX_ROWS] per-row counters of the push-row kernel
    unsigned* gran_epochs;  // [MAX_GRAN] per-granule counters of the GEMM-epilogue push
};

// byte offsets inside every allocation
constexpr size_t push_off(size_t slot_bytes) { return HDR + 2 * slot_bytes; }
inline size_t gran_off(size_t slot_bytes, int world) { return push_off(slot_bytes) + 2 * (size_t)world * slot_bytes; }
inline size_t alloc_bytes(size_t slot_bytes, int world) { return gran_off(slot_bytes, world) + 2 * (size_t)world * slot_bytes; }

// What a GEMM epilogue needs to all-reduce its tiles (kernel argument; world == 0: no TP push).
struct TPPush {
    Peers peers;
    int rank, world;
    long long region;   // gran_off: parity p, source rank q at region + (p * world + q) * slot
    long long slot;     // bytes per source rank
    unsigned* epochs;   // gran_epochs
    unsigned* error;
};

inline TPPush tp_push_of(const ArHandle* h) {
    TPPush t;
    for (int r = 0; r < MAX_RANKS; ++r) t.peers.base[r] = h ? h->peers.base[r] : nullptr;
    t.rank = h ? h->rank : 0;
    t.world = h ? h->world : 0;
    t.region = h ? (long long)gran_off(h->max_bytes, h->world) : 0;
    t.slot = h ? (long long)h->max_bytes : 0;
    t.epochs = h ? h->gran_epochs : nullptr;
    t.error = h ? h->error : nullptr;
    return t;
}

__device__ __forceinline__ void st_release_sys(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Write-through publish (WT): payload stored with system-scope relaxed atomic stores (global_store
// sc0 sc1: coherent at system scope once acknowledged), every store drained (s_waitcnt vmcnt(0)),
// then a relaxed system-scope flag store.  The fenced form (release fence + release flag store)
// emits two buffer_wbl2, each writing back EVERY dirty line of this XCD's L2 -- inside a decode graph
// the preceding GEMM's split-K slabs -- for a payload that lives in uncached memory and never
// touches L2.  (The same drained-payload-then-flag hand-off as attn_decode.hip's write-through merge;
// MI355X_MICROARCH.md "Valid forms".)
__device__ __forceinline__ void st_wt8(void* p, unsigned long long v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_flag(unsigned* p, unsigned v, bool wt) {
    if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else st_release_sys(p, v);
}

// Spin (relaxed system-scope loads, s_sleep between polls) until *f >= epoch, bounded in WALL time by
// the 100 MHz s_memrealtime counter: ranks are launched by independent host threads and may lag each
// other by host-side jitter (GC, logging, a first kernel-library load), so the bound is generous (4 s) but
// finite -- a peer that is gone sets the sticky error word (checked by the host after every generate)
// instead of hanging the GPU.  Once the error is set, later waits do not spin at all.
constexpr unsigned long long WAIT_TICKS = 400000000ull;  // 4 s at 100 MHz

__device__ __forceinline__ void wait_flag(const unsigned* f, unsigned epoch, unsigned* error) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= epoch) return;
    if (__hip_atomic_load(error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > WAIT_TICKS) {
            atomicOr(error, 1u);
            break;
        }
    }
}

// ---- TP push of GEMM output tiles (stream_gemm.hip header "TP push"): tagged 8-byte words --------------
// An item = 4 consecutive columns c.. of one output row: two words (2 bf16 | epoch << 32) at byte offset
// off = (row * ncols + c) * 4 of every rank's (parity, source rank) slot.
__device__ __forceinline__ long long tp_item_off(int row, int ncols, int c) {
    return ((long long)row * ncols + c) * 4;
}

// push bf16(v) of this rank's item to every rank (fire and forget)
__device__ __forceinline__ void tp_push_item(const TPPush& tp, long long off, unsigned epoch, float4 v) {
    const unsigned long long tag = (unsigned long long)epoch << 32;
    const unsigned long long w0 = tag | pack2(v.x, v.y), w1 = tag | pack2(v.z, v.w);
    const long long par = (long long)(epoch & 1) * tp.world;
    for (int p = 0; p < tp.world; ++p) {
        char* d = tp.peers.base[p] + tp.region + (par + tp.rank) * tp.slot + off;
        st_wt8(d, w0);
        st_wt8(d + 8, w1);
    }
}

// poll my own slots until every rank's two words of the item carry ``epoch`` (the data is its own flag:
// 8-byte single-copy-atomic system-scope loads of uncached memory, no fence), then the rank-ordered fp32
// sum of the bf16 values -- identical on every rank.  Bounded like wait_flag (sticky error word).
__device__ __forceinline__ float4 tp_gather_item(const TPPush& tp, long long off, unsigned epoch) {
    unsigned long long a[MAX_RANKS][2];
    unsigned done = 0;
    const unsigned full = (1u << tp.world) - 1u;
    const char* mine = tp.peers.base[tp.rank] + tp.region + (long long)(epoch & 1) * tp.world * tp.slot + off;
    unsigned long long t0 = 0;
    for (int spin = 0;; ++spin) {
#pragma unroll
        for (int q = 0; q < MAX_RANKS; ++q)
            if (q < tp.world && !((done >> q) & 1u)) {
                const unsigned long long* w = reinterpret_cast<const unsigned long long*>(mine + q * tp.slot);
                a[q][0] = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                a[q][1] = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
#pragma unroll
        for (int q = 0; q < MAX_RANKS; ++q)
            if (q < tp.world && (a[q][0] >> 32) == epoch && (a[q][1] >> 32) == epoch) done |= 1u << q;
        if (done == full) break;
        if (spin == 0) {
            t0 = __builtin_amdgcn_s_memrealtime();
        } else if (__builtin_amdgcn_s_memrealtime() - t0 > WAIT_TICKS ||
                   __hip_atomic_load(tp.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            atomicOr(tp.error, 1u);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < MAX_RANKS; ++q)
        if (q < tp.world) {
            const unsigned x0 = (unsigned)a[q][0], x1 = (unsigned)a[q][1];
            acc.x += __uint_as_float(x0 << 16);
            acc.y += __uint_as_float(x0 & 0xffff0000u);
            acc.z += __uint_as_float(x1 << 16);
            acc.w += __uint_as_float(x1 & 0xffff0000u);
        }
    return acc;
}
}  // namespace mrsum_ar
