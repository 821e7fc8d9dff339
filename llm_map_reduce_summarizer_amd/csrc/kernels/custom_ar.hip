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
//   3. spin (system-scope acquire, s_sleep, bounded: wait_flag) until my flags[b][r] >= epoch for all r
//   4. out[slice] = sum_r slot_r[slice]                            -- remote uncached loads
// The epoch is a per-block counter in device memory advanced by the block itself, so the kernel
// is replay-safe inside a hipGraph (no host-side arguments change between calls).  Reuse of a slot
// two calls later is safe: passing call e+1's flag wait for block b means every peer's block b
// started e+1, i.e. (stream order) finished reading slot e & 1 in call e.
// Uncached memory keeps remote data and flags out of every L2 (no stale lines across GPUs); the
// release store orders the slot stores before the flag (buffer_wbl2 + s_waitcnt before it).
// A wait that exceeds its bound sets an error word (read by the host) instead of hanging the GPU.
#include "ar_common.h"

#include <cstring>
#include <new>

using namespace mrsum_ar;

enum { OP_SUM_F32 = 0, OP_MAX_U64 = 1 };

// Block b always owns bytes [b * CH, (b + 1) * CH) of a message, whatever the op and size, so the
// slot-reuse argument above holds per block across calls of different kinds.
template <int OP, bool WT>
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
        if constexpr (WT) {
            const unsigned long long* src = reinterpret_cast<const unsigned long long*>(in + i);
#pragma unroll
            for (int k = 0; k < VB / 8; ++k) st_wt8(mine + i + 8 * k, src[k]);
        } else if constexpr (VB == 16) {
            *reinterpret_cast<float4*>(mine + i) = *reinterpret_cast<const float4*>(in + i);
        } else {
            *reinterpret_cast<unsigned long long*>(mine + i) = *reinterpret_cast<const unsigned long long*>(in + i);
        }
    }
    // every wave retires its own slot stores at system scope before the flag can be published
    if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // 2. announce to every rank
    if (tid < world) {
        unsigned* f = reinterpret_cast<unsigned*>(peers.base[tid]) + b * MAX_RANKS + rank;
        st_flag(f, epoch, WT);
    }
    // 3. wait for every rank's slice b (relaxed polling, one acquire after: the invalidate it
    //    implies runs once, and covers the whole block's later reads through the barrier)
    if (tid < world) {
        const unsigned* f = reinterpret_cast<const unsigned*>(peers.base[rank]) + b * MAX_RANKS + tid;
        // sticky error: once a wait has timed out, later calls do not wait again (the host sees the
        // error word at its next check and stops using this path)
        wait_flag(f, epoch, error);
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


// ---------------------------------------------------------------------------------------------
// Push-mode fused all-reduce + residual add + RMSNorm (the row-parallel o / down projections of a
// TP decode step).  One block per row r of the [T, D] output:
//   1. v = sum_s parts[s][r]                   -- this rank's split-K slabs, fp32, in registers
//   2. store bf16(v) into push[(epoch & 1)][me][r] of EVERY rank   -- remote stores over xGMI
//      (posted: no round trip, unlike reading the peers' copies).  The payload is bf16 (like a
//      Megatron bf16 all-reduce): a push sends T x D x (world - 1) elements per rank, so at decode
//      batches of ~40 rows the xGMI links, not the latency, bound an fp32 payload.
//   3. release fence (system scope), then flag[r][me] = epoch on every rank
//   4. wait until my flag[r][p] >= epoch for all p, acquire
//   5. a = sum_p push[(epoch & 1)][p][r] in rank order from LOCAL memory (every rank adds the same
//      values in the same order: the TP replicas stay bit-identical)
//   6. residual[r] = bf16(residual[r] + a); out[r] = rmsnorm(residual[r]) * w
// Replaces the one-shot all-reduce + add_rmsnorm_parts pair (one launch less per projection, the
// split-K sum folded in, so the producing GEMM keeps its split count under TP).  Slot reuse is safe
// for the same reason as above, per row: a peer can only push call e+2 into my slot e & 1 after
// passing call e+1's wait for row r, which needs my flag of call e+1, i.e. my call e is complete.
template <int VPT, bool WT>  // float4 vectors per thread: D <= 1024 * VPT
__global__ __launch_bounds__(256) void ar_add_rmsnorm_kernel(Peers peers, int rank, int world, size_t slot_bytes,
                                                             const float* __restrict__ parts, int S, int T,
                                                             bf16* __restrict__ residual, const bf16* __restrict__ w,
                                                             bf16* __restrict__ out, int D, int out_stride, float eps,
                                                             unsigned* __restrict__ epochs,
                                                             unsigned* __restrict__ error) {
    __shared__ float red[16];
    __shared__ unsigned s_epoch;
    const int row = blockIdx.x, tid = threadIdx.x;
    const int nv = D >> 2;
    if (tid == 0) s_epoch = epochs[row] + 1;
    float4 v[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = tid + i * 256;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < nv) {
            for (int s = 0; s < S; ++s) {
                const float4 a = reinterpret_cast<const float4*>(parts + ((size_t)s * T + row) * D)[c];
                v[i].x += a.x; v[i].y += a.y; v[i].z += a.z; v[i].w += a.w;
            }
        }
    }
    __syncthreads();
    const unsigned epoch = s_epoch;
    const size_t region = push_off(slot_bytes) + (size_t)(epoch & 1) * world * slot_bytes;
    const size_t mine_off = region + (size_t)rank * slot_bytes + (size_t)row * D * 2;
    uint2 pv[VPT];
#pragma unroll
    for (int i = 0; i < VPT; ++i) pv[i] = make_uint2(pack2(v[i].x, v[i].y), pack2(v[i].z, v[i].w));
    for (int p = 0; p < world; ++p) {
        uint2* dst = reinterpret_cast<uint2*>(peers.base[p] + mine_off);
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int c = tid + i * 256;
            if (c < nv) {
                if constexpr (WT) st_wt8(dst + c, __builtin_bit_cast(unsigned long long, pv[i]));
                else dst[c] = pv[i];
            }
        }
    }
    if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < world) {
        unsigned* f = reinterpret_cast<unsigned*>(peers.base[tid] + PUSH_FLAGS) + row * MAX_RANKS + rank;
        st_flag(f, epoch, WT);
    }
    if (tid < world) {
        const unsigned* f = reinterpret_cast<const unsigned*>(peers.base[rank] + PUSH_FLAGS) + row * MAX_RANKS + tid;
        wait_flag(f, epoch, error);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // 5 + 6: rank-ordered sum from local memory, residual add (bf16 rounding), RMSNorm
    const char* base = peers.base[rank] + region + (size_t)row * D * 2;
    bf16* rrow = residual + (size_t)row * D;
    float ss = 0.f;
    float x[VPT][4];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = tid + i * 256;
        if (c < nv) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int p = 0; p < world; ++p) {
                const uint2 a = reinterpret_cast<const uint2*>(base + (size_t)p * slot_bytes)[c];
                acc.x += __uint_as_float(a.x << 16);
                acc.y += __uint_as_float(a.x & 0xffff0000u);
                acc.z += __uint_as_float(a.y << 16);
                acc.w += __uint_as_float(a.y & 0xffff0000u);
            }
            const uint2 rv = reinterpret_cast<const uint2*>(rrow)[c];
            x[i][0] = (float)(bf16)(__uint_as_float(rv.x << 16) + acc.x);
            x[i][1] = (float)(bf16)(__uint_as_float(rv.x & 0xffff0000u) + acc.y);
            x[i][2] = (float)(bf16)(__uint_as_float(rv.y << 16) + acc.z);
            x[i][3] = (float)(bf16)(__uint_as_float(rv.y & 0xffff0000u) + acc.w);
            reinterpret_cast<uint2*>(rrow)[c] = make_uint2(pack2(x[i][0], x[i][1]), pack2(x[i][2], x[i][3]));
#pragma unroll
            for (int j = 0; j < 4; ++j) ss += x[i][j] * x[i][j];
        }
    }
    ss = block_sum(ss, red);
    const float inv = rsqrtf(ss / (float)D + eps);
    bf16* orow = out + (size_t)row * out_stride;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = tid + i * 256;
        if (c < nv) {
            const uint2 wv = reinterpret_cast<const uint2*>(w)[c];
            const float w0 = __uint_as_float(wv.x << 16), w1 = __uint_as_float(wv.x & 0xffff0000u);
            const float w2 = __uint_as_float(wv.y << 16), w3 = __uint_as_float(wv.y & 0xffff0000u);
            reinterpret_cast<uint2*>(orow)[c] = make_uint2(pack2(x[i][0] * inv * w0, x[i][1] * inv * w1),
                                                           pack2(x[i][2] * inv * w2, x[i][3] * inv * w3));
        }
    }
    if (tid == 0) epochs[row] = epoch;
}

// Publish form: write-through (sc1) payload stores, no release fence -- the fenced form (buffer_wbl2 of
// the whole XCD L2, full of the preceding GEMMs' slabs) measured slower inside the decode graph
// (profiles/r1_custom_ar_wt_ab.jsonl); the template keeps both forms for the record.
constexpr bool AR_WT = true;

static int launch_ar(ArHandle* h, int op, const void* in, void* out, size_t nbytes, hipStream_t s) {
    if (nbytes == 0) return 0;
    if (nbytes > h->max_bytes || nbytes > (size_t)MAX_BLOCKS * CH) return (int)hipErrorInvalidValue;
    for (int r = 0; r < h->world; ++r)
        if (!h->peers.base[r]) return (int)hipErrorInvalidValue;
    const int nblk = (int)((nbytes + CH - 1) / CH);
#define AR_ONE(OP_, WT_)                                                                                 \
    ar_oneshot_kernel<OP_, WT_><<<nblk, 256, 0, s>>>(h->peers, h->rank, h->world, h->max_bytes, (const char*)in, \
                                                     (char*)out, nbytes, h->epochs, h->error)
    if (op == OP_SUM_F32) AR_ONE(OP_SUM_F32, AR_WT);
    else AR_ONE(OP_MAX_U64, AR_WT);
#undef AR_ONE
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
    if (hipExtMallocWithFlags(&p, alloc_bytes(max_bytes, world), hipDeviceMallocUncached) != hipSuccess) {
        delete h;
        return nullptr;
    }
    h->mine = (char*)p;
    constexpr size_t n_ctr = MAX_BLOCKS + 16 + MAX_ROWS + MAX_GRAN;  // epochs | error (+pad) | push | granule epochs
    if (hipMemset(p, 0, HDR) != hipSuccess || hipMalloc((void**)&h->epochs, n_ctr * sizeof(unsigned))) {
        (void)hipFree(p);
        delete h;
        return nullptr;
    }
    (void)hipMemset(h->epochs, 0, n_ctr * sizeof(unsigned));
    h->error = h->epochs + MAX_BLOCKS;
    h->push_epochs = h->epochs + MAX_BLOCKS + 16;
    h->gran_epochs = h->push_epochs + MAX_ROWS;
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


// residual[T, D] += all-reduce(sum_s parts[s]) ; out = rmsnorm(residual) * w   (push-mode, see above)
// parts fp32 [S, T, D]; residual, w, out bf16; T <= 256, T * D * 2 <= max_bytes, D % 4 == 0, D <= 8192
MRSUM_API int mrsum_ar_add_rmsnorm(void* hv, const void* parts, int S, int T, void* residual, const void* w,
                                   void* out, int D, int out_stride, float eps, hipStream_t s) {
    auto h = (ArHandle*)hv;
    if (T <= 0) return 0;
    if (S < 1 || T > MAX_ROWS || D % 4 || D > 8192 || (size_t)T * D * 2 > h->max_bytes) return (int)hipErrorInvalidValue;
    for (int r = 0; r < h->world; ++r)
        if (!h->peers.base[r]) return (int)hipErrorInvalidValue;
    const int vpt = (D / 4 + 255) / 256;
    auto P = (const float*)parts; auto R = (bf16*)residual; auto W = (const bf16*)w; auto O = (bf16*)out;
#define AR_NORM_(V, WT_)                                                                                     \
    ar_add_rmsnorm_kernel<V, WT_><<<T, 256, 0, s>>>(h->peers, h->rank, h->world, h->max_bytes, P, S, T, R, W, O, D, \
                                                    out_stride, eps, h->push_epochs, h->error)
#define AR_NORM(V) AR_NORM_(V, AR_WT)
    if (vpt <= 1) AR_NORM(1);
    else if (vpt <= 2) AR_NORM(2);
    else if (vpt <= 4) AR_NORM(4);
    else AR_NORM(8);
#undef AR_NORM
#undef AR_NORM_
    return (int)hipGetLastError();
}

// Clear this rank's whole allocation (flags, one-shot / push-row / granule-push slots) and every local
// counter (epochs, the sticky error word, push-row and granule epochs).  COLLECTIVE at the host level
// (parallel/custom_ar.py CustomAllReduce.reset): every rank of the group must be idle (no kernel of this
// handle in flight anywhere) before, and must not launch one before every rank has returned -- then all
// ranks restart from epoch 1 against zeroed slots, so no stale tag or flag can match a new epoch.
MRSUM_API int mrsum_ar_reset(void* hv) {
    auto h = (ArHandle*)hv;
    if (!h) return (int)hipErrorInvalidValue;
    constexpr size_t n_ctr = MAX_BLOCKS + 16 + MAX_ROWS + MAX_GRAN;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemset(h->mine, 0, alloc_bytes(h->max_bytes, h->world));
    if (e == hipSuccess) e = hipMemset(h->epochs, 0, n_ctr * sizeof(unsigned));
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return (int)e;
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
