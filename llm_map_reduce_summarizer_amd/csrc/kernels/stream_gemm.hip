// Decode GEMM with an LDS-DMA weight ring: out[M, N] = x[M, K] . W[N, K]^T, M <= 64.
//
// Why a second decode GEMM: the register-streaming kernels (skinny_gemm.hip) keep 8-16 KiB of W
// in flight per workgroup and reach 4-5 TB/s; at M = 16-64 the x fragments they re-read and the
// per-k-block barrier of the LDS-x variant cap them near 3.5-4 TB/s.  A streaming CU needs
// ~80-130 KiB in flight to cover loaded HBM latency (MI355X_MICROARCH.md "ldsdma-fill": 8 x 16 KiB
// ring = 6.4-6.8 TB/s chip-wide), which register staging cannot hold next to the accumulators.
//
// Structure (one workgroup per CU, grid = N / (16 WPB) x splitK chosen by the host ~= #CUs):
//   * ring of D slots in ONE __shared__ array; slot = [16 WPB W rows | 16 MT x rows] x one
//     128-wide k block, each row block as two 1 KiB pieces of 8 rows x 128 B.  Every piece is ONE
//     global_load_lds_dwordx4 wave instruction (full 128-B lines, cdna_hip_programming.md §5 "x
//     operand ... through LDS in full 128-B lines"); lane l lands at piece + 16 l, so the bank
//     swizzle goes on the SOURCE address (rule 21): LDS chunk slot s of row r holds global chunk
//     s ^ (r & 7).
//   * every wave issues the same number of DMA instructions per slot (the x pieces are padded
//     with dummy pieces into a scratch KiB) so one counted `s_waitcnt vmcnt(NI * (D-2))` retires
//     exactly the slot about to be read; raw s_barrier (never __syncthreads, whose fence would
//     drain the ring); the slot consumed in iteration j-1 is refilled right after iteration j's
//     barrier (WAR ordered by that barrier).
//   * wave w owns W rows [16w, 16w + 16) of the tile: per k block 4 x v_mfma_f32_16x16x32_bf16
//     per x tile, A = W fragment (ds_read_b128), B = x fragment (ds_read_b128) -- the same
//     swapped out^T product and epilogues as skinny_gemm.hip (bf16 | fp32 split-K slab | SwiGLU
//     over [8 gate | 8 up] row blocks).
//
// Deferred RMSNorm (the decode layer's two add + RMSNorm passes folded into the GEMMs around them):
//   * producer (o / down projection, EPI_RESID_SPLIT): split-K partial tiles are published
//     write-through; the last split of a column tile to arrive sums them in split order onto the
//     residual rows (h = bf16(residual + sum), exactly the add_rmsnorm_parts arithmetic), stores h
//     back and writes the tile's per-row sums of squares of h to ssp[M][tiles];
//   * consumer (qkv / gate_up / LM head, any epilogue, e.ssq != null): x = the residual rows h and
//     the norm gain folded into W (W' = W diag(g), engine/model.py), so rmsnorm(h) W^T =
//     rsqrt(mean(h^2) + eps) * (h W'^T): the row scale multiplies the accumulator in the epilogue,
//     from the producer's per-tile sums reduced in a fixed order (deterministic).
// Two kernels per layer fewer than GEMM -> add_rmsnorm_parts -> GEMM.
//
// TP push (tensor-parallel decode, e.tp.world > 0): the producer's partial sum is this rank's share of a
// row-parallel projection.  Its last arriver all-reduces the column tile across the TP group before the
// residual update -- the custom all-reduce's push protocol (custom_ar.hip ar_add_rmsnorm_kernel) moved
// into the GEMM epilogue, per 16-column granule instead of per row:
//   1. bf16(tile partial sum) -> granule-push slot (epoch & 1, me) of EVERY rank over xGMI, as TAGGED
//      8-byte words: 2 bf16 | the epoch (system-scope single-copy-atomic stores, fire and forget)
//   2. poll my own slots until every rank's words carry this epoch -- the data is its own flag: no flag
//      store, no drain before it, no acquire (the NCCL "LL" idea; 2 B of tag per 2 B of payload, nothing
//      at M <= 16 rows)
//   3. h = bf16(residual + sum_p slot[p] in rank order) -- every rank adds the same bf16 values in the
//      same order, so the TP replicas of the residual stay bit-identical -- then the residual store and
//      the per-tile sums of squares exactly as the local producer.
// The epoch of a granule is a local counter advanced by the workgroup that owns the granule (every call
// covers all granules of the hidden dimension, so all counters agree, whatever the tiling).  Payload
// slot reuse two calls later is safe: a peer pushing call e+2 into parity e & 1 has passed call e+1's
// wait, which needs my words of call e+1, pushed after my call e (stream order) read the slot.  Spinning
// last arrivers hold at most one CU per column tile (< #CUs), so every rank completes all its tiles
// whatever its peers do: no cross-rank deadlock.  One launch per projection fewer than GEMM ->
// ar_add_rmsnorm, and the consumer takes the deferred norm as at TP = 1.
#include "ar_common.h"

namespace {
enum { EPI_BF16 = 0, EPI_F32_PARTIAL = 1, EPI_SWIGLU = 2, EPI_SWIGLU_SPLIT = 3, EPI_RESID_SPLIT = 4 };
constexpr int SS_PARTS = 8;  // consumer: the tiles' sums of squares of a row reduced as 8 fixed partials
constexpr int KBLK = 128;
// one KiB scratch for the dummy x pieces + 2 KiB for the consumer's row-norm partials [64][SS_PARTS]
constexpr int LDS_XTRA = 3 * 1024;
constexpr int LDS_BUDGET = 160 * 1024 - LDS_XTRA;

// deferred-RMSNorm operands (see the header); all null / zero for a plain GEMM
struct NormArgs {
    const float* ssq;  // consumer: [M][ssq_tiles] row sums of squares of x per producer column tile
    int ssq_tiles;     // multiple of 4 * SS_PARTS
    float inv_k, eps;  // 1 / hidden, RMSNorm epsilon
    bf16* resid;       // producer: residual rows [M][ldr] (in / out)
    int ldr;
    float* ssp;        // producer: [M][gridDim.x] row sums of squares of h per column tile
    int slab_m;        // F32_PARTIAL: rows per slab (0: M) -- row chunks of decode batches above 64 rows
    mrsum_ar::TPPush tp;  // RESID_SPLIT: all-reduce the tile over the TP group (tp.world == 0: off)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14; others at max = no wait
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// raw barrier with compiler fences: keeps LDS reads/DMA issues on their side without the vmcnt(0)
// that __syncthreads() would add
__device__ __forceinline__ void raw_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ int img_off(int row, int chunk) {
    return (((row >> 3) << 1) + (chunk >> 3)) * 1024 + ((row & 7) << 7) + ((((chunk & 7) ^ (row & 7))) << 4);
}

template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* g, char* lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds, 16, 0, AUX);
}

// consumer: s_ss[8 m + p] = sum of partial p (ssq_tiles / 8 consecutive tiles, fixed order) of row m
__device__ __forceinline__ void row_norm_partials(const NormArgs& e, int M, int tid, int nthr, float* s_ss) {
    const int C = e.ssq_tiles / SS_PARTS;
    for (int i = tid; i < SS_PARTS * M; i += nthr) {
        const int m = i / SS_PARTS, p = i % SS_PARTS;
        const float4* src = reinterpret_cast<const float4*>(e.ssq + (size_t)m * e.ssq_tiles + p * C);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int q = 0; q < C / 4; ++q) {
            const float4 v = src[q];
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
        s_ss[i] = (a.x + a.y) + (a.z + a.w);
    }
}

__device__ __forceinline__ float row_scale(const NormArgs& e, const float* s_ss, int m) {
    float t = 0.f;
#pragma unroll
    for (int p = 0; p < SS_PARTS; ++p) t += s_ss[SS_PARTS * m + p];
    return rsqrtf(t * e.inv_k + e.eps);
}

// split-K arrival: every wave drained its write-through partial stores; returns true in the last of
// the nsplit workgroups of column tile ``tile`` to arrive.  No acquire: the last arriver reads the
// partial tiles with L1-bypassing sc1 loads only (common.h ld_sc1_f4; the write-through publish +
// drained ticket form of cdna_hip_programming.md Guideline 16), ~1.7 us of buffer_inv wait saved per
// reduction.  The caller's last arriver re-arms the ticket when it is done (rearm), off the
// reduction's critical path -- the next launch's arrivals are ordered after it by the kernel boundary.
// The flag goes through the kernel's one LDS array (a second __shared__ object can de-pipeline the
// ring: cdna_hip_programming.md "Projection GEMM at M = 256" item 4(a)).
__device__ __forceinline__ bool last_arrival(int* counters, int tile, int nsplit, int tid, int* s_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {  // partials are write-through stores, drained above: no release fence (buffer_wbl2)
        const int prev = __hip_atomic_fetch_add(counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = prev == nsplit - 1;
    }
    __syncthreads();
    const bool last = *s_flag != 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: no load hoisted above the ticket
    return last;
}

__device__ __forceinline__ void rearm(int* counters, int tile, int tid) {
    if (tid == 0) __hip_atomic_store(counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

namespace {
// TP push of one column tile (header "TP push"): thread tid owns items it = tid + j NT < M * Q = (row mm,
// 4 columns at c).  h[j] holds this rank's fp32 partial sums on entry and the rank-ordered all-reduced
// bf16 sums plus the residual rv[j] on exit (rounded exactly as ar_add_rmsnorm_kernel).  Every item is
// pushed before the first is gathered.  ``epoch``: this launch's epoch of the tile's granules (read
// before the split-K ticket).
template <int IT, int Q, int NT, int GT>
__device__ __forceinline__ void tp_push_tile(const mrsum_ar::TPPush& tp, float (&h)[IT][4], const uint2 (&rv)[IT],
                                             const int M, const int n0, const int ncols, const int tid,
                                             const unsigned epoch) {
    using namespace mrsum_ar;
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int it = tid + j * NT;
        if (it < M * Q)
            tp_push_item(tp, tp_item_off(it / Q, ncols, n0 + 4 * (it % Q)), epoch,
                         make_float4(h[j][0], h[j][1], h[j][2], h[j][3]));
    }
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int it = tid + j * NT;
        if (it < M * Q) {
            const float4 acc = tp_gather_item(tp, tp_item_off(it / Q, ncols, n0 + 4 * (it % Q)), epoch);
            h[j][0] = __uint_as_float(rv[j].x << 16) + acc.x;
            h[j][1] = __uint_as_float(rv[j].x & 0xffff0000u) + acc.y;
            h[j][2] = __uint_as_float(rv[j].y << 16) + acc.z;
            h[j][3] = __uint_as_float(rv[j].y & 0xffff0000u) + acc.w;
        }
    }
    if (tid < GT) tp.epochs[n0 / GRAN + tid] = epoch;
}

// Epilogue shared by the bf16 and fp8 stream kernels.  acc[m]: lane holds out^T[n = n0 + 16w + 4g + jj]
// [m = 16 mt + r] (fp8: already times the weight row scales).  ``lds`` = the kernel's one LDS array
// (the ring is drained by now), ``s_ss`` its 2 KiB row-norm partials region.
template <int MT, int EPI, int WPB>
__device__ __forceinline__ void stream_epilogue(f32x4 (&acc)[MT], char* lds, float* s_ss, const int n0, const int M,
                                                void* __restrict__ out, const int ldo, float* __restrict__ parts,
                                                int* __restrict__ counters, const NormArgs& e) {
    // F32_PARTIAL slab s starts slab_m rows after slab s-1 (slab_m > M: a row chunk of a taller slab set)
    const int slab_m = e.slab_m > 0 ? e.slab_m : M;
    constexpr int R = 16 * WPB;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    // deferred RMSNorm consumer: scale row m of the product by rsqrt(mean(h_m^2) + eps) (the ring is
    // drained: the partial-sum loads cannot stall it)
    if (e.ssq) {
        row_norm_partials(e, M, tid, 64 * WPB, s_ss);
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const float sc = row_scale(e, s_ss, min(16 * m + r, M - 1));
            acc[m][0] *= sc; acc[m][1] *= sc; acc[m][2] *= sc; acc[m][3] *= sc;
        }
    }

    // C: lane holds out^T[n = n0 + 16w + 4g + jj][m = 16 mt + r]
    const int nw = n0 + 16 * w;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int mm = 16 * m + r;
        if constexpr (EPI == EPI_SWIGLU) {
            f32x4 up;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) up[jj] = __shfl_xor(acc[m][jj], 32, 64);
            if (g < 2 && mm < M) {
                float rr[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const float gv = acc[m][jj];
                    rr[jj] = gv / (1.f + __expf(-gv)) * up[jj];
                }
                uint2 o;
                o.x = pack2(rr[0], rr[1]);
                o.y = pack2(rr[2], rr[3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)mm * ldo + (nw >> 1) + 4 * g) = o;
            }
        } else if (mm < M) {
            if constexpr (EPI == EPI_BF16) {
                uint2 o;
                o.x = pack2(acc[m][0], acc[m][1]);
                o.y = pack2(acc[m][2], acc[m][3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)mm * ldo + nw + 4 * g) = o;
            } else if constexpr (EPI == EPI_F32_PARTIAL) {
                float* o = reinterpret_cast<float*>(out) + ((size_t)blockIdx.y * slab_m + mm) * ldo + nw + 4 * g;
                *reinterpret_cast<float4*>(o) = make_float4(acc[m][0], acc[m][1], acc[m][2], acc[m][3]);
            } else {  // write-through (global_store sc1): read by another XCD's last arriver, no release fence
                float* o = parts + ((size_t)blockIdx.y * M + mm) * (gridDim.x * R) + nw + 4 * g;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    __hip_atomic_store(o + jj, acc[m][jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if constexpr (EPI == EPI_SWIGLU_SPLIT || EPI == EPI_RESID_SPLIT) {
        // the last of the gridDim.y split workgroups of this column tile to arrive sums the fp32 partial
        // tiles (write-through publish / ticket / acquire, as attn_decode.hip combine_if_last<G, true>)
        // TP push: this launch's epoch of the tile's granules, loaded ahead of the ticket's drain
        const unsigned tp_epoch = EPI == EPI_RESID_SPLIT && e.tp.world > 0 ? e.tp.epochs[n0 / mrsum_ar::GRAN] + 1 : 0;
        if (!last_arrival(counters, blockIdx.x, gridDim.y, tid, reinterpret_cast<int*>(lds))) return;
        const int S = gridDim.y;
        const size_t ncols = (size_t)gridDim.x * R;
        const __amdgpu_buffer_rsrc_t rp = sc1_rsrc(parts);  // partial tiles: sc1 loads only (last_arrival)
        // every thread handles at most IT items and keeps all their partial-tile loads (4 splits at a time)
        // in flight together: the reduction is a few memory round trips, not one per item
        constexpr int NT = 64 * WPB;
        if constexpr (EPI == EPI_SWIGLU_SPLIT) {
            // silu(gate) * up.  Lets a narrow gate_up projection (TP shards: N = 3584) fill the chip with
            // split-K instead of streaming its weights through N / (16 WPB) CUs.
            // item = (row, 16-row block, half): 4 features = gate rows n0 + 16 bl + 4 hf .. +4, up rows + 8
            constexpr int IT = (64 * 2 * WPB + NT - 1) / NT;
            int pg[IT];  // element offset of the item in slab 0
            float4 gs[IT], us[IT];
#pragma unroll
            for (int j = 0; j < IT; ++j) {
                const int it = min(tid + j * NT, M * 2 * WPB - 1);
                const int mm = it / (2 * WPB), q = it % (2 * WPB), bl = q >> 1, hf = q & 1;
                pg[j] = mm * (int)ncols + n0 + 16 * bl + 4 * hf;
                gs[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                us[j] = gs[j];
            }
            const int slab = M * (int)ncols;
            for (int s0 = 0; s0 < S; s0 += 4) {
                float4 ga[IT][4], ua[IT][4];
#pragma unroll
                for (int j = 0; j < IT; ++j)
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int p = pg[j] + min(s0 + u, S - 1) * slab;
                        ga[j][u] = ld_sc1_f4(rp, 4 * p);
                        ua[j][u] = ld_sc1_f4(rp, 4 * (p + 8));
                    }
#pragma unroll
                for (int j = 0; j < IT; ++j)
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (s0 + u < S) {
                            gs[j].x += ga[j][u].x; gs[j].y += ga[j][u].y; gs[j].z += ga[j][u].z; gs[j].w += ga[j][u].w;
                            us[j].x += ua[j][u].x; us[j].y += ua[j][u].y; us[j].z += ua[j][u].z; us[j].w += ua[j][u].w;
                        }
            }
#pragma unroll
            for (int j = 0; j < IT; ++j) {
                const int it = tid + j * NT;
                if (it >= M * 2 * WPB) break;
                const int mm = it / (2 * WPB), q = it % (2 * WPB), bl = q >> 1, hf = q & 1;
                const float4 g4 = gs[j], u4 = us[j];
                uint2 o;
                o.x = pack2(g4.x / (1.f + __expf(-g4.x)) * u4.x, g4.y / (1.f + __expf(-g4.y)) * u4.y);
                o.y = pack2(g4.z / (1.f + __expf(-g4.z)) * u4.z, g4.w / (1.f + __expf(-g4.w)) * u4.w);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)mm * ldo + (n0 >> 1) + 8 * bl + 4 * hf) = o;
            }
            rearm(counters, blockIdx.x, tid);
        } else {
            // h = bf16(residual + partial 0 + partial 1 + ...) (add_rmsnorm_parts order), stored back; the
            // tile's per-row sum of h^2 (of the rounded values) to ssp[m][tile] in a fixed order.
            constexpr int Q = R / 4;  // 4-column items per row
            constexpr int IT = (64 * Q + NT - 1) / NT;
            float* s_sq = reinterpret_cast<float*>(lds + 64);  // [M][Q]; the ring is drained
            int pg[IT];  // element offset of the item in slab 0
            uint2* rsp[IT];
            uint2 rv[IT];
#pragma unroll
            for (int j = 0; j < IT; ++j) {
                const int it = min(tid + j * NT, M * Q - 1);
                const int mm = it / Q, c = n0 + 4 * (it % Q);
                pg[j] = mm * (int)ncols + c;
                rsp[j] = reinterpret_cast<uint2*>(e.resid + (size_t)mm * e.ldr + c);
                rv[j] = *rsp[j];  // residual: written by the previous kernels only (plain load)
            }
            const int slab = M * (int)ncols;
            const bool tp = e.tp.world > 0;  // TP push: the partials first, the residual after the all-reduce
            float h[IT][4];
#pragma unroll
            for (int j = 0; j < IT; ++j) {
                h[j][0] = tp ? 0.f : __uint_as_float(rv[j].x << 16);
                h[j][1] = tp ? 0.f : __uint_as_float(rv[j].x & 0xffff0000u);
                h[j][2] = tp ? 0.f : __uint_as_float(rv[j].y << 16);
                h[j][3] = tp ? 0.f : __uint_as_float(rv[j].y & 0xffff0000u);
            }
            for (int s0 = 0; s0 < S; s0 += 4) {
                float4 a4[IT][4];
#pragma unroll
                for (int j = 0; j < IT; ++j)
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        a4[j][u] = ld_sc1_f4(rp, 4 * (pg[j] + min(s0 + u, S - 1) * slab));
#pragma unroll
                for (int j = 0; j < IT; ++j)
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (s0 + u < S) {
                            h[j][0] += a4[j][u].x; h[j][1] += a4[j][u].y; h[j][2] += a4[j][u].z; h[j][3] += a4[j][u].w;
                        }
            }
            if (tp) tp_push_tile<IT, Q, NT, WPB>(e.tp, h, rv, M, n0, (int)ncols, tid, tp_epoch);
#pragma unroll
            for (int j = 0; j < IT; ++j) {
                const int it = tid + j * NT;
                if (it >= M * Q) break;
                const uint2 hv = make_uint2(pack2(h[j][0], h[j][1]), pack2(h[j][2], h[j][3]));
                *rsp[j] = hv;
                const float h0 = __uint_as_float(hv.x << 16), h1 = __uint_as_float(hv.x & 0xffff0000u);
                const float h2 = __uint_as_float(hv.y << 16), h3 = __uint_as_float(hv.y & 0xffff0000u);
                s_sq[it] = (h0 * h0 + h1 * h1) + (h2 * h2 + h3 * h3);
            }
            __syncthreads();
            for (int mm = tid; mm < M; mm += 64 * WPB) {
                float t = 0.f;
                for (int q = 0; q < Q; ++q) t += s_sq[mm * Q + q];
                e.ssp[(size_t)mm * gridDim.x + blockIdx.x] = t;
            }
            rearm(counters, blockIdx.x, tid);
        }
    }
}
}  // namespace

// NTW: weight pieces loaded with the nontemporal policy (aux = 2): decode weights are read once per
// step by one CU (MI355X_MICROARCH.md "nt-weights"); the x pieces keep the default policy (re-read by
// every column tile from L2).
template <int MT, int EPI, int WPB, bool NTW>
__global__ __launch_bounds__(64 * WPB, 1) void stream_gemm_kernel(const bf16* __restrict__ x, int ldx,
                                                                  const bf16* __restrict__ W, int K, int M,
                                                                  void* __restrict__ out, int ldo, int kper,
                                                                  float* __restrict__ parts, int* __restrict__ counters,
                                                                  const NormArgs e) {
    constexpr int R = 16 * WPB, BM = 16 * MT;
    constexpr int WBYTES = R * 256, SLOT = WBYTES + BM * 256;
    constexpr int D = (LDS_BUDGET / SLOT) < 6 ? (LDS_BUDGET / SLOT) : 6;
    static_assert(D >= 2, "ring too shallow");
    constexpr int XP = 2 * BM / 8;               // x pieces per slot (= 4 MT)
    constexpr int XI = (XP + WPB - 1) / WPB;     // x pieces per wave (padded)
    constexpr int NI = 4 + XI;                   // DMA instructions per wave per slot (W: R/4 pieces / WPB = 4)
    __shared__ __attribute__((aligned(1024))) char lds[D * SLOT + LDS_XTRA];
    float* const s_ss = reinterpret_cast<float*>(lds + D * SLOT + 1024);  // consumer row-norm partials

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * R;
    const int ks = blockIdx.y * kper;
    const int nkb = kper / KBLK;

    // per-lane source rows/chunks of this wave's pieces (fixed over k)
    const int prow = lane >> 3, pslot = lane & 7;
    // W pieces q = 4w + p (p < 4): rows 8 (q >> 1) + prow, k half q & 1
    const bf16* wsrc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int q = 4 * w + p;
        const int row = 8 * (q >> 1) + prow;
        wsrc[p] = W + (size_t)(n0 + row) * K + ks + 8 * (8 * (q & 1) + (pslot ^ prow));
    }
    const bf16* xsrc[XI];
    int xdst[XI];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int q = w + WPB * i;  // x piece index; >= XP -> dummy
        const int qq = q < XP ? q : 0;
        const int row = 8 * (qq >> 1) + prow;
        xsrc[i] = x + (size_t)min(row, M - 1) * ldx + ks + 8 * (8 * (qq & 1) + (pslot ^ prow));
        xdst[i] = q < XP ? WBYTES + q * 1024 : -1;
    }
#define ISSUE(slot, kb)                                                                              \
    {                                                                                                \
        char* base = lds + (slot) * SLOT;                                                            \
        _Pragma("unroll") for (int p = 0; p < 4; ++p) glds16<NTW ? 2 : 0>(wsrc[p] + (kb), base + (4 * w + p) * 1024); \
        _Pragma("unroll") for (int i = 0; i < XI; ++i)                                               \
            glds16(xsrc[i] + (kb), xdst[i] >= 0 ? base + xdst[i] : lds + D * SLOT);                  \
    }

    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: D-1 slots in flight (clamped k blocks past the end are never read)
#pragma unroll
    for (int s = 0; s < D - 1; ++s) ISSUE(s, min(s, nkb - 1) * KBLK);

    const int r = lane & 15, g = lane >> 4;
    for (int j = 0; j < nkb; ++j) {
        if (j + D - 2 < nkb) wait_vmcnt<NI * (D - 2)>();  // slots j+1 .. j+D-2 stay in flight
        else wait_vmcnt<0>();
        raw_barrier();
        if (j + D - 1 < nkb) ISSUE((j + D - 1) % D, (j + D - 1) * KBLK);
        const char* wl = lds + (j % D) * SLOT;
        const char* xl = wl + WBYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4 av = *reinterpret_cast<const u32x4*>(wl + img_off(16 * w + r, 4 * i + g));
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                const u32x4 bv = *reinterpret_cast<const u32x4*>(xl + img_off(16 * m + r, 4 * i + g));
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                                 __builtin_bit_cast(bf16x8, bv), acc[m], 0, 0, 0);
            }
        }
    }
#undef ISSUE

    stream_epilogue<MT, EPI, WPB>(acc, lds, s_ss, n0, M, out, ldo, parts, counters, e);
}

// ar (RESID_SPLIT only, may be null): a custom all-reduce handle (custom_ar.hip) whose group the residual
// update all-reduces over (header "TP push"); every peer mapped, M * N * 2 <= its slot bytes.
static bool tp_push_ok(const void* ar, int epi, int M, int N) {
    using namespace mrsum_ar;
    if (!ar) return true;
    auto h = (const ArHandle*)ar;
    if (epi != EPI_RESID_SPLIT || N % GRAN || N / GRAN > MAX_GRAN || (size_t)M * N * 4 > h->max_bytes)
        return false;
    for (int r = 0; r < h->world; ++r)
        if (!h->peers.base[r]) return false;
    return true;
}

// out: bf16 [M, ldo] (EPI_BF16), fp32 slabs [splits, slab_m (0: M), ldo] (EPI_F32_PARTIAL), bf16 [M, ldo] of N/2
// SwiGLU features (EPI_SWIGLU, splits = 1; EPI_SWIGLU_SPLIT with ``parts`` fp32 [splits, M, N] scratch),
// or the residual update of EPI_RESID_SPLIT (``out`` unused; resid [M, ldr] bf16 += the product, ssp
// fp32 [M, N / (16 wpb)] row sums of squares per column tile; ``parts`` scratch as SwiGLU_SPLIT).
// Split-K last-arriver epilogues take ``counters`` >= N / (16 wpb) ints, zero on the first call (every
// launch leaves them zero again).  ssq (any epilogue): deferred-RMSNorm input, [M, ssq_tiles] fp32 row
// sums of squares of x (x = the un-normalised residual rows), ssq_tiles % 32 == 0; the product rows are
// scaled by rsqrt(sum / K + eps).  N % (16 wpb) == 0, wpb in {4, 5, 6, 7, 8}, M <= 64 -- or 64 < M <= 128
// (decode batches of 65-128 sequences: 96- / 128-row x tiles, one pass over the weights instead of one per
// 64-row chunk) for the bf16 / fp32-slab / SwiGLU epilogues without a deferred norm.
// Decode weights are streamed with nontemporal loads (each weight row read once per step by one CU:
// MI355X_MICROARCH.md "nt-weights"; profiles/r1_decode_nt_ab.jsonl).
MRSUM_API int mrsum_stream_gemm(const void* x, int ldx, const void* W, int N, int K, int M, void* out, int ldo,
                                int epi, int splits, int wpb, void* parts, int* counters, const float* ssq,
                                int ssq_tiles, float eps, void* resid, int ldr, float* ssp, int slab_m, void* ar,
                                hipStream_t s) {
    if (M <= 0) return 0;
    if (wpb < 4 || wpb > 8 || M > 128 || K % KBLK || N % (16 * wpb) || splits < 1 || (K / KBLK) % splits ||
        epi < EPI_BF16 || epi > EPI_RESID_SPLIT)
        return (int)hipErrorInvalidValue;
    if (M > 64 && (ssq || (epi != EPI_BF16 && epi != EPI_F32_PARTIAL && epi != EPI_SWIGLU)))
        return (int)hipErrorInvalidValue;  // tall tiles: no deferred norm, no split-K last-arriver epilogue
    if (M > 64) {
        // tall tiles only at widths whose slot (16 wpb W rows + 16 MT x rows, 256 B each) leaves a ring of at
        // least 3 slots (one being filled, two published); ops/hip.py _TALL_WPB lists the same widths
        const int slot = (16 * wpb + 16 * (M > 96 ? 8 : 6)) * 256;
        if (LDS_BUDGET / slot < 3) return (int)hipErrorInvalidValue;
    }
    const bool split_epi = epi == EPI_SWIGLU_SPLIT || epi == EPI_RESID_SPLIT;
    if (epi != EPI_F32_PARTIAL && !split_epi && splits != 1) return (int)hipErrorInvalidValue;
    if (split_epi && (!parts || !counters)) return (int)hipErrorInvalidValue;
    if (epi == EPI_RESID_SPLIT && (!resid || !ssp || ldr % 4)) return (int)hipErrorInvalidValue;
    if (ssq && (ssq_tiles <= 0 || ssq_tiles % (4 * SS_PARTS))) return (int)hipErrorInvalidValue;
    if (slab_m && (slab_m < M || epi != EPI_F32_PARTIAL)) return (int)hipErrorInvalidValue;
    if (!tp_push_ok(ar, epi, M, N)) return (int)hipErrorInvalidValue;
    NormArgs e;
    e.ssq = ssq; e.ssq_tiles = ssq_tiles; e.inv_k = 1.f / (float)K; e.eps = eps;
    e.resid = (bf16*)resid; e.ldr = ldr; e.ssp = ssp; e.slab_m = slab_m;
    e.tp = mrsum_ar::tp_push_of((const mrsum_ar::ArHandle*)ar);
    const int kper = K / splits;
    const int mt = (M + 15) / 16;
    dim3 grid(N / (16 * wpb), splits), block(64 * wpb);
    auto X = (const bf16*)x;
    auto Wp = (const bf16*)W;
    auto P = (float*)parts;
#define L(MT_, EPI_, WPB_)                                                                                   \
    stream_gemm_kernel<MT_, EPI_, WPB_, true><<<grid, block, 0, s>>>(X, ldx, Wp, K, M, out, ldo, kper, P, counters, e)
#define BY_WPB(MT_, EPI_)                          \
    switch (wpb) {                                 \
        case 4: L(MT_, EPI_, 4); break;            \
        case 5: L(MT_, EPI_, 5); break;            \
        case 6: L(MT_, EPI_, 6); break;            \
        case 7: L(MT_, EPI_, 7); break;            \
        default: L(MT_, EPI_, 8); break;           \
    }
#define BY_EPI(MT_)                                                           \
    if (epi == EPI_BF16) { BY_WPB(MT_, EPI_BF16) }                            \
    else if (epi == EPI_F32_PARTIAL) { BY_WPB(MT_, EPI_F32_PARTIAL) }         \
    else if (epi == EPI_SWIGLU) { BY_WPB(MT_, EPI_SWIGLU) }                   \
    else if (epi == EPI_SWIGLU_SPLIT) { BY_WPB(MT_, EPI_SWIGLU_SPLIT) }       \
    else { BY_WPB(MT_, EPI_RESID_SPLIT) }
#define BY_EPI_TALL(MT_)                                                      \
    if (epi == EPI_BF16) { BY_WPB(MT_, EPI_BF16) }                            \
    else if (epi == EPI_F32_PARTIAL) { BY_WPB(MT_, EPI_F32_PARTIAL) }         \
    else { BY_WPB(MT_, EPI_SWIGLU) }
    switch (mt) {
        case 1: BY_EPI(1); break;
        case 2: BY_EPI(2); break;
        case 3: BY_EPI(3); break;
        case 4: BY_EPI(4); break;
        case 5: case 6: BY_EPI_TALL(6); break;
        default: BY_EPI_TALL(8); break;
    }
#undef BY_EPI_TALL
#undef BY_EPI
#undef BY_WPB
#undef L
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// W8A16 (OCP e4m3fn weights, per-row fp32 scales) variant for the fp8 Llama-3-70B decode.  The ring is
// bound by its slot rate (~1 us per slot at full chip load, profiles/r1_fp8_stream_gemm_experiment.txt:
// a 128-wide fp8 slot carried half the bf16 bytes and halved the bandwidth), so an fp8 slot spans 256
// k: the SAME 256 B per weight row as a bf16 slot (same pieces, same swizzle), twice the x bytes (two
// bf16 images of 128 k).  A fragments: 8 fp8 per lane per 32-k MFMA step (ds_read_b64), converted
// exactly by v_cvt_scalef32_pk_bf16_fp8; the row scale multiplies the fp32 accumulator in the epilogue
// (before SwiGLU for gate / up rows).
namespace {
constexpr int KB8 = 256;

__device__ __forceinline__ bf16x8 fp8x8_bf16(uint2 d) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d.x, 1.0f, false);
    const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d.x, 1.0f, true);
    const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d.y, 1.0f, false);
    const bf16x2 e = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d.y, 1.0f, true);
    return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], e[0], e[1]};
}
}  // namespace

// XR (one x row, kper <= XR_MAX_K): the workgroup's whole x slice is DMA'd into LDS once, ahead of the
// ring, and the ring carries weight pieces only -- at M = 1 the padded 16-row x images were a third of
// every slot (15 copies of the clamped row), which left fewer weight bytes in flight per CU.
constexpr int XR_MAX_K = 8192;

template <int MT, int EPI, int WPB, bool XR>
__global__ __launch_bounds__(64 * WPB, 1) void stream_fp8_kernel(const bf16* __restrict__ x, int ldx,
                                                                 const unsigned char* __restrict__ W,
                                                                 const float* __restrict__ wscale, int K, int M,
                                                                 void* __restrict__ out, int ldo, int kper,
                                                                 float* __restrict__ parts, int* __restrict__ counters,
                                                                 const NormArgs e) {
    constexpr int R = 16 * WPB, BM = 16 * MT;
    constexpr int WBYTES = R * 256, XBYTES = BM * 256, SLOT = XR ? WBYTES : WBYTES + 2 * XBYTES;
    constexpr int XRES = XR ? XR_MAX_K * 2 : 0;  // resident x row image (bf16)
    constexpr int DCAP = XR ? 8 : 6;
    constexpr int D = ((LDS_BUDGET - XRES) / SLOT) < DCAP ? ((LDS_BUDGET - XRES) / SLOT) : DCAP;
    static_assert(D >= 2, "ring too shallow");
    static_assert(!XR || MT == 1, "resident x: one row");
    constexpr int XP = XR ? 0 : 2 * (2 * BM / 8);  // x pieces per slot: two 128-k images
    constexpr int XI = (XP + WPB - 1) / WPB;
    constexpr int NI = 4 + XI;
    __shared__ __attribute__((aligned(1024))) char lds[D * SLOT + XRES + LDS_XTRA];
    char* const xres = lds + D * SLOT;      // XR: x[0][ks .. ks + kper) as bf16
    char* const xtra = lds + D * SLOT + XRES;  // dummy x pieces | row-norm partials

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int n0 = blockIdx.x * R;
    const int ks = blockIdx.y * kper;
    const int nkb = kper / KB8;
    const int prow = lane >> 3, pslot = lane & 7;
    const unsigned char* wsrc[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int q = 4 * w + p;
        const int row = 8 * (q >> 1) + prow;
        wsrc[p] = W + (size_t)(n0 + row) * K + ks + 16 * (8 * (q & 1) + (pslot ^ prow));
    }
    // x piece q: image q / (2 BM / 8) (k half of the 256-wide block), then the bf16 piece layout
    constexpr int XPI = 2 * BM / 8;  // pieces per image
    const bf16* xsrc[XI > 0 ? XI : 1];
    int xdst[XI > 0 ? XI : 1];
#pragma unroll
    for (int i = 0; i < XI; ++i) {
        const int q = w + WPB * i;
        const int qq = q < XP ? q : 0;
        const int img = qq / XPI, qi = qq % XPI;
        const int row = 8 * (qi >> 1) + prow;
        xsrc[i] = x + (size_t)min(row, M - 1) * ldx + ks + 128 * img + 8 * (8 * (qi & 1) + (pslot ^ prow));
        xdst[i] = q < XP ? WBYTES + img * XBYTES + qi * 1024 : -1;
    }
#define ISSUE8(slot, kb)                                                                             \
    {                                                                                                \
        char* base = lds + (slot) * SLOT;                                                            \
        _Pragma("unroll") for (int p = 0; p < 4; ++p) glds16<2>(wsrc[p] + (kb), base + (4 * w + p) * 1024); \
        _Pragma("unroll") for (int i = 0; i < XI; ++i)                                               \
            glds16(xsrc[i] + (kb), xdst[i] >= 0 ? base + xdst[i] : xtra);                            \
    }
    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (XR) {
        // the x slice as contiguous 1 KiB pieces (512 bf16), issued before the ring prologue: the first
        // counted ring wait (every op older than the newest D-2 slots) covers them
        for (int p = w; p < kper / 512; p += WPB) glds16(x + ks + 512 * p + 8 * lane, xres + 1024 * p);
    }
#pragma unroll
    for (int s = 0; s < D - 1; ++s) ISSUE8(s, min(s, nkb - 1) * KB8);

    const int r = lane & 15, g = lane >> 4;
    for (int j = 0; j < nkb; ++j) {
        if (j + D - 2 < nkb) wait_vmcnt<NI * (D - 2)>();
        else wait_vmcnt<0>();
        raw_barrier();
        if (j + D - 1 < nkb) ISSUE8((j + D - 1) % D, (j + D - 1) * KB8);
        const char* wl = lds + (j % D) * SLOT;
        const char* xl = wl + WBYTES;
        // MFMA steps in pairs (2p, 2p+1): lane (r, g) reads the 16-B chunk 4p + g of its weight row (fp8 k =
        // 64p + 16g .. +16) with one ds_read_b128 and feeds its low 8 bytes to step 2p and its high 8 bytes
        // to step 2p+1; the x operand takes the same k permutation (the MFMA k order is free).  8-byte A
        // reads were merged by hipcc into ds_read2st64_b64, whose lost alias info made the waitcnt pass drain
        // vmcnt(0) -- every in-flight ring slot -- before each slot's first read (XR variant).  Same-box A/B:
        // neutral to +7 % (profiles/r3_fp8_stream_vmcnt_fix_ab.jsonl; 6.2 TB/s on the 70B down shape on
        // that box, 4.8 on another: compare only same-box numbers).
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const u32x4 a4 = *reinterpret_cast<const u32x4*>(wl + img_off(16 * w + r, 4 * p + g));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const bf16x8 av = fp8x8_bf16(make_uint2(a4[2 * h], a4[2 * h + 1]));
                if constexpr (XR) {  // every lane reads row 0 (broadcast); rows >= M are never stored
                    const u32x4 bv = *reinterpret_cast<const u32x4*>(xres + 2 * (KB8 * j + 64 * p + 16 * g + 8 * h));
                    acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, bv), acc[0], 0, 0, 0);
                } else {
#pragma unroll
                    for (int m = 0; m < MT; ++m) {
                        const u32x4 bv = *reinterpret_cast<const u32x4*>(xl + (p >> 1) * XBYTES +
                                                                         img_off(16 * m + r, 8 * (p & 1) + 2 * g + h));
                        acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, bv), acc[m], 0, 0, 0);
                    }
                }
            }
        }
    }
#undef ISSUE8

    // weight row scales first (n = n0 + 16w + 4g + jj), then the shared epilogue
    const float4 sc = *reinterpret_cast<const float4*>(wscale + n0 + 16 * w + 4 * g);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        acc[m][0] *= sc.x; acc[m][1] *= sc.y; acc[m][2] *= sc.z; acc[m][3] *= sc.w;
    }
    stream_epilogue<MT, EPI, WPB>(acc, lds, reinterpret_cast<float*>(xtra + 1024), n0, M, out, ldo, parts, counters, e);
}

// Same contract as mrsum_stream_gemm (epilogues BF16 / F32_PARTIAL / SWIGLU / SWIGLU_SPLIT / RESID_SPLIT, deferred
// RMSNorm operands) with W e4m3fn [N, K] row-major and wscale fp32 [N]; K % 256 == 0, (K / 256) % splits == 0.
MRSUM_API int mrsum_stream_fp8(const void* x, int ldx, const void* W, const float* wscale, int N, int K, int M,
                               void* out, int ldo, int epi, int splits, int wpb, void* parts, int* counters,
                               const float* ssq, int ssq_tiles, float eps, void* resid, int ldr, float* ssp,
                               void* ar, hipStream_t s) {
    if (M <= 0) return 0;
    if (wpb < 4 || wpb > 8 || M > 64 || K % KB8 || N % (16 * wpb) || splits < 1 || (K / KB8) % splits ||
        epi < EPI_BF16 || epi > EPI_RESID_SPLIT)
        return (int)hipErrorInvalidValue;
    const bool split_epi = epi == EPI_SWIGLU_SPLIT || epi == EPI_RESID_SPLIT;
    if (epi != EPI_F32_PARTIAL && !split_epi && splits != 1) return (int)hipErrorInvalidValue;
    if (split_epi && (!parts || !counters)) return (int)hipErrorInvalidValue;
    if (epi == EPI_RESID_SPLIT && (!resid || !ssp || ldr % 4)) return (int)hipErrorInvalidValue;
    if (ssq && (ssq_tiles <= 0 || ssq_tiles % (4 * SS_PARTS))) return (int)hipErrorInvalidValue;
    if (!tp_push_ok(ar, epi, M, N)) return (int)hipErrorInvalidValue;
    NormArgs e;
    e.ssq = ssq; e.ssq_tiles = ssq_tiles; e.inv_k = 1.f / (float)K; e.eps = eps;
    e.resid = (bf16*)resid; e.ldr = ldr; e.ssp = ssp; e.slab_m = 0;
    e.tp = mrsum_ar::tp_push_of((const mrsum_ar::ArHandle*)ar);
    const int kper = K / splits;
    const int mt = (M + 15) / 16;
    dim3 grid(N / (16 * wpb), splits), block(64 * wpb);
    auto X = (const bf16*)x;
    auto Wp = (const unsigned char*)W;
    auto P = (float*)parts;
    // one row: x resident in LDS (weight-only ring)
    const bool xr = M == 1 && kper <= XR_MAX_K && kper % 512 == 0;
#define L8(MT_, EPI_, WPB_)                                                                                      \
    do {                                                                                                         \
        if (MT_ == 1 && xr)                                                                                      \
            stream_fp8_kernel<1, EPI_, WPB_, true><<<grid, block, 0, s>>>(X, ldx, Wp, wscale, K, M, out, ldo, kper, P, \
                                                                          counters, e);                          \
        else                                                                                                     \
            stream_fp8_kernel<MT_, EPI_, WPB_, false><<<grid, block, 0, s>>>(X, ldx, Wp, wscale, K, M, out, ldo,  \
                                                                             kper, P, counters, e);              \
    } while (0)
#define BY_WPB8(MT_, EPI_)                          \
    switch (wpb) {                                  \
        case 4: L8(MT_, EPI_, 4); break;            \
        case 5: L8(MT_, EPI_, 5); break;            \
        case 6: L8(MT_, EPI_, 6); break;            \
        case 7: L8(MT_, EPI_, 7); break;            \
        default: L8(MT_, EPI_, 8); break;           \
    }
#define BY_EPI8(MT_)                                                      \
    if (epi == EPI_BF16) { BY_WPB8(MT_, EPI_BF16) }                       \
    else if (epi == EPI_F32_PARTIAL) { BY_WPB8(MT_, EPI_F32_PARTIAL) }    \
    else if (epi == EPI_SWIGLU) { BY_WPB8(MT_, EPI_SWIGLU) }              \
    else if (epi == EPI_SWIGLU_SPLIT) { BY_WPB8(MT_, EPI_SWIGLU_SPLIT) }  \
    else { BY_WPB8(MT_, EPI_RESID_SPLIT) }
    switch (mt) {
        case 1: BY_EPI8(1); break;
        case 2: BY_EPI8(2); break;
        case 3: BY_EPI8(3); break;
        default: BY_EPI8(4); break;
    }
#undef BY_EPI8
#undef BY_WPB8
#undef L8
    return (int)hipGetLastError();
}
