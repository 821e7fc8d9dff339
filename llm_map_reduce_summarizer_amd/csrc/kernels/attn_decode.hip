// Paged GQA decode attention, split-K over the context.
//
// One query token per sequence.  Work item = (split s, kv head, sequence b):
// a 256-thread workgroup streams keys [ks, ke) of ONE kv head from the paged
// cache and serves all G = Hq/Hkv query heads that share it, so every K/V
// byte is read from HBM exactly once per step (the op is HBM bound: at B=44,
// 4.5k context, Llama-3-8B reads ~26 GB of KV per step).
//
// The workgroup stages 64-key pages of K and V through LDS and scores them on
// MFMA (attn_decode_mfma_kernel below); its 4 waves merge their online-softmax
// states through LDS at the end.  Scores are in the log2 domain (scale folded
// with log2(e)) so the exponentials are exp2.
//
// Output: unnormalised partials part_o [B, Hq, S, D] f32 and part_ml
// [B, Hq, S, 2] = (running max, running sum), merged into out [B, Hq*D] bf16
// IN THE SAME LAUNCH by the last of the S split workgroups of a (b, kv head)
// to finish: every split publishes its slab (vmcnt drain, barrier, one
// agent-scope release) and draws a ticket from a per-(b, kv head) counter;
// the ticket S-1 holder acquires (agent scope) and combines, then re-arms the
// counter to 0 for the next launch / graph replay (cdna_hip_programming.md
// §5 "in-launch split-K reduction", placement-independent across XCDs).
// With no counter buffer a separate combine kernel is launched instead.
// Context length = positions[b] + 1 is read on the device, so the launch
// shape is fixed and the kernel can live inside a captured decode graph.
#include "kv8.h"

// splits of one (sequence, kv head): up to 256 so a TP shard's single kv head at long contexts still fills the
// chip (70B fp8 TP=8 shard at 32k: 64 splits = 64 workgroups left its 16.8 MB of K/V at ~1.1 TB/s)
constexpr int MAX_SPLITS = 256;

// Diagnostic build only (tools/exp_attn_stamps.py compiles this file with -DMRSUM_ATTN_STAMPS into
// _native/diag/): every wave accumulates s_memtime deltas per phase of the split kernel -- prologue, tile
// compute, the barrier after it, the next tile's LDS write + load issue, the barrier after that, epilogue --
// and lane 0 stores them to g_attn_stamps[(workgroup * 4 + wave) * 8 + phase] (6: total, 7: tiles).
#ifdef MRSUM_ATTN_STAMPS
__device__ unsigned long long* g_attn_stamps;
MRSUM_API int mrsum_attn_set_stamps(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), &p, sizeof(p));
}
#define ST_DECL                                                        \
    unsigned long long st_last_ = __builtin_amdgcn_s_memtime(), st_t0_ = st_last_; \
    unsigned long long st_acc_[6] = {0, 0, 0, 0, 0, 0};
#define ST(i)                                                          \
    {                                                                  \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();   \
        st_acc_[i] += n_ - st_last_;                                   \
        st_last_ = n_;                                                 \
    }
#define ST_STORE(NT_)                                                                                   \
    if (g_attn_stamps && (threadIdx.x & 63) == 0) {                                                      \
        const size_t wg_ = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;      \
        unsigned long long* o_ = g_attn_stamps + (wg_ * 4 + (threadIdx.x >> 6)) * 8;                   \
        for (int i_ = 0; i_ < 6; ++i_) o_[i_] = st_acc_[i_];                                            \
        o_[6] = __builtin_amdgcn_s_memtime() - st_t0_;                                                  \
        o_[7] = (unsigned long long)(NT_);                                                              \
    }
#else
#define ST_DECL
#define ST(i)
#define ST_STORE(NT_)
#endif

// partial-result store: agent-scope atomic (global_store sc1, write-through) when a last-arriving
// workgroup of another XCD will read it in the same launch (combine_if_last<G, true>), else plain
__device__ __forceinline__ void st_part(float* p, float v, bool wt) {
    if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// Merge the S split partials of one (b, kv head) group -- G query heads x D -- with all 256
// threads: the (max, sum) pairs are read in parallel into LDS and turned into per-split weights
// once, then each output element sums S slabs with independent (unrolled) loads, so the merge
// costs ~S/8 memory round trips instead of S dependent ones.
// SC1: the partials were published write-through in THIS launch and are read with L1-bypassing sc1
// loads (common.h ld_sc1_*) instead of behind an agent-scope acquire.
template <int G, bool SC1 = false>
__device__ __forceinline__ void combine_group(const float* part_o, const float* part_ml, bf16* out, int out_stride,
                                              int b, int kvh, int Hq, int S, float* sw /* [G][S] LDS */,
                                              float* sden /* [G] */) {
    constexpr int D = 128;
    constexpr int NV = G * D / 4;                 // float4 output items
    constexpr int NH = NV >= 256 ? 1 : 256 / NV;  // interleaved split subsets per item
    constexpr int NR = NV > 256 ? NV / 256 : 1;   // item rounds (G = 16: 2)
    constexpr int PRE = 16 / NR;                  // partial loads per thread issued up front
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const size_t bh0 = (size_t)b * Hq + (size_t)kvh * G;
    // this group's partials: part_o [G][S][D] and part_ml [G][S][2] from one wave-uniform base each
    const float* po0 = part_o + bh0 * S * D;
    const float* pm0 = part_ml + bh0 * S * 2;
    const __amdgpu_buffer_rsrc_t ro = sc1_rsrc(po0), rm = sc1_rsrc(pm0);  // (used by SC1 only)
    auto ld_o = [&](int g, int sp, int d4) -> float4 {  // slab sp, float4 column d4 of head g
        const int idx = (g * S + sp) * (D / 4) + d4;
        if constexpr (SC1) return ld_sc1_f4(ro, idx * 16);
        else return reinterpret_cast<const float4*>(po0)[idx];
    };
    // 1. the first PRE partial slabs of every (item, subset) are loaded BEFORE the split weights are
    //    known, so the slab loads and the (max, sum) loads share one memory round trip
    float4 pre[NR][PRE];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int t = r * 256 + tid, item = t % NV, h = t / NV;
        const int g = item / (D / 4), d4 = item % (D / 4);
#pragma unroll
        for (int j = 0; j < PRE; ++j) {
            const int sp = h + j * NH;
            // unconditional load (clamped index; unused values weighted 0 below): no branch around it
            const float4 v = ld_o(g, min(sp, S - 1), d4);
            pre[r][j] = (h < NH && sp < S) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    // 2. split weights: one wave per head, lane l holds splits l, l + 64, l + 128, l + 192 (S <= MAX_SPLITS)
    static_assert(MAX_SPLITS <= 4 * 64, "four splits per lane");
    for (int g = wv; g < G; g += 4) {
        float ms[4], ls[4], mloc = -INFINITY;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int sp = lane + 64 * q;
            const int sl = min(sp, S - 1);
            float2 v;
            if constexpr (SC1) v = ld_sc1_f2(rm, (g * S + sl) * 8);
            else v = reinterpret_cast<const float2*>(pm0)[g * S + sl];
            ms[q] = sp < S ? v.x : -INFINITY;
            ls[q] = sp < S ? v.y : 0.f;
            mloc = fmaxf(mloc, ms[q]);
        }
        const float M = wave_max(mloc);
        float wl = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int sp = lane + 64 * q;
            const float w = ms[q] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ms[q] - M);
            wl += w * ls[q];
            if (sp < S) sw[g * S + sp] = w;
        }
        const float den = wave_sum(wl);
        if (lane == 0) sden[g] = den;
    }
    __syncthreads();
    // 3. weighted sums (the rare splits beyond the preloaded ones loaded now), subsets merged through LDS
    __shared__ float4 red[NH > 1 ? 256 : 1];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int t = r * 256 + tid, item = t % NV, h = t / NV;
        const int g = item / (D / 4), d4 = item % (D / 4);
        const float* w = sw + g * S;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if (h < NH) {
#pragma unroll
            for (int j = 0; j < PRE; ++j) {
                const int sp = h + j * NH;
                const float ws = sp < S ? w[sp] : 0.f;
                acc.x += ws * pre[r][j].x;
                acc.y += ws * pre[r][j].y;
                acc.z += ws * pre[r][j].z;
                acc.w += ws * pre[r][j].w;
            }
            // splits beyond the preloaded ones (S > PRE * NH: the one-row TP-shard plans of 128-256 splits)
            // in batches of 8 independent loads (clamped, weighted 0 past S): a few round trips, not one per
            // split; the same summation order as one at a time
            for (int sp0 = h + PRE * NH; sp0 < S; sp0 += 8 * NH) {
                float4 v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = ld_o(g, min(sp0 + j * NH, S - 1), d4);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int sp = sp0 + j * NH;
                    if (sp < S) {
                        const float ws = w[sp];
                        acc.x += ws * v[j].x;
                        acc.y += ws * v[j].y;
                        acc.z += ws * v[j].z;
                        acc.w += ws * v[j].w;
                    }
                }
            }
        }
        if constexpr (NH > 1) {
            red[tid] = acc;
            __syncthreads();
            if (h == 0) {
#pragma unroll
                for (int j = 1; j < NH; ++j) {
                    const float4 v = red[j * NV + item];
                    acc.x += v.x;
                    acc.y += v.y;
                    acc.z += v.z;
                    acc.w += v.w;
                }
            }
        }
        if (h == 0) {
            const float den = sden[g];
            const float inv = den > 0.f ? 1.f / den : 0.f;
            uint2 o;
            o.x = pack2(acc.x * inv, acc.y * inv);
            o.y = pack2(acc.z * inv, acc.w * inv);
            *reinterpret_cast<uint2*>(out + (size_t)b * out_stride + (kvh * G + g) * D + 4 * d4) = o;
        }
    }
}

// Publish this workgroup's partials and, if it is the last split of (b, kvh) to arrive, merge all S.
// WT (write-through publish): the partials were stored with agent-scope atomic stores (global_store sc1,
// coherent at the device level once drained), so no release fence is needed -- the fence is a
// buffer_wbl2 that writes back EVERY dirty line of this XCD's L2, i.e. the preceding GEMMs' split-K
// slabs too, which is what made the fenced form lose inside the decode graph.
template <int G, bool WT = false>
__device__ __forceinline__ void combine_if_last(const float* part_o, const float* part_ml, int* counters,
                                                bf16* out, int out_stride, int b, int kvh, int Hq, int Hkv, int S,
                                                int* s_last, float* sw, float* sden) {
    const int tid = threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
    __syncthreads();
    if (tid == 0) {
        if constexpr (!WT) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int prev = __hip_atomic_fetch_add(counters + b * Hkv + kvh, 1, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
        *s_last = prev == S - 1;
    }
    __syncthreads();
    if (!*s_last) return;
    if constexpr (WT) {
        // write-through partials, drained before every ticket add: the merge reads them with sc1 loads
        // (L1 bypass), no acquire; the fence below only keeps the compiler from hoisting the loads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        combine_group<G, true>(part_o, part_ml, out, out_stride, b, kvh, Hq, S, sw, sden);
    } else {
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        combine_group<G>(part_o, part_ml, out, out_stride, b, kvh, Hq, S, sw, sden);
    }
    if (tid == 0) __hip_atomic_store(counters + b * Hkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int G>
__global__ __launch_bounds__(256) void attn_decode_combine_kernel(const float* __restrict__ part_o,
                                                                  const float* __restrict__ part_ml,
                                                                  bf16* __restrict__ out, int out_stride, int Hq,
                                                                  int Hkv, int S) {
    __shared__ float s_w[G * MAX_SPLITS];
    __shared__ float s_den[G];
    combine_group<G>(part_o, part_ml, out, out_stride, blockIdx.x / Hkv, blockIdx.x % Hkv, Hq, S, s_w, s_den);
}

// ---------------------------------------------------------------------------------------------
// MFMA variant (page size 64): the (b, kv head, split) workgroup stages each 64-key page of K and
// V through LDS (256 threads, 16-B coalesced loads of the contiguous 16 KiB page images, next
// page prefetched into registers while the current one is consumed), and each wave scores 16 of
// the 64 keys against all G query heads with MFMA:
//   S^T[16 keys][16 heads] = K . Q^T        v_mfma_f32_16x16x32_bf16, A = K rows (ds_read_b128,
//                                           chunks XOR-swizzled by key&15), B = Q^T in VGPRs
//   O^T[d][head]         += V^T . P^T       v_mfma_f32_16x16x16bf16_1k: the S^T accumulator IS the
//                                           B operand (same lane map), A = V^T from
//                                           ds_read_b64_tr_b16 (V chunks swizzled by (key&7)<<1)
// Softmax is per head column: 4 in-lane values + two xor shuffles per 16 keys.  No q.k lane
// reductions, no per-key VALU dot products -- the VALU only does the online softmax.
// Heads G <= 16 (columns >= G are computed on zero q and never stored).
// GQA ratios other than 1/2/4/8/16 (e.g. Llama-3.2-3B: 24 / 8 = 3) run the G = 1 instantiation over
// Hkv = Hq "virtual kv heads" (grid.y), one per query head, each streaming the pages of its cache kv head
// kvr = kvh / gq of Hc (gq = Hq / Hc); for them the split holding the new token writes the same K/V row
// from each of the gq virtual heads (identical bytes; every reader patches that row from LDS anyway).
namespace {
// Column reductions over the 4 rows of 16 lanes (lanes l, l^16, l^32, l^48) on the VALU: v_permlane16_swap /
// v_permlane32_swap of a value with itself give (even rows | odd rows) and (low half | high half) pairs, so one
// swap + one op per step -- no ds_bpermute round trip through the LDS pipe in the per-tile softmax chain.
__device__ __forceinline__ float rows_max4(float v) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float rows_sum4(float v) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;
__device__ __forceinline__ int dk_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }
__device__ __forceinline__ int dv_off(int row, int chunk) { return row * 256 + ((chunk ^ ((row & 7) << 1)) << 4); }
}  // namespace

// ROPE variant (decode): q is not a bf16 row but the QKV GEMM's fp32 split-K slabs ``qkv_parts``
// [SP, B, (Hq + 2 Hkv) D] -- the workgroup sums its G query heads' slabs, rotates them (RoPE at
// position ctx - 1) in registers, and the workgroup whose split holds position ctx - 1 also builds
// the new token's rotated K and V row from the slabs and writes it into the paged cache before
// streaming (its split is the only reader of that page in this launch: splits are whole pages).
// This folds the separate rope_kv_parts launch into the attention kernel.
struct RopeArgs {
    const float* parts;   // slab 0, row 0
    size_t slab_stride;   // elements between slabs (B * width)
    int SP;               // number of slabs
    int width;            // (Hq + 2 Hkv) * D elements per token row
    int hq_total;         // Hq of this rank
    const float2* cos_sin;  // [max_pos, D/2]
};

// The fp32 slab sums the ROPE variant needs, by all 256 threads: q of the G heads of head group ``kvh``
// (G D floats) and, with ``with_kv``, the new token's K and V rows of cache kv head ``kvr`` (of ``Hc``;
// kvr = kvh except for the per-query-head fallback of other GQA ratios) (D floats each), into ``sq``.
// Work items = float4 columns x slab subsets (NH subsets when there are fewer than 256 columns), so
// every thread has its loads in flight at once; the subsets are merged through LDS.
template <int G>
__device__ __forceinline__ void rope_slab_sums(const RopeArgs& ra, const float* prow, int kvh, int kvr, int Hc,
                                               bool with_kv, float* sq) {
    constexpr int D = 128;
    const int tid = threadIdx.x;
    const int nq = G * D / 4;                    // q float4 columns
    const int nv = nq + (with_kv ? 2 * D / 4 : 0);
    const int nh = nv >= 256 ? 1 : 256 / nv;
    float4* red = reinterpret_cast<float4*>(sq) + nv;  // [nh][nv] partials after the [nv] result
    for (int it = tid; it < nv * nh; it += 256) {
        const int item = it % nv, h = it / nv;
        int colf;
        if (item < nq) colf = kvh * G * D + 4 * item;
        else if (item < nq + D / 4) colf = (ra.hq_total + kvr) * D + 4 * (item - nq);
        else colf = (ra.hq_total + Hc + kvr) * D + 4 * (item - nq - D / 4);
        const float* src = prow + colf;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int s2 = h; s2 < ra.SP; s2 += nh) {
            const float4 v = *reinterpret_cast<const float4*>(src + (size_t)s2 * ra.slab_stride);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        red[it] = acc;
    }
    __syncthreads();
    float4* out = reinterpret_cast<float4*>(sq);
    for (int item = tid; item < nv; item += 256) {
        float4 acc = red[item];
        for (int h = 1; h < nh; ++h) {
            const float4 v = red[h * nv + item];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        out[item] = acc;
    }
    __syncthreads();
}

// KV page loads: nontemporal (each page is read once per step by one workgroup) when NT
template <bool NT, typename T>
__device__ __forceinline__ u32x4 ld_kv(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}

// KV8 (FP8 KV cache, kv8.h): each (page, kv head) is an 8.25 KiB slab of e4m3 rows + fp32 row scales.
// The staging loads half the bytes (thread -> row tid / 8 + 32 i, 16-B chunk tid % 8 = 16 dims, 2 rows per
// tile per thread) plus each row's scale, and converts every row to bf16 exactly (power-of-two scales)
// while writing it into the SAME LDS image the bf16 cache fills: QK^T, softmax and PV are unchanged.
// The fused RoPE writer quantises the new token's rows (kv8 row rule) and patches their DEQUANTISED
// values into the tile, so this step and later steps see the same K/V.  KVM is a bitmask: bit 0 = the K
// cache is fp8 slabs, bit 1 = the V cache is; KVM 2 ("fp8v": bf16 K, fp8 V) stages K with the bf16
// mapping and V with the slab mapping, each into its own LDS tile.
template <int G, bool ROPE, bool NT = false, int KVM = 0>
__global__ __launch_bounds__(256, 3) void attn_decode_mfma_kernel(
    const bf16* __restrict__ q, int q_stride, bf16* __restrict__ kc, bf16* __restrict__ vc,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ positions,
    float* __restrict__ part_o, float* __restrict__ part_ml, int Hkv, int S, float scale_log2, RopeArgs ra,
    int* __restrict__ counters, bf16* __restrict__ out, int out_stride, int Hc_rt, int gq) {
    constexpr int D = 128, PG = 64;
    ST_DECL
    __shared__ __attribute__((aligned(16))) char lds[2 * PG * 256 + 2 * 4 * 16 * 4];
    __shared__ __attribute__((aligned(16))) bf16 lds_new[2 * D];  // ROPE: the new token's K | V row (bf16)
    // fused split merge (``counters``): weights [G][MAX_SPLITS] + denominators + last flag, aliasing lds
    float* c_sw = reinterpret_cast<float*>(lds);
    float* c_den = c_sw + G * MAX_SPLITS;
    int* c_last = reinterpret_cast<int*>(c_den + 16);
    char* ldsK = lds;
    char* ldsV = lds + PG * 256;
    float* sm_ml = reinterpret_cast<float*>(lds + 2 * PG * 256);  // [2][4 waves][16 heads]

    const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
    const int Hq = Hkv * G;
    // cache kv head / cache kv heads (the per-query-head fallback exists only as G = 1)
    const int kvr = G == 1 ? kvh / gq : kvh;
    const int Hc = G == 1 ? Hc_rt : Hkv;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, col = lane & 15, grp = lane >> 4;
    const int ctx = positions[b] + 1;
    int chunk = (ctx + S - 1) / S;
    chunk = (chunk + PG - 1) & ~(PG - 1);
    const int ks = split * chunk;
    const int ke = min(ctx, ks + chunk);
    const size_t ml_base = ((size_t)b * Hq + (size_t)kvh * G) * S + split;
    if (ks >= ke) {
        // an empty split (the context ends before it) still publishes a zero slab: the merge weights it by
        // 0, and 0 x a stale NaN / inf left in the (reused, uninitialised) workspace would be NaN
        for (int i = tid; i < G * D; i += 256)
            st_part(part_o + (ml_base + (size_t)(i / D) * S) * D + i % D, 0.f, counters != nullptr);
        if (tid < G) {
            st_part(part_ml + (ml_base + (size_t)tid * S) * 2 + 0, -INFINITY, counters != nullptr);
            st_part(part_ml + (ml_base + (size_t)tid * S) * 2 + 1, 0.f, counters != nullptr);
        }
        if (counters) combine_if_last<G, true>(part_o, part_ml, counters, out, out_stride, b, kvh, Hq, Hkv, S, c_last, c_sw, c_den);
        return;
    }
    const int ntiles = (ke - ks + PG - 1) / PG;

    const float* prow = ROPE ? ra.parts + (size_t)b * ra.width : nullptr;
    const float2* cs = ROPE ? ra.cos_sin + (size_t)(ctx - 1) * (D / 2) : nullptr;
    const int* bt = block_tables + (size_t)b * bt_stride + ks / PG;
    const int st_row = tid >> 4, st_chunk = tid & 15;
    const size_t head_off = (size_t)kvr * PG * D + (size_t)st_row * D + st_chunk * 8;
    // KV8 staging: row r8 + 32 i, 16-B fp8 chunk c8 (dims 16 c8 .. +16) of the (page, head) slab
    const int r8 = tid >> 3, c8 = tid & 7;
    const size_t head8 = (size_t)kvr * kv8::SLAB;
    const unsigned char* kc8 = reinterpret_cast<const unsigned char*>(kc);
    const unsigned char* vc8 = reinterpret_cast<const unsigned char*>(vc);
    float ksc[2], vsc[2], ksc2[2], vsc2[2];  // fp8 slabs: row scales of register sets A and B
    constexpr bool K8 = (KVM & 1) != 0, V8 = (KVM & 2) != 0;
    // staging registers are plain named arrays indexed only by unrolled constants (a lambda
    // capturing them by reference put them in scratch), and the prefetch is unconditional (no
    // branch around the loads) so hipcc keeps them in flight.
    // (issued first by every split, the one holding the new token included: its new K/V row reaches
    // the tile through the LDS patch, so the page loads need not wait for the slab sums)
    // TWO tiles in flight: register sets A (kreg/vreg) and B (kreg2/vreg2) alternate; the (up to two)
    // loads past the last tile stay unconditional but read the scratch page 0, which every workgroup's
    // overshoot shares and so stays in L2 (re-reading the workgroup's own last tile cost ~9 % extra HBM
    // traffic at B=39, PMC FETCH_SIZE).
    u32x4 kreg[4], vreg[4], kreg2[4], vreg2[4];
#define KV_ISSUE(KR, VR, KS, VS, TILE)                                                              \
    {                                                                                               \
        const int pg_ = bt[min((TILE), ntiles - 1)];                                                \
        const int pgx_ = (TILE) < ntiles ? pg_ : 0;                                                 \
        const size_t base8_ = (size_t)pgx_ * Hc * kv8::SLAB + head8;                                \
        const size_t base_ = (size_t)pgx_ * Hc * PG * D + head_off;                                 \
        if constexpr (K8) {                                                                         \
            _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                         \
                KR[i] = ld_kv<NT>(kc8 + base8_ + (size_t)(r8 + 32 * i) * D + 16 * c8);               \
                KS[i] = *reinterpret_cast<const float*>(kc8 + base8_ + PG * D + 4 * (r8 + 32 * i)); \
            }                                                                                       \
        } else {                                                                                    \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) KR[i] = ld_kv<NT>(kc + base_ + (size_t)16 * i * D); \
        }                                                                                           \
        if constexpr (V8) {                                                                         \
            _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                         \
                VR[i] = ld_kv<NT>(vc8 + base8_ + (size_t)(r8 + 32 * i) * D + 16 * c8);               \
                VS[i] = *reinterpret_cast<const float*>(vc8 + base8_ + PG * D + 4 * (r8 + 32 * i)); \
            }                                                                                       \
        } else {                                                                                    \
            _Pragma("unroll") for (int i = 0; i < 4; ++i) VR[i] = ld_kv<NT>(vc + base_ + (size_t)16 * i * D); \
        }                                                                                           \
    }
    KV_ISSUE(kreg, vreg, ksc, vsc, 0)
    KV_ISSUE(kreg2, vreg2, ksc2, vsc2, 1)
    // ROPE: the q rows of this group (and, for the split holding the new token, its K and V rows)
    // summed over the SP slabs by ALL 256 threads in one round of independent loads into an fp32
    // LDS image (aliasing the K/V tile buffers, which are first written after it is consumed):
    // q at [0, G D), K at [G D, G D + D), V after it.  A per-lane serial sum cost SP / 4 dependent
    // L2/MALL round trips per operand (22 us per layer at TP = 8, SP = 16).
    float* sq = reinterpret_cast<float*>(lds);
    const bool has_pos = ROPE && ks <= ctx - 1 && ctx - 1 < ke;
    if constexpr (ROPE) {
        if (has_pos) {
            rope_slab_sums<G>(ra, prow, kvh, kvr, Hc, true, sq);
            // the new token's K (rotated) and V row of this kv head -> paged cache for the next steps;
            // THIS launch never reads it back from memory (no store drain on the critical path): the
            // staging of the page that holds it patches the row into LDS from the fp32 image
            // (lds_new); only this split reads that page in this launch
            const int pos = ctx - 1;
            const int page = block_tables[(size_t)b * bt_stride + pos / PG];
            const size_t dst = ((size_t)page * Hc * PG + (size_t)kvr * PG + (pos % PG)) * D;
            const float* kr = sq + G * D;
            if (tid < D / 4) {  // lanes 0-15: rotated K chunk (8 dims); 16-31: V chunk -> cache + LDS patch row
                const bool isk = tid < D / 8;
                const int c = (isk ? tid : tid - D / 8) * 8, cl = c & (D / 2 - 1);
                float kv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (isk) {
                        const float2 e = cs[cl + j];
                        const float lo = kr[cl + j], hi = kr[cl + j + D / 2];
                        kv[j] = c < D / 2 ? lo * e.x - hi * e.y : hi * e.x + lo * e.y;
                    } else {
                        kv[j] = kr[D + c + j];
                    }
                }
                bf16* pdst = lds_new + (isk ? 0 : D) + c;
                if constexpr (KVM != 0) {
                    // quantise the bf16-rounded row, as every other writer does (rope_kv.hip), then the row's 16
                    // lanes (K: 0-15, V: 16-31) reduce max|x| (kv8.h row rule) -- all 32 lanes shuffle, a row
                    // whose cache is bf16 (fp8v: K) then takes the bf16 store below
#pragma unroll
                    for (int j = 0; j < 8; ++j) kv[j] = (float)(bf16)kv[j];
                    float amax = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(kv[j]));
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
                    if (isk ? !K8 : !V8) {
                        const uint4 pk = pack8(kv);
                        *reinterpret_cast<uint4*>((isk ? kc : vc) + dst + c) = pk;
                        *reinterpret_cast<uint4*>(pdst) = pk;
                    } else {
                    const float sc = kv8::row_scale(amax), inv = 1.f / sc;
                    const uint2 q = make_uint2(kv8::pack4(kv[0] * inv, kv[1] * inv, kv[2] * inv, kv[3] * inv),
                                               kv8::pack4(kv[4] * inv, kv[5] * inv, kv[6] * inv, kv[7] * inv));
                    unsigned char* cb = reinterpret_cast<unsigned char*>(isk ? kc : vc) +
                                        (size_t)page * Hc * kv8::SLAB + head8;
                    *reinterpret_cast<uint2*>(cb + (size_t)(pos % PG) * D + c) = q;
                    if (c == 0) *reinterpret_cast<float*>(cb + PG * D + 4 * (pos % PG)) = sc;
                    // patch row = the dequantised values later steps read back
                    u32x4 lo, hi;
                    kv8::dequant16(u32x4{q.x, q.y, 0u, 0u}, sc, lo, hi);
                    *reinterpret_cast<u32x4*>(pdst) = lo;
                    }
                } else {
                    const uint4 pk = pack8(kv);
                    *reinterpret_cast<uint4*>((isk ? kc : vc) + dst + c) = pk;
                    *reinterpret_cast<uint4*>(pdst) = pk;
                }
            }
        }
    }

    // Q^T fragments (B operand of 16x16x32): lane holds Q[head col][dims 32k + 8grp .. +8]; built
    // after the first page's loads are in flight (the ROPE slab sums are an L2 round trip of their own)
    bf16x8 qf[4];
    if constexpr (ROPE) {
        // dims 32k + 8grp + j (k = 0, 1) pair with dims 64 + the same (k = 2, 3): the rotation of a
        // lane's q values needs only the lane's own values
        if (!has_pos) rope_slab_sums<G>(ra, prow, kvh, kvr, Hc, false, sq);  // overlaps the first page's loads
        float a[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int j = 0; j < 8; ++j) a[k][j] = col < G ? sq[col * D + 32 * k + 8 * grp + j] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            float lo[8], hi[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float2 e = cs[32 * k + 8 * grp + j];
                lo[j] = a[k][j] * e.x - a[k + 2][j] * e.y;
                hi[j] = a[k + 2][j] * e.x + a[k][j] * e.y;
            }
            qf[k] = __builtin_bit_cast(bf16x8, pack8(lo));
            qf[k + 2] = __builtin_bit_cast(bf16x8, pack8(hi));
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (col < G) v = *reinterpret_cast<const uint4*>(q + (size_t)b * q_stride + (kvh * G + col) * D + 32 * k + 8 * grp);
            qf[k] = __builtin_bit_cast(bf16x8, v);
        }
    }
    // the new token's row (row pr of tile ptile) is staged from lds_new, not from the page loads
    const int ptile = has_pos ? (ctx - 1 - ks) / PG : -1;
    const int pr = (ctx - 1 - ks) % PG;
    const bool patcher_k = has_pos && (K8 ? r8 == (pr & 31) : st_row == (pr & 15));
    const bool patcher_v = has_pos && (V8 ? r8 == (pr & 31) : st_row == (pr & 15));
    if constexpr (ROPE) {
        __syncthreads();  // every lane has its q out of the fp32 image the tiles overwrite
    }
#define KV_WRITE(KR, VR, KS, VS, TILE)                                                                          \
    if constexpr (K8) {                                                                                         \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                         \
            const bool pt = ROPE && ptile == (TILE) && patcher_k && i == (pr >> 5);                             \
            const int row_ = r8 + 32 * i;                                                                       \
            u32x4 klo, khi;                                                                                     \
            kv8::dequant16(KR[i], KS[i], klo, khi);                                                             \
            if (pt) {                                                                                           \
                klo = *reinterpret_cast<const u32x4*>(lds_new + 16 * c8);                                       \
                khi = *reinterpret_cast<const u32x4*>(lds_new + 16 * c8 + 8);                                   \
            }                                                                                                   \
            *reinterpret_cast<u32x4*>(ldsK + dk_off(row_, 2 * c8)) = klo;                                      \
            *reinterpret_cast<u32x4*>(ldsK + dk_off(row_, 2 * c8 + 1)) = khi;                                  \
        }                                                                                                       \
    } else {                                                                                                    \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                         \
            const bool pt = ROPE && ptile == (TILE) && patcher_k && i == (pr >> 4);                             \
            *reinterpret_cast<u32x4*>(ldsK + dk_off(st_row + 16 * i, st_chunk)) =                               \
                pt ? *reinterpret_cast<const u32x4*>(lds_new + st_chunk * 8) : KR[i];                           \
        }                                                                                                       \
    }                                                                                                           \
    if constexpr (V8) {                                                                                         \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                         \
            const bool pt = ROPE && ptile == (TILE) && patcher_v && i == (pr >> 5);                             \
            const int row_ = r8 + 32 * i;                                                                       \
            u32x4 vlo, vhi;                                                                                     \
            kv8::dequant16(VR[i], VS[i], vlo, vhi);                                                             \
            if (pt) {                                                                                           \
                vlo = *reinterpret_cast<const u32x4*>(lds_new + D + 16 * c8);                                   \
                vhi = *reinterpret_cast<const u32x4*>(lds_new + D + 16 * c8 + 8);                               \
            }                                                                                                   \
            *reinterpret_cast<u32x4*>(ldsV + dv_off(row_, 2 * c8)) = vlo;                                      \
            *reinterpret_cast<u32x4*>(ldsV + dv_off(row_, 2 * c8 + 1)) = vhi;                                  \
        }                                                                                                       \
    } else {                                                                                                    \
        _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                         \
            const bool pt = ROPE && ptile == (TILE) && patcher_v && i == (pr >> 4);                             \
            *reinterpret_cast<u32x4*>(ldsV + dv_off(st_row + 16 * i, st_chunk)) =                               \
                pt ? *reinterpret_cast<const u32x4*>(lds_new + D + st_chunk * 8) : VR[i];                       \
        }                                                                                                       \
    }
    KV_WRITE(kreg, vreg, ksc, vsc, 0)
    KV_ISSUE(kreg, vreg, ksc, vsc, 2)

    f32x4 o[8];
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    const int q4 = col >> 2, p4 = col & 3;
    __syncthreads();

    auto compute = [&](int t) {
        const int key0 = ks + t * PG + 16 * w;  // this wave's 16 keys
        if (key0 < ke) {
            f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint4 a = *reinterpret_cast<const uint4*>(ldsK + dk_off(16 * w + col, 4 * k + grp));
                sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), qf[k], sacc, 0, 0, 0);
            }
            const int kb = key0 + 4 * grp;
            const float s0 = kb + 0 < ke ? sacc[0] * scale_log2 : -INFINITY;
            const float s1 = kb + 1 < ke ? sacc[1] * scale_log2 : -INFINITY;
            const float s2 = kb + 2 < ke ? sacc[2] * scale_log2 : -INFINITY;
            const float s3 = kb + 3 < ke ? sacc[3] * scale_log2 : -INFINITY;
            float mt = fmaxf(fmaxf(s0, s1), fmaxf(s2, s3));
            mt = rows_max4(mt);
            const float mn = fmaxf(m, mt);  // finite: key0 < ke is a valid key for every head
            const float alpha = __builtin_amdgcn_exp2f(m - mn);
            m = mn;
            const float p0 = __builtin_amdgcn_exp2f(s0 - mn), p1 = __builtin_amdgcn_exp2f(s1 - mn), p2 = __builtin_amdgcn_exp2f(s2 - mn), p3 = __builtin_amdgcn_exp2f(s3 - mn);
            lsum = lsum * alpha + (p0 + p1) + (p2 + p3);
            const s4v pb = {__builtin_bit_cast(short, (bf16)p0), __builtin_bit_cast(short, (bf16)p1),
                            __builtin_bit_cast(short, (bf16)p2), __builtin_bit_cast(short, (bf16)p3)};
            const int vrow = 16 * w + 4 * grp + q4;
#pragma unroll
            for (int dt = 0; dt < 8; ++dt) {
                o[dt] *= alpha;
                const s4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s4v*)(ldsV + dv_off(vrow, 2 * dt + (p4 >> 1)) + 8 * (p4 & 1)));
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, pb, o[dt], 0, 0, 0);
            }
        }
    };
    // LDS holds tile t; set B carries tile t + 1 and set A tile t + 2 (two tiles in flight while a tile
    // is scored); unrolled by two so every register array is indexed statically.  (Four sets in flight at
    // one workgroup per CU measured SLOWER in round 5: B=1 at 13.5k +1.5-2.5 %, the TP=8 shard +10 %, the
    // overshoot loads past a short split's last tile outweighing the deeper queue: r5_attn_deep_ab.jsonl; again
    // in round 6, r6_attn_deep_ring_insitu.jsonl.  Nor did 4 staging waves beside the 4 scoring ones over two
    // LDS tile buffers: the loaders wait on the page loads, r6_attn_stamps.jsonl.)
    ST(0)
    for (int t = 0; t < ntiles; t += 2) {
        compute(t);
        ST(1)
        __syncthreads();
        ST(2)
        if (t + 1 < ntiles) {
            KV_WRITE(kreg2, vreg2, ksc2, vsc2, t + 1)
            KV_ISSUE(kreg2, vreg2, ksc2, vsc2, t + 3)
            ST(3)
            __syncthreads();
            ST(4)
            compute(t + 1);
            ST(1)
            __syncthreads();
            ST(2)
        }
        if (t + 2 < ntiles) {
            KV_WRITE(kreg, vreg, ksc, vsc, t + 2)
            KV_ISSUE(kreg, vreg, ksc, vsc, t + 4)
            ST(3)
            __syncthreads();
            ST(4)
        }
    }
#undef KV_ISSUE
#undef KV_WRITE

    // merge the 4 waves: lane (grp, col) holds O^T[d = 16dt + 4grp + j][head col]
    lsum = rows_sum4(lsum);
    float* sm_o = reinterpret_cast<float*>(lds);  // [4][128][16] f32 = 32 KiB, reuses the tile buffers
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int j = 0; j < 4; ++j) sm_o[(w * D + 16 * dt + 4 * grp + j) * 16 + col] = o[dt][j];
    if (grp == 0) {
        sm_ml[w * 16 + col] = m;
        sm_ml[64 + w * 16 + col] = lsum;
    }
    __syncthreads();
    for (int i = tid; i < G * D; i += 256) {
        const int h = i / D, d = i % D;
        float M = -INFINITY;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, sm_ml[ww * 16 + h]);
        float acc = 0.f, L = 0.f;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) {
            const float mw = sm_ml[ww * 16 + h];
            const float wt = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M);
            acc += wt * sm_o[(ww * D + d) * 16 + h];
            L += wt * sm_ml[64 + ww * 16 + h];
        }
        const size_t pi = ml_base + (size_t)h * S;
        st_part(part_o + pi * D + d, acc, counters != nullptr);
        if (d == 0) {
            st_part(part_ml + pi * 2 + 0, M, counters != nullptr);
            st_part(part_ml + pi * 2 + 1, L, counters != nullptr);
        }
    }
    if (counters) combine_if_last<G, true>(part_o, part_ml, counters, out, out_stride, b, kvh, Hq, Hkv, S, c_last, c_sw, c_den);
    ST(5)
    ST_STORE(ntiles)
}

// KV page loads are nontemporal from 64 (sequence, kv head) groups up -- measured, step at 4k context:
// B=39 x 8 kv heads 7.02-7.05 vs 7.18-7.26 ms with the default policy; B <= 10 0.7-1 % slower with nt
// (profiles/r1_decode_nt_ab.jsonl)
constexpr int NT_MIN_GROUPS = 64;

static bool decode_packed(int G) { return G == 1 || G == 2 || G == 4 || G == 8 || G == 16; }

// Head groups (grid.y) the decode attention runs for Hq query / Hkv kv heads: Hkv for the packed GQA ratios,
// Hq (one per query head) for the fallback -- the split workspace and merge tickets are sized by it.
MRSUM_API int mrsum_attn_decode_groups(int Hq, int Hkv) {
    if (Hkv <= 0 || Hq % Hkv || Hq / Hkv > 64) return -1;
    return decode_packed(Hq / Hkv) ? Hkv : Hq;
}

static int launch_mfma(const void* q, int q_stride, const void* kcache, const void* vcache, const int* block_tables,
                       int bt_stride, const int* positions, void* part_o, void* part_ml, void* out, int out_stride,
                       int B, int Hq, int Hkv, int D, int P, int S, float scale, const RopeArgs* rope, int* counters,
                       int kv8, hipStream_t s) {
    if (B <= 0) return 0;
    if (D != 128 || P != 64 || Hkv <= 0 || Hq % Hkv || Hq / Hkv > 64 || S < 1 || S > MAX_SPLITS ||
        (kv8 != 0 && kv8 != 2 && kv8 != 3) || !out)
        return (int)hipErrorInvalidValue;
    const int Hc = Hkv;                          // kv heads of the cache
    const int gq = decode_packed(Hq / Hc) ? 1 : Hq / Hc;
    Hkv = Hq / (decode_packed(Hq / Hc) ? Hq / Hc : 1);  // head groups of the grid (virtual kv heads)
    const int G = Hq / Hkv;
    const float sl = scale * 1.4426950408889634f;
    dim3 grid(S, Hkv, B), block(256);
    auto Qp = (const bf16*)q; auto K = (bf16*)kcache; auto V = (bf16*)vcache;
    auto PO = (float*)part_o; auto PM = (float*)part_ml;
    const RopeArgs ra = rope ? *rope : RopeArgs{nullptr, 0, 0, 0, 0, nullptr};
#define MFMA_K(G_, R_, NT_, K8_)                                                                                \
    attn_decode_mfma_kernel<G_, R_, NT_, K8_><<<grid, block, 0, s>>>(Qp, q_stride, K, V, block_tables, bt_stride,  \
                                                                     positions, PO, PM, Hkv, S, sl, ra, counters, \
                                                                     (bf16*)out, out_stride, Hc, gq)
#define MFMA_L(G_, R_)                                                                                        \
    do {                                                                                                      \
        const bool nt_ = B * Hkv >= NT_MIN_GROUPS;                                                            \
        if (kv8 == 3) { if (nt_) MFMA_K(G_, R_, true, 3); else MFMA_K(G_, R_, false, 3); }                    \
        else if (kv8 == 2) { if (nt_) MFMA_K(G_, R_, true, 2); else MFMA_K(G_, R_, false, 2); }               \
        else { if (nt_) MFMA_K(G_, R_, true, 0); else MFMA_K(G_, R_, false, 0); }                             \
    } while (0)
#define MFMA_G(R_)                            \
    switch (G) {                              \
        case 1: MFMA_L(1, R_); break;         \
        case 2: MFMA_L(2, R_); break;         \
        case 4: MFMA_L(4, R_); break;         \
        case 8: MFMA_L(8, R_); break;         \
        case 16: MFMA_L(16, R_); break;       \
        default: return (int)hipErrorInvalidValue; \
    }
    if (rope) { MFMA_G(true) } else { MFMA_G(false) }
#undef MFMA_G
#undef MFMA_L
#undef MFMA_K
    int e = (int)hipGetLastError();
    if (e || counters) return e;
    if (S > 16) {
        // many splits (long contexts): one merge workgroup per query head instead of per kv-head group,
        // G x more workgroups with G x fewer partial loads each (B=1, 11k context, S=48: 8 workgroups
        // took 10 us)
        attn_decode_combine_kernel<1><<<B * Hq, 256, 0, s>>>(PO, PM, (bf16*)out, out_stride, Hq, Hq, S);
        return (int)hipGetLastError();
    }
    switch (G) {
        case 1: attn_decode_combine_kernel<1><<<B * Hkv, 256, 0, s>>>(PO, PM, (bf16*)out, out_stride, Hq, Hkv, S); break;
        case 2: attn_decode_combine_kernel<2><<<B * Hkv, 256, 0, s>>>(PO, PM, (bf16*)out, out_stride, Hq, Hkv, S); break;
        case 4: attn_decode_combine_kernel<4><<<B * Hkv, 256, 0, s>>>(PO, PM, (bf16*)out, out_stride, Hq, Hkv, S); break;
        case 8: attn_decode_combine_kernel<8><<<B * Hkv, 256, 0, s>>>(PO, PM, (bf16*)out, out_stride, Hq, Hkv, S); break;
        case 16: attn_decode_combine_kernel<16><<<B * Hkv, 256, 0, s>>>(PO, PM, (bf16*)out, out_stride, Hq, Hkv, S); break;
    }
    return (int)hipGetLastError();
}

MRSUM_API int mrsum_attn_decode_mfma(const void* q, int q_stride, const void* kcache, const void* vcache,
                                     const int* block_tables, int bt_stride, const int* positions, void* part_o,
                                     void* part_ml, void* out, int out_stride, int B, int Hq, int Hkv, int D, int P,
                                     int S, float scale, int* counters, int kv8, hipStream_t s) {
    return launch_mfma(q, q_stride, kcache, vcache, block_tables, bt_stride, positions, part_o, part_ml, out,
                       out_stride, B, Hq, Hkv, D, P, S, scale, nullptr, counters, kv8, s);
}

// Decode attention straight from the QKV GEMM's fp32 split-K slabs [SP, B, (Hq + 2 Hkv) D]: RoPE on q,
// the new token's K/V rotated + written into the paged cache, attention, split merge (2 launches).
MRSUM_API int mrsum_attn_decode_rope(const void* qkv_parts, int SP, const void* cos_sin, void* kcache, void* vcache,
                                     const int* block_tables, int bt_stride, const int* positions, void* part_o,
                                     void* part_ml, void* out, int out_stride, int B, int Hq, int Hkv, int D, int P,
                                     int S, float scale, int* counters, int kv8, hipStream_t s) {
    if (SP < 1 || !qkv_parts || !cos_sin) return (int)hipErrorInvalidValue;
    const int width = (Hq + 2 * Hkv) * D;
    const RopeArgs ra{(const float*)qkv_parts, (size_t)B * width, SP, width, Hq, (const float2*)cos_sin};
    return launch_mfma(nullptr, 0, kcache, vcache, block_tables, bt_stride, positions, part_o, part_ml, out,
                       out_stride, B, Hq, Hkv, D, P, S, scale, &ra, counters, kv8, s);
}
