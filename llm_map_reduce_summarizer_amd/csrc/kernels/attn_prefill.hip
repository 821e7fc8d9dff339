// Causal varlen flash attention for prefill on MFMA.
//
// Packed batch: qkv [T, row_stride] bf16 (Q heads, then K heads, then V
// heads, D=128 each, already rotated by rope_kv), cu_seqlens [nseq+1].
// Work item = (sequence, query block of 256/G positions) x KV HEAD, G = Hq / Hkv: the 8 waves
// of a workgroup run all G query heads of their kv head (wave w: head kvh*G + w%G, rows 32(w/G)..+32), so a
// staged K/V tile always feeds 256 query rows, and the causal diagonal of a block is only 256/G rows deep
// (64 for Llama-3-8B, 32 for 70B: waves idle on masked diagonal tiles far less than with 256-row blocks of
// one head).  Items are listed by the host heaviest-first (blocks late in a sequence do the most key tiles).
//
// Workgroup: 8 waves (one per CU, 2 per SIMD at ~216 VGPRs).  K/V tiles go through a two-stage LDS ring with
// one barrier per tile: right after barrier t every wave writes tile t+1 (loaded into registers one tile
// earlier) into the other stage and issues the global loads of tile t+2, then consumes tile t.  The LDS
// operand reads run ahead of their MFMAs under sched_group_barrier (8 fragments deep, counted lgkmcnt
// waits; hipcc otherwise sank each read next to its MFMA behind an lgkmcnt(0)).  GQA packing + ring +
// read-ahead: 8 x 4k 728 -> 873 TF/s, 1 x 32k 839 -> 1092, 70B heads 1 x 32k 874 -> 1100
// (profiles/r3_attn_prefill_gqa_ab.jsonl, r3_attn_prefill_stagger_ab.jsonl).
// Per 64-key tile (K and V staged through LDS, next tile prefetched into
// registers while the current one is consumed - issue early / write late):
//
//   S^T = K . Q^T   v_mfma_f32_32x32x16_bf16, A = K rows from LDS
//                   (ds_read_b128, 16-B chunks XOR-swizzled by row&15 so a
//                   16-lane group hits 16 distinct slots), B = Q^T fragments
//                   held in VGPRs for the whole loop.  The "swapped" product
//                   puts one query row per lane (col = lane&31), so the row
//                   max is 31 in-lane fmax + one v_permlane32_swap.
//   softmax         online, log2 domain; causal + length mask only on tiles that reach the
//                   diagonal or the sequence end; one FMA + raw v_exp_f32 per score; the running
//                   max (and the o/l rescale) only moves when it grows by > 2^8 (deferred rescale).
//                   ~160 VALU ops per 32 scores instead of ~350 (MFMA utilisation 20 % -> 26 %, PMC).
//   O^T += V^T . P^T  the S^T accumulator registers, converted to bf16, are
//                   directly the B operand (cdna_hip_programming.md §3
//                   "accumulator tile as the next MFMA's operand"); the A
//                   operand V^T comes from ds_read_b64_tr_b16 transposed
//                   reads of the row-major V tile, whose 16-B chunks are
//                   XOR-swizzled by (row&3)<<2 so the four rows of one
//                   transposed read land on four different 64-B bank ranges.
//
// PAGED (chunked prefill): the packed rows are SLICES of prompts whose first prefix[seq] tokens are
// already in the paged KV cache (rope_kv wrote this slice's K/V there too, before this launch).  Keys
// are then read from the cache -- one 64-key tile is exactly one page of one kv head, 16 KiB
// contiguous -- for positions [0, prefix + slice), and query row qi sits at absolute position
// prefix + qi (causal offset).  With prefix = 0 it is the same attention as the contiguous path.
//
// PAGED + KV8 (fp8 KV cache, kv8.h): a 64-key tile is one (page, head) slab of e4m3 rows + row scales;
// each thread loads one 16-B chunk (16 dims) of one row of K and of V plus the two row scales, and the
// store converts them exactly to bf16 into the same LDS image (the rest of the kernel is unchanged).
// KVM is a bitmask (bit 0: the K cache is fp8 slabs, bit 1: the V cache is); KVM 2 ("fp8v") stages K as
// bf16 rows and V as fp8 slab rows, each into its half of the tile.
//
// Numerics: bf16 inputs, fp32 accumulation and softmax, bf16 output.
#include "kv8.h"

namespace {
constexpr int D = 128;
constexpr int NW = 8;             // waves per workgroup, 32 query rows each
constexpr int NTHR = 64 * NW;
constexpr int SROWS = NTHR / 16;  // tile rows staged per load round (16 lanes x 16 B per 256-B row)
constexpr int BN = 64;            // keys per tile
constexpr int SIT = BN / SROWS;   // load rounds per 64-row tile
constexpr int STAGE = 2 * BN * 256;  // bytes of one ring stage: K tile | V tile
constexpr float RESCALE_LOG2 = 8.0f;  // deferred-rescale threshold (log2 units), see the softmax

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ int k_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }
__device__ __forceinline__ int v_off(int row, int chunk) { return row * 256 + ((chunk ^ ((row & 3) << 2)) << 4); }

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// v_permlane32_swap of one value with itself: x0 = [lo | lo], x1 = [hi | hi]
__device__ __forceinline__ float halves_max(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
}  // namespace

struct PagedKV {
    const bf16* kc;            // [pages, Hkv, 64, D]
    const bf16* vc;
    const int* block_tables;   // [slots, bt_stride]
    int bt_stride;
    const int* seq_slot;       // [nseq] decode slot (block-table row) of every packed sequence
    const int* prefix;         // [nseq] tokens already cached before this slice
};

// G = query heads per kv head served by one workgroup: wave w runs query head kvh*G + w%G over query rows
// [qblock + 32(w/G), +32), so one workgroup covers 256/G query positions of ALL G heads of its kv head and
// every staged K/V tile feeds 8 x 32 query rows whatever the GQA ratio.
// Other GQA ratios (e.g. Llama-3.2-3B: 24 / 8 = 3) run the G = 1 instantiation over Hg = Hq "virtual kv
// heads", one per query head, each reading the K/V columns of its real kv head h / gq (gq = Hq / Hkv):
// no K/V reuse across the group inside a workgroup, but any ratio works.  Hg = Hkv and gq = 1 otherwise.
template <bool PAGED, int G, int KVM = 0>
__global__ __launch_bounds__(NTHR, 1) void attn_prefill_kernel(const bf16* __restrict__ qkv, int row_stride,
                                                              const int* __restrict__ cu_seqlens,
                                                              const int2* __restrict__ items,
                                                              bf16* __restrict__ out, int out_stride, int Hq,
                                                              int Hkv, int Hg, int gq, float scale_log2, PagedKV pk,
                                                              int kv_major) {
    constexpr int BMP = 32 * (NW / G);  // query positions per workgroup
    // two-stage ring of [K tile | V tile]: tile t+1 is written into the other stage while tile t is
    // consumed, one barrier per tile
    __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

    // Block order.  Small grids (kv_major = 0): block b = item b / Hkv x kv head b % Hkv, the host's heaviest-
    // first order across ALL kv heads -- kv-head-major order started kv head 7's heaviest blocks only after
    // kv head 0-6's lists (1 x 4k: 580 vs 870 TF/s).  Large grids (kv_major = 1): block b = kv head
    // b / n_items x item b % n_items, so the blocks in flight share one kv head and its K/V stays in the
    // Infinity Cache (39 x 4k: 912 vs 815 TF/s); profiles/r3_attn_prefill_grid_order_ab.jsonl.
    const int n_items = gridDim.x / Hg;
    const int item = kv_major ? blockIdx.x % n_items : blockIdx.x / Hg;
    const int2 it = items[item];
    const int seq = it.x, qblock = it.y;
    const int kvg = kv_major ? blockIdx.x / n_items : blockIdx.x % Hg;  // head group of this workgroup
    const int kvh = G == 1 ? kvg / gq : kvg;                             // its real kv head
    const int tid = threadIdx.x, lane = tid & 63, half = lane >> 5, r32 = lane & 31;
    const int w = tid >> 6;
    const int h = G == 1 ? kvg : kvh * G + w % G, rb = w / G;
    const int s0 = cu_seqlens[seq], len = cu_seqlens[seq + 1] - s0;
    const bf16* base = qkv + (size_t)s0 * row_stride;
    const int kcol = (Hq + kvh) * D, vcol = (Hq + Hkv + kvh) * D;
    // keys live at absolute positions [0, pre + len); query row qi at pre + qi
    const int pre = PAGED ? pk.prefix[seq] : 0;
    const int* btab = PAGED ? pk.block_tables + (size_t)pk.seq_slot[seq] * pk.bt_stride : nullptr;
    const size_t head_pg = (size_t)kvh * BN * D;  // this kv head's 64-row slab inside a page

    // Q^T fragments: lane holds Q[row r32][dims 16ks + 8half .. +8] for ks = 0..7
    const int q0 = qblock + 32 * rb;  // the wave's first query row
    const int qi = q0 + r32;
    bf16x8 qf[8];
    {
        const bool ok = qi < len;
        const bf16* qp = base + (size_t)(ok ? qi : 0) * row_stride + h * D + 8 * half;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            uint4 v = *reinterpret_cast<const uint4*>(qp + 16 * ks);
            if (!ok) v = make_uint4(0, 0, 0, 0);
            qf[ks] = as_bf16x8(v);
        }
    }

    const int kend = pre + min(len, qblock + BMP);
    const int ntiles = (kend + BN - 1) / BN;

    // staging: thread loads rows tid/16 + SROWS i (i < SIT), chunk tid%16.  Named u32x4 registers and
    // UNCONDITIONAL loads (tile index clamped to the last tile, key clamped to the last row of the
    // sequence; such rows are masked out of the scores and V rows stay finite) -- a conditional prefetch
    // made hipcc serialise the loop on vmcnt(0).
    const int st_chunk = tid & 15, st_row0 = tid >> 4;
    u32x4 kreg[SIT], vreg[SIT];
    // fp8 slab staging: row tid / 8 (0..63) of the slab, 16-B chunk tid % 8; one round per tile
    const int r8 = tid >> 3, c8 = tid & 7;
    float ks8 = 1.f, vs8 = 1.f;
    constexpr bool K8 = (KVM & 1) != 0, V8 = (KVM & 2) != 0;
    static_assert(KVM == 0 || NTHR / 8 == BN, "fp8 slab staging: one slab row per 8 threads");
#define LOAD_TILE(t)                                                                              \
    if constexpr (PAGED && KVM != 0) {                                                            \
        const size_t sb = kv8::slab_off(btab[t], Hkv, kvh);                                       \
        const size_t pg = (size_t)btab[t] * Hkv * BN * D + head_pg + st_chunk * 8;                \
        if constexpr (K8) {                                                                       \
            const unsigned char* kb_ = reinterpret_cast<const unsigned char*>(pk.kc) + sb;       \
            kreg[0] = *reinterpret_cast<const u32x4*>(kb_ + r8 * D + 16 * c8);                    \
            ks8 = *reinterpret_cast<const float*>(kb_ + BN * D + 4 * r8);                         \
        } else {                                                                                  \
            _Pragma("unroll") for (int i = 0; i < SIT; ++i)                                         \
                kreg[i] = *reinterpret_cast<const u32x4*>(pk.kc + pg + (size_t)(st_row0 + SROWS * i) * D); \
        }                                                                                         \
        if constexpr (V8) {                                                                       \
            const unsigned char* vb_ = reinterpret_cast<const unsigned char*>(pk.vc) + sb;       \
            vreg[0] = *reinterpret_cast<const u32x4*>(vb_ + r8 * D + 16 * c8);                    \
            vs8 = *reinterpret_cast<const float*>(vb_ + BN * D + 4 * r8);                         \
        } else {                                                                                  \
            _Pragma("unroll") for (int i = 0; i < SIT; ++i)                                         \
                vreg[i] = *reinterpret_cast<const u32x4*>(pk.vc + pg + (size_t)(st_row0 + SROWS * i) * D); \
        }                                                                                         \
    } else if constexpr (PAGED) {                                                                 \
        const size_t pg = (size_t)btab[t] * Hkv * BN * D + head_pg + st_chunk * 8;                \
        _Pragma("unroll") for (int i = 0; i < SIT; ++i) {                                           \
            kreg[i] = *reinterpret_cast<const u32x4*>(pk.kc + pg + (size_t)(st_row0 + SROWS * i) * D); \
            vreg[i] = *reinterpret_cast<const u32x4*>(pk.vc + pg + (size_t)(st_row0 + SROWS * i) * D); \
        }                                                                                         \
    } else {                                                                                      \
        _Pragma("unroll") for (int i = 0; i < SIT; ++i) {                                           \
            const int key = min((t) * BN + st_row0 + SROWS * i, len - 1);                           \
            const bf16* p = base + (size_t)key * row_stride + st_chunk * 8;                      \
            kreg[i] = *reinterpret_cast<const u32x4*>(p + kcol);                                 \
            vreg[i] = *reinterpret_cast<const u32x4*>(p + vcol);                                 \
        }                                                                                         \
    }
#define STORE_TILE(st)                                                                            \
    if constexpr (KVM != 0) {                                                                     \
        u32x4 lo_, hi_;                                                                           \
        if constexpr (K8) {                                                                       \
            kv8::dequant16(kreg[0], ks8, lo_, hi_);                                               \
            *reinterpret_cast<u32x4*>(lds + (st) + k_off(r8, 2 * c8)) = lo_;                      \
            *reinterpret_cast<u32x4*>(lds + (st) + k_off(r8, 2 * c8 + 1)) = hi_;                  \
        } else {                                                                                  \
            _Pragma("unroll") for (int i = 0; i < SIT; ++i)                                         \
                *reinterpret_cast<u32x4*>(lds + (st) + k_off(st_row0 + SROWS * i, st_chunk)) = kreg[i]; \
        }                                                                                         \
        if constexpr (V8) {                                                                       \
            kv8::dequant16(vreg[0], vs8, lo_, hi_);                                               \
            *reinterpret_cast<u32x4*>(lds + (st) + BN * 256 + v_off(r8, 2 * c8)) = lo_;           \
            *reinterpret_cast<u32x4*>(lds + (st) + BN * 256 + v_off(r8, 2 * c8 + 1)) = hi_;       \
        } else {                                                                                  \
            _Pragma("unroll") for (int i = 0; i < SIT; ++i)                                         \
                *reinterpret_cast<u32x4*>(lds + (st) + BN * 256 + v_off(st_row0 + SROWS * i, st_chunk)) = vreg[i]; \
        }                                                                                         \
    } else                                                                                        \
    _Pragma("unroll") for (int i = 0; i < SIT; ++i) {                                               \
        const int row = st_row0 + SROWS * i;                                                         \
        *reinterpret_cast<u32x4*>(lds + (st) + k_off(row, st_chunk)) = kreg[i];                    \
        *reinterpret_cast<u32x4*>(lds + (st) + BN * 256 + v_off(row, st_chunk)) = vreg[i];         \
    }

    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16{};
    float m = -INFINITY, l = 0.f;

    LOAD_TILE(0);
    STORE_TILE(0);
    LOAD_TILE(min(1, ntiles - 1));

    const int wave_last_q = pre + q0 + 31;  // absolute position of the wave's last row
    // PV operand addressing (loop-invariant parts): lane (g, q4, p4) reads V rows 4(g>>1) + q4 (+8) of each
    // 16-key slab at columns dt*32 + 16(g&1) + 4p4
    const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
    // (A GEMM-style stagger -- waves 4-7 half a tile behind waves 0-3, two barriers per tile, so one
    // wave's QK^T runs beside its partner's softmax + P.V -- measured 3-7 % slower than this one-barrier
    // loop, as did raising waves 0-3's priority: profiles/r3_attn_prefill_stagger_ab.jsonl.  A T15 software
    // pipeline -- QK^T of tile t+1 in one scheduling region with tile t's exponentials, P.V(t) beside tile
    // t+1's mask + max, three-stage ring, 246 VGPRs -- measured 7-9 % slower on every shape:
    // profiles/r3_attn_prefill_pipelined_experiment.jsonl.  Issuing tile 1's and Q's loads with tile 0's
    // (one exposed memory latency in the prologue instead of two) measured neutral to -1 %:
    // profiles/r3_attn_prefill_prologue_experiment.jsonl.)
    for (int t = 0; t < ntiles; ++t) {
        const int cur = (t & 1) * STAGE;
        const int kv0 = t * BN;
        const bool act = kv0 <= wave_last_q;  // wave-uniform: tiles wholly above the diagonal are skipped
        __syncthreads();  // tile t visible in stage t&1; every wave is done with tile t-1 (stage (t+1)&1)
        STORE_TILE(STAGE - cur);
        LOAD_TILE(min(t + 2, ntiles - 1));
        const char* ldsK = lds + cur;
        const char* ldsV = ldsK + BN * 256;
        if (!act) continue;
        // S^T = K Q^T: all 16 K fragments read up front (64 VGPRs, dead after the QK^T MFMAs), so the
        // ds_reads run ahead of the MFMA chain instead of one exposed LDS round trip per MFMA
        uint4 kf[2][8];
        f32x16 sacc[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
                kf[kt][ks] = *reinterpret_cast<const uint4*>(ldsK + k_off(kt * 32 + r32, 2 * ks + half));
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            sacc[kt] = f32x16{};
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
                sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kf[kt][ks]), qf[ks], sacc[kt], 0, 0, 0);
        }
        // schedule (cdna_hip_programming.md T19): 8 reads ahead, then one read per MFMA gap -- without it the
        // machine scheduler sinks every read next to its MFMA and waits lgkmcnt(0) before each one
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        // mask + row max (key index of reg i: kt*32 + (i&3) + 8(i>>2) + 4half).  The causal/length mask is
        // only needed on tiles that reach past the wave's first query row or the sequence end (wave-uniform
        // test); scores stay unscaled until the exponent, which is one FMA: p = 2^(s * scale_log2 - m), with
        // the raw v_exp_f32.
        const int kmax = pre + min(qi, len - 1) - kv0 - 4 * half;  // last valid key offset for row qi
        if (kv0 + BN - 1 > pre + q0 || kv0 + BN > pre + len) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int koff = kt * 32 + (i & 3) + 8 * (i >> 2);  // key - kv0 - 4*half
                    sacc[kt][i] = koff <= kmax ? sacc[kt][i] : -INFINITY;
                }
        }
        float mt = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sacc[kt][i]);
        mt = halves_max(mt);
        // deferred rescale (cdna_hip_programming.md T13): the running max m only moves (and o, l are
        // rescaled) when some row's max grew by more than RESCALE_LOG2 -- until then p <= 2^RESCALE_LOG2,
        // harmless in fp32 and in the bf16 P operand.  The previous tile's P.V is complete (program order)
        // and this tile's P is exponentiated after the decision.  Key 0 is valid for every row, so m is
        // finite after tile 0.
        const float mc = mt * scale_log2;
        if (__ballot(mc > m + RESCALE_LOG2)) {
            const float mn = fmaxf(m, mc);
            const float alpha = __builtin_amdgcn_exp2f(m - mn);  // m = -inf before tile 0 -> 0
            m = mn;
            l *= alpha;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
        }
        float ls = 0.f;
        bf16x8 pf[2][2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float p = __builtin_amdgcn_exp2f(fmaf(sacc[kt][i], scale_log2, -m));
                ls += p;
                pf[kt][i >> 3][i & 7] = (bf16)p;
            }
        }
        l += ls;
        // O^T[d][q] += V^T[d][key] P^T[key][q]: per 32-dim block dt, its 8 transposed reads, then 4 MFMAs
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const int col = dt * 32 + 16 * (g & 1) + 4 * p4;  // this lane's address column
            const int chunk = col >> 3, inoff = (col & 7) * 2;
            v8s va[2][2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const int rowa = kt * 32 + 16 * s + 4 * (g >> 1) + q4;
                    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(ldsV + v_off(rowa, chunk) + inoff));
                    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(ldsV + v_off(rowa + 8, chunk) + inoff));
                    va[kt][s] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int s = 0; s < 2; ++s)
                    o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, va[kt][s]), pf[kt][s],
                                                                    o[dt], 0, 0, 0);
        }
        // 8 transposed reads ahead, two per MFMA gap after that
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 1);
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 1);
    }
#undef LOAD_TILE
#undef STORE_TILE

    // normalise and store.  Reg i of tile dt holds d = dt*32 + (i&3) + 8(i>>2) + 4half for query qi; one
    // v_permlane32_swap per dword pair regroups two 4-dim groups so every lane stores 16 contiguous bytes
    // (cdna_hip_programming.md T21): lane < 32 dims 16j..16j+7, lane >= 32 dims 16j+8..16j+15 of row qi.
    const float lt = halves_sum(l);
    const float inv = 1.f / lt;
    uint4 ov[4][2];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // groups g4 = 2j, 2j+1 of this 32-dim block
            const uint32_t a0 = pack2(o[dt][8 * j + 0] * inv, o[dt][8 * j + 1] * inv);
            const uint32_t a1 = pack2(o[dt][8 * j + 2] * inv, o[dt][8 * j + 3] * inv);
            const uint32_t b0 = pack2(o[dt][8 * j + 4] * inv, o[dt][8 * j + 5] * inv);
            const uint32_t b1 = pack2(o[dt][8 * j + 6] * inv, o[dt][8 * j + 7] * inv);
            const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
            const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
            ov[dt][j] = make_uint4(r0[0], r1[0], r0[1], r1[1]);
        }
    }
    if (qi < len) {
        bf16* op = out + (size_t)(s0 + qi) * out_stride + h * D + 8 * half;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int j = 0; j < 2; ++j) *reinterpret_cast<uint4*>(op + dt * 32 + 16 * j) = ov[dt][j];
    }
}

template <bool PAGED, int G>
static void launch_g(dim3 grid, hipStream_t s, const bf16* Q, int row_stride, const int* cu, const int2* it, bf16* out,
                     int out_stride, int Hq, int Hkv, int Hg, int gq, float sl, const PagedKV& p, int kv8) {
    // kv-head-major order from 8 blocks per CU up (measured crossover: 4096 blocks neutral, 19656 kv-major)
    const int kv_major = grid.x > 8 * 256;
    if constexpr (PAGED) {
        if (kv8 == 3 || kv8 == 2) {
            if (kv8 == 3)
                attn_prefill_kernel<PAGED, G, 3><<<grid, NTHR, 0, s>>>(Q, row_stride, cu, it, out, out_stride, Hq,
                                                                       Hkv, Hg, gq, sl, p, kv_major);
            else
                attn_prefill_kernel<PAGED, G, 2><<<grid, NTHR, 0, s>>>(Q, row_stride, cu, it, out, out_stride, Hq,
                                                                       Hkv, Hg, gq, sl, p, kv_major);
            return;
        }
    }
    attn_prefill_kernel<PAGED, G, 0><<<grid, NTHR, 0, s>>>(Q, row_stride, cu, it, out, out_stride, Hq, Hkv, Hg,
                                                                   gq, sl, p, kv_major);
}

static bool packed_ratio(int G) { return G == 1 || G == 2 || G == 4 || G == 8; }

// Query positions per workgroup for a GQA ratio (the host's work list must use the same block size):
// 256 / G for the packed ratios, 256 for the per-query-head fallback of any other ratio.
MRSUM_API int mrsum_attn_prefill_block_m(int Hq, int Hkv) {
    if (Hkv <= 0 || Hq % Hkv || Hq / Hkv > 64) return -1;
    const int G = Hq / Hkv;
    return packed_ratio(G) ? 32 * (NW / G) : 32 * NW;
}

static int launch_prefill(const void* qkv, int row_stride, const int* cu_seqlens, const int* items, int n_items,
                          int block_m, void* out, int out_stride, int Hq, int Hkv, int Dh, float scale,
                          const PagedKV* pk, int kv8, hipStream_t s) {
    if (n_items <= 0) return 0;
    if (Dh != D || mrsum_attn_prefill_block_m(Hq, Hkv) != block_m) return (int)hipErrorInvalidValue;
    const int G = Hq / Hkv;
    const int Hg = packed_ratio(G) ? Hkv : Hq;  // head groups per work item (see the kernel's header)
    const int gq = packed_ratio(G) ? 1 : G;
    dim3 grid(n_items * Hg);
    const float sl = scale * 1.4426950408889634f;
    auto Q = (const bf16*)qkv;
    auto IT = (const int2*)items;
    auto O = (bf16*)out;
    const PagedKV p = pk ? *pk : PagedKV{nullptr, nullptr, nullptr, 0, nullptr, nullptr};
#define DISPATCH(PG)                                                                                                 \
    switch (packed_ratio(G) ? G : 1) {                                                                               \
        case 1: launch_g<PG, 1>(grid, s, Q, row_stride, cu_seqlens, IT, O, out_stride, Hq, Hkv, Hg, gq, sl, p, kv8); break; \
        case 2: launch_g<PG, 2>(grid, s, Q, row_stride, cu_seqlens, IT, O, out_stride, Hq, Hkv, Hg, gq, sl, p, kv8); break; \
        case 4: launch_g<PG, 4>(grid, s, Q, row_stride, cu_seqlens, IT, O, out_stride, Hq, Hkv, Hg, gq, sl, p, kv8); break; \
        default: launch_g<PG, 8>(grid, s, Q, row_stride, cu_seqlens, IT, O, out_stride, Hq, Hkv, Hg, gq, sl, p, kv8); break; \
    }
    if (pk) { DISPATCH(true) } else { DISPATCH(false) }
#undef DISPATCH
    return (int)hipGetLastError();
}

// items: (sequence, first query row) pairs of block_m = mrsum_attn_prefill_block_m(Hq, Hkv) rows each.
MRSUM_API int mrsum_attn_prefill(const void* qkv, int row_stride, const int* cu_seqlens, const int* items,
                                 int n_items, int block_m, void* out, int out_stride, int Hq, int Hkv, int Dh,
                                 float scale, hipStream_t s) {
    return launch_prefill(qkv, row_stride, cu_seqlens, items, n_items, block_m, out, out_stride, Hq, Hkv, Dh, scale,
                          nullptr, 0, s);
}

// Chunked-prefill attention: q rows of the packed slices (qkv, cu_seqlens), keys / values from the paged
// cache for absolute positions [0, prefix[seq] + slice length) of every sequence (page size 64).
MRSUM_API int mrsum_attn_prefill_paged(const void* qkv, int row_stride, const int* cu_seqlens, const int* items,
                                       int n_items, int block_m, void* out, int out_stride, int Hq, int Hkv, int Dh,
                                       float scale, const void* kcache, const void* vcache, const int* block_tables,
                                       int bt_stride, const int* seq_slot, const int* prefix, int kv8, hipStream_t s) {
    if (!kcache || !vcache || !block_tables || !seq_slot || !prefix || (kv8 != 0 && kv8 != 2 && kv8 != 3))
        return (int)hipErrorInvalidValue;  // an fp8 K with a bf16 V cache is not a layout the engine makes
    const PagedKV pk{(const bf16*)kcache, (const bf16*)vcache, block_tables, bt_stride, seq_slot, prefix};
    return launch_prefill(qkv, row_stride, cu_seqlens, items, n_items, block_m, out, out_stride, Hq, Hkv, Dh, scale,
                          &pk, kv8, s);
}
