// Causal varlen flash attention for prefill on MFMA.
//
// Packed batch: qkv [T, row_stride] bf16 (Q heads, then K heads, then V
// heads, D=128 each, already rotated by rope_kv), cu_seqlens [nseq+1].
// Work item = (sequence, 256-row query block) x query head; items are listed
// by the host heaviest-first (causal blocks late in a sequence do the most
// key tiles), blockIdx.y = query head.
//
// Workgroup: 8 waves (one per CU, 2 per SIMD at 209 VGPRs), wave w owns query rows [32w, 32w+32) of
// the block: every staged K/V tile serves 256 query rows (8 x 4000-token / 32k prompts: +4-6 % over two
// 4-wave 128-row workgroups per CU; 8 x 4096: -2 %, profiles/r2_attn_prefill_8wave_256rows_ab.jsonl).
// Per 64-key tile (K and V staged through LDS, next tile prefetched into
// registers while the current one is consumed - issue early / write late):
//
//   S^T = K . Q^T   v_mfma_f32_32x32x16_bf16, A = K rows from LDS
//                   (ds_read_b128, 16-B chunks XOR-swizzled by row&15 so a
//                   16-lane group hits 16 distinct slots), B = Q^T fragments
//                   held in VGPRs for the whole loop.  The "swapped" product
//                   puts one query row per lane (col = lane&31), so the row
//                   max is 31 in-lane fmax + one xor-32 shuffle.
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
// Numerics: bf16 inputs, fp32 accumulation and softmax, bf16 output.
#include "common.h"

namespace {
constexpr int D = 128;
constexpr int NW = 8;            // waves per workgroup (32 query rows each)
constexpr int BM = 32 * NW;      // query rows per workgroup
constexpr int NTHR = 64 * NW;
constexpr int SROWS = NTHR / 16;  // tile rows staged per load round (16 lanes x 16 B per 256-B row)
constexpr int BN = 64;   // keys per tile
constexpr int SIT = BN / SROWS;   // load rounds per 64-row tile
constexpr float RESCALE_LOG2 = 8.0f;  // deferred-rescale threshold (log2 units), see the softmax

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

__device__ __forceinline__ int k_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }
__device__ __forceinline__ int v_off(int row, int chunk) { return row * 256 + ((chunk ^ ((row & 3) << 2)) << 4); }

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
}  // namespace

struct PagedKV {
    const bf16* kc;            // [pages, Hkv, 64, D]
    const bf16* vc;
    const int* block_tables;   // [slots, bt_stride]
    int bt_stride;
    const int* seq_slot;       // [nseq] decode slot (block-table row) of every packed sequence
    const int* prefix;         // [nseq] tokens already cached before this slice
};

template <bool PAGED>
__global__ __launch_bounds__(NTHR, 1) void attn_prefill_kernel(const bf16* __restrict__ qkv, int row_stride,
                                                              const int* __restrict__ cu_seqlens,
                                                              const int2* __restrict__ items,
                                                              bf16* __restrict__ out, int out_stride, int Hq,
                                                              int Hkv, float scale_log2, PagedKV pk) {
    // one stage of [K tile | V tile]; a 2-stage ring with one barrier per tile measured 2-4 % slower
    // (its tile writes land between other waves' tile reads instead of behind a barrier)
    __shared__ __attribute__((aligned(16))) char lds[1][2 * BN * 256];

    const int2 it = items[blockIdx.x];
    const int seq = it.x, qblock = it.y;
    const int h = blockIdx.y, kvh = h / (Hq / Hkv);
    const int s0 = cu_seqlens[seq], len = cu_seqlens[seq + 1] - s0;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5, r32 = lane & 31;
    const bf16* base = qkv + (size_t)s0 * row_stride;
    const int kcol = (Hq + kvh) * D, vcol = (Hq + Hkv + kvh) * D;
    // keys live at absolute positions [0, pre + len); query row qi at pre + qi
    const int pre = PAGED ? pk.prefix[seq] : 0;
    const int* btab = PAGED ? pk.block_tables + (size_t)pk.seq_slot[seq] * pk.bt_stride : nullptr;
    const size_t head_pg = (size_t)kvh * BN * D;  // this kv head's 64-row slab inside a page

    // Q^T fragments: lane holds Q[row r32][dims 16ks + 8half .. +8] for ks = 0..7
    const int qi = qblock + 32 * w + r32;
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

    const int kend = pre + min(len, qblock + BM);
    const int ntiles = (kend + BN - 1) / BN;

    // staging: thread loads rows tid/16 + SROWS i (i < SIT), chunk tid%16.  Named u32x4 registers and
    // UNCONDITIONAL loads (key clamped to the last row of the sequence; such rows are masked out of
    // the scores, and V rows stay finite) -- a conditional or lambda-captured prefetch made hipcc
    // serialise the loop on vmcnt(0).
    const int st_chunk = tid & 15, st_row0 = tid >> 4;
    u32x4 kreg[SIT], vreg[SIT];
#define LOAD_TILE(t)                                                                              \
    if constexpr (PAGED) {                                                                        \
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
#define STORE_TILE(stage)                                                                         \
    _Pragma("unroll") for (int i = 0; i < SIT; ++i) {                                               \
        const int row = st_row0 + SROWS * i;                                                         \
        *reinterpret_cast<u32x4*>(lds[stage] + k_off(row, st_chunk)) = kreg[i];                  \
        *reinterpret_cast<u32x4*>(lds[stage] + BN * 256 + v_off(row, st_chunk)) = vreg[i];       \
    }

    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16{};
    float m = -INFINITY, l = 0.f;

    LOAD_TILE(0);
    STORE_TILE(0);
    __syncthreads();

    const int wave_last_q = pre + qblock + 32 * w + 31;  // absolute position of the wave's last row
    const char* ldsK = lds[0];
    const char* ldsV = ldsK + BN * 256;
    for (int t = 0; t < ntiles; ++t) {
        LOAD_TILE(min(t + 1, ntiles - 1));
        const int kv0 = t * BN;
        if (kv0 <= wave_last_q) {  // wave-uniform: tiles wholly above the diagonal are skipped
            f32x16 sacc[2];
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                sacc[kt] = f32x16{};
                const int row = kt * 32 + r32;
#pragma unroll
                for (int ks = 0; ks < 8; ++ks) {
                    const uint4 kv = *reinterpret_cast<const uint4*>(ldsK + k_off(row, 2 * ks + half));
                    sacc[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(kv), qf[ks], sacc[kt], 0, 0, 0);
                }
            }
            // mask + row max (key index of reg i: kt*32 + (i&3) + 8(i>>2) + 4half).  The causal/length
            // mask is only needed on tiles that reach past the wave's first query row or the sequence
            // end (wave-uniform test); scores stay unscaled until the exponent, which is one FMA:
            // p = 2^(s * scale_log2 - m), with the raw v_exp_f32 (no denormal range reduction: the
            // library exp2f costs 4 extra VALU ops per score).
            const int kmax = pre + min(qi, len - 1) - kv0 - 4 * half;  // last valid key offset for row qi
            if (kv0 + BN - 1 > pre + qblock + 32 * w || kv0 + BN > pre + len) {
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
            mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
            // deferred rescale: the running max m only moves (and o, l are rescaled) when some row's
            // max grew by more than RESCALE_LOG2 -- until then p <= 2^RESCALE_LOG2, harmless in fp32
            // and in the bf16 P operand.  Key 0 is valid for every row, so m is finite after tile 0.
            // (PAGED: rows past the slice end see keys up to pre + len - 1 only; stale page rows past
            // that are masked like any key beyond the causal limit.)
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
            // O^T[d][q] += V^T[d][key] P^T[key][q]
            const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int col = dt * 32 + 16 * (g & 1) + 4 * p4;  // this lane's address column
                const int chunk = col >> 3, inoff = (col & 7) * 2;
#pragma unroll
                for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        const int rowa = kt * 32 + 16 * s + 4 * (g >> 1) + q4;
                        const int rowb = rowa + 8;
                        const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_v4s*)(ldsV + v_off(rowa, chunk) + inoff));
                        const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                            (lds_v4s*)(ldsV + v_off(rowb, chunk) + inoff));
                        typedef short v8s __attribute__((ext_vector_type(8)));
                        const v8s a = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), pf[kt][s],
                                                                        o[dt], 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();
        if (t + 1 < ntiles) {
            STORE_TILE(0);
            __syncthreads();
        }
    }
#undef LOAD_TILE
#undef STORE_TILE

    // normalise and store: reg i of tile dt holds d = dt*32 + (i&3) + 8(i>>2) + 4half for query qi
    const float lt = l + __shfl_xor(l, 32, 64);
    if (qi < len) {
        const float inv = 1.f / lt;
        bf16* op = out + (size_t)(s0 + qi) * out_stride + h * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int d = dt * 32 + 8 * g4 + 4 * half;
                uint2 v;
                v.x = pack2(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
                v.y = pack2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
                *reinterpret_cast<uint2*>(op + d) = v;
            }
        }
    }
}

static int launch_prefill(const void* qkv, int row_stride, const int* cu_seqlens, const int* items, int n_items,
                          void* out, int out_stride, int Hq, int Hkv, int Dh, float scale, const PagedKV* pk,
                          hipStream_t s) {
    if (n_items <= 0) return 0;
    if (Dh != D || Hq % Hkv) return (int)hipErrorInvalidValue;
    dim3 grid(n_items, Hq), block(NTHR);
    const float sl = scale * 1.4426950408889634f;
    auto Q = (const bf16*)qkv;
    auto IT = (const int2*)items;
    const PagedKV p = pk ? *pk : PagedKV{nullptr, nullptr, nullptr, 0, nullptr, nullptr};
    if (pk) attn_prefill_kernel<true><<<grid, block, 0, s>>>(Q, row_stride, cu_seqlens, IT, (bf16*)out, out_stride, Hq, Hkv, sl, p);
    else attn_prefill_kernel<false><<<grid, block, 0, s>>>(Q, row_stride, cu_seqlens, IT, (bf16*)out, out_stride, Hq, Hkv, sl, p);
    return (int)hipGetLastError();
}

MRSUM_API int mrsum_attn_prefill(const void* qkv, int row_stride, const int* cu_seqlens, const int* items,
                                 int n_items, void* out, int out_stride, int Hq, int Hkv, int Dh, float scale,
                                 hipStream_t s) {
    return launch_prefill(qkv, row_stride, cu_seqlens, items, n_items, out, out_stride, Hq, Hkv, Dh, scale, nullptr, s);
}

// Chunked-prefill attention: q rows of the packed slices (qkv, cu_seqlens), keys / values from the paged
// cache for absolute positions [0, prefix[seq] + slice length) of every sequence (page size 64).
MRSUM_API int mrsum_attn_prefill_paged(const void* qkv, int row_stride, const int* cu_seqlens, const int* items,
                                       int n_items, void* out, int out_stride, int Hq, int Hkv, int Dh, float scale,
                                       const void* kcache, const void* vcache, const int* block_tables,
                                       int bt_stride, const int* seq_slot, const int* prefix, hipStream_t s) {
    if (!kcache || !vcache || !block_tables || !seq_slot || !prefix) return (int)hipErrorInvalidValue;
    const PagedKV pk{(const bf16*)kcache, (const bf16*)vcache, block_tables, bt_stride, seq_slot, prefix};
    return launch_prefill(qkv, row_stride, cu_seqlens, items, n_items, out, out_stride, Hq, Hkv, Dh, scale, &pk, s);
}
