// Rotary embedding on Q and K fused with the paged KV-cache write
// (SURVEY.md §2.6 K6).
//
// qkv      [T, row_stride] bf16: per token [Hq*D | Hkv*D | Hkv*D]; Q and K are
//          rotated IN PLACE (prefill attention reads them back from here),
//          rotated K and raw V are also scattered into the paged cache.
// positions[T] int32, seq_idx[T] int32 (row of block_tables for the token; < 0: not cached),
// block_tables [*, bt_stride] int32 page ids,
// cache    K and V: [num_pages, Hkv, P, D] bf16 (one page = P consecutive
//          positions of one kv head: 16 KiB at P=64, D=128, so a decode
//          workgroup streams whole contiguous pages).
// cos_sin  [max_pos, D/2] float2 (cos, sin), HF "rotate_half" pairing
//          (i, i + D/2), precomputed on the host (no device trig).
//
// One 256-thread block per token; a work item is 8 rotary pairs of one head
// (two 16-B loads, two 16-B stores) or 16 dims of one V head (two 16-B vectors): 8 items per
// head for K and for V, so the 8 lanes of a head's row sit together (fp8 row scale below).
//
// FP8 KV cache (KV8): the cache is byte slabs [num_pages, Hkv, SLAB], SLAB = P * D + 4 * P (kv8.h):
// row r of a (page, head) slab is D OCP e4m3fn bytes at r * D, its fp32 scale at P * D + 4 r.  A
// row is quantised as a whole (rotated K, raw V): scale = the power of two >= max|x| / 448 (the
// 8 lanes of the row reduce the max with xor shuffles), q = e4m3(x / scale).  Power-of-two scales
// make the decode-side dequantisation (cvt_scalef32 to bf16) exact.  KVM is a bitmask: bit 0 = the K
// cache is fp8 slabs, bit 1 = the V cache is (KVM 2, "fp8v": bf16 K, fp8 V -- K rounding is what peaked
// attention amplifies, profiles/r4_fp8_kv_emulation.txt).
#include "kv8.h"

// Source of one token row: the bf16 qkv row itself, or (PARTS) the sum of S
// fp32 split-K slabs of the decode QKV GEMM -- the GEMM's split-K reduction
// is folded into this pass.
template <bool PARTS>
struct RowSrc {
    const bf16* row;     // !PARTS
    const float* parts;  // PARTS: slab 0 row start; slab s at + s * slab_stride
    size_t slab_stride;
    int S;
    __device__ __forceinline__ void load8(int col, float* f) const {
        if constexpr (!PARTS) {
            unpack8(*reinterpret_cast<const uint4*>(row + col), f);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = 0.f;
            // slabs in batches of 4 with every load of a batch issued before the first add: a plain
            // runtime-S loop waits one L2 round trip per slab
            for (int s0 = 0; s0 < S; s0 += 4) {
                float4 a[4], b[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4* p = reinterpret_cast<const float4*>(parts + min(s0 + u, S - 1) * slab_stride + col);
                    a[u] = p[0];
                    b[u] = p[1];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (s0 + u < S) {
                        f[0] += a[u].x; f[1] += a[u].y; f[2] += a[u].z; f[3] += a[u].w;
                        f[4] += b[u].x; f[5] += b[u].y; f[6] += b[u].z; f[7] += b[u].w;
                    }
                }
            }
        }
    }
};

template <int D, bool PARTS, int KVM>
__global__ __launch_bounds__(256) void rope_kv_kernel(const bf16* __restrict__ qkv_in, const float* __restrict__ parts,
                                                      int S, int T, bf16* __restrict__ qkv_out, int row_stride,
                                                      const int* __restrict__ positions,
                                                      const int* __restrict__ seq_idx,
                                                      const int* __restrict__ block_tables, int bt_stride,
                                                      bf16* __restrict__ kcache, bf16* __restrict__ vcache,
                                                      const float2* __restrict__ cos_sin, int Hq, int Hkv,
                                                      int P, int write_cache) {
    constexpr int HALF = D / 2;
    constexpr int RI = HALF / 8;   // rotation items per head
    constexpr int VI = D / 16;     // copy items per v head (16 dims each)
    static_assert(RI == VI, "K and V rows must take the same number of lanes");
    const int t = blockIdx.x;  // blockIdx.y: 256-item slice of the token's work (one item per thread)
    const int pos = positions[t];
    const int width = (Hq + 2 * Hkv) * D;
    RowSrc<PARTS> src;
    if constexpr (PARTS) {
        src.parts = parts + (size_t)t * width;
        src.slab_stride = (size_t)T * width;
        src.S = S;
    } else {
        src.row = qkv_in + (size_t)t * row_stride;
    }
    bf16* row = qkv_out + (size_t)t * row_stride;
    size_t page_base = 0;
    // seq_idx < 0: a padding token of the prefill batch (engine._prefill) -- rotated, never cached
    write_cache = write_cache && seq_idx[t] >= 0;
    int page = 0;
    if (write_cache) {
        page = block_tables[(size_t)seq_idx[t] * bt_stride + pos / P];
        page_base = (size_t)page * Hkv * P + (pos % P);
    }
    const float2* cs = cos_sin + (size_t)pos * HALF;
    const int n_rot = (Hq + Hkv) * RI;
    const int n_all = n_rot + Hkv * VI;
    for (int it = blockIdx.y * blockDim.x + threadIdx.x; it < n_all; it += blockDim.x * gridDim.y) {
        if (it < n_rot) {
            const int h = it / RI, c = (it % RI) * 8;
            float a[8], b[8];
            src.load8(h * D + c, a);
            src.load8(h * D + c + HALF, b);
            float ra[8], rb[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float2 e = cs[c + j];
                ra[j] = a[j] * e.x - b[j] * e.y;
                rb[j] = b[j] * e.x + a[j] * e.y;
            }
            const uint4 pa = pack8(ra), pb = pack8(rb);
            bf16* hp = row + h * D;
            *reinterpret_cast<uint4*>(hp + c) = pa;
            *reinterpret_cast<uint4*>(hp + c + HALF) = pb;
            if constexpr ((KVM & 1) != 0) {
                if (h >= Hq) {  // head-uniform over the row's RI lanes: the shuffles stay inside the row
                    float f[16];
                    unpack8(pa, f);
                    unpack8(pb, f + 8);
                    kv8::put_row16(kcache, page, Hkv, h - Hq, pos % P, P, D, c, c + HALF, f, write_cache);
                }
            } else if (write_cache && h >= Hq) {
                bf16* kp = kcache + (page_base + (size_t)(h - Hq) * P) * D;
                *reinterpret_cast<uint4*>(kp + c) = pa;
                *reinterpret_cast<uint4*>(kp + c + HALF) = pb;
            }
        } else {
            const int i = it - n_rot;
            const int h = i / VI, c = (i % VI) * 16;
            const int col = (Hq + Hkv + h) * D + c;
            uint4 v[2];
            if constexpr (PARTS) {
                float f[8];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    src.load8(col + 8 * u, f);
                    v[u] = pack8(f);
                    *reinterpret_cast<uint4*>(row + col + 8 * u) = v[u];
                }
            } else {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    v[u] = *reinterpret_cast<const uint4*>(src.row + col + 8 * u);
                    if (qkv_out != qkv_in) *reinterpret_cast<uint4*>(row + col + 8 * u) = v[u];
                }
            }
            if constexpr ((KVM & 2) != 0) {
                float f[16];
                unpack8(v[0], f);
                unpack8(v[1], f + 8);
                kv8::put_row16(vcache, page, Hkv, h, pos % P, P, D, c, c + 8, f, write_cache);
            } else if (write_cache) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    *reinterpret_cast<uint4*>(vcache + (page_base + (size_t)h * P) * D + c + 8 * u) = v[u];
            }
        }
    }
}

template <bool PARTS>
static int launch_rope(const void* qkv_in, const void* parts, int S, void* qkv_out, int T, int row_stride,
                       const int* positions, const int* seq_idx, const int* block_tables, int bt_stride,
                       void* kcache, void* vcache, const void* cos_sin, int Hq, int Hkv, int D, int P,
                       int write_cache, int kv8, hipStream_t s) {
    if (T <= 0) return 0;
    if (kv8 < 0 || kv8 > 3 || (kv8 && D != 128)) return (int)hipErrorInvalidValue;
    const int items = (Hq + 2 * Hkv) * (D / 16);
    dim3 g(T, ceil_div(items, 256)), b(256);
    auto QI = (const bf16*)qkv_in; auto PA = (const float*)parts; auto QO = (bf16*)qkv_out;
    auto K = (bf16*)kcache; auto V = (bf16*)vcache; auto CS = (const float2*)cos_sin;
#define RK(D_, M_) rope_kv_kernel<D_, PARTS, M_><<<g, b, 0, s>>>(QI, PA, S, T, QO, row_stride, positions, seq_idx, \
                                                                  block_tables, bt_stride, K, V, CS, Hq, Hkv, P, write_cache)
    if (kv8 == 3) RK(128, 3);
    else if (kv8 == 2) RK(128, 2);
    else if (kv8 == 1) RK(128, 1);
    else if (D == 128) RK(128, 0);
    else if (D == 64) RK(64, 0);
    else
        return (int)hipErrorInvalidValue;
#undef RK
    return (int)hipGetLastError();
}

// kv8: bit 0 the K cache, bit 1 the V cache is the fp8 byte-slab layout (kv8.h), else bf16 [pages, Hkv, P, D]
MRSUM_API int mrsum_rope_kv(void* qkv, int T, int row_stride, const int* positions, const int* seq_idx,
                            const int* block_tables, int bt_stride, void* kcache, void* vcache,
                            const void* cos_sin, int Hq, int Hkv, int D, int P, int write_cache, int kv8,
                            hipStream_t s) {
    return launch_rope<false>(qkv, nullptr, 1, qkv, T, row_stride, positions, seq_idx, block_tables, bt_stride,
                              kcache, vcache, cos_sin, Hq, Hkv, D, P, write_cache, kv8, s);
}

// parts: fp32 [S, T, (Hq+2Hkv)*D] split-K slabs; qkv_out: bf16 [T, row_stride]
MRSUM_API int mrsum_rope_kv_parts(const void* parts, int S, void* qkv_out, int T, int row_stride,
                                  const int* positions, const int* seq_idx, const int* block_tables, int bt_stride,
                                  void* kcache, void* vcache, const void* cos_sin, int Hq, int Hkv, int D, int P,
                                  int kv8, hipStream_t s) {
    if (S < 1) return (int)hipErrorInvalidValue;
    return launch_rope<true>(nullptr, parts, S, qkv_out, T, row_stride, positions, seq_idx, block_tables, bt_stride,
                             kcache, vcache, cos_sin, Hq, Hkv, D, P, 1, kv8, s);
}

// ---------------------------------------------------------------------------------------------
// K/V row scatter into the paged cache (context-parallel prefill, engine.prefill_export_cp): rows [n, 2, Hkv,
// D] bf16 (K then V of every kv head of one token, as all-gathered from the other ranks) -> kc / vc [pages,
// Hkv, P, D] at (page[i], slot[i]) for i < n; entries with page < 0 are skipped (all-gather padding).  One
// 256-thread block per 4 tokens x ... : a work item is one 16-B vector (8 dims) of one head's K or V row.
__global__ __launch_bounds__(256) void kv_scatter_kernel(const bf16* __restrict__ rows, int n, int Hkv, int D,
                                                         const int* __restrict__ page, const int* __restrict__ slot,
                                                         bf16* __restrict__ kc, bf16* __restrict__ vc, int P) {
    const int vec_per_tok = 2 * Hkv * (D / 8);
    const long total = (long)n * vec_per_tok;
    for (long it = (long)blockIdx.x * 256 + threadIdx.x; it < total; it += (long)gridDim.x * 256) {
        const int i = (int)(it / vec_per_tok), rem = (int)(it % vec_per_tok);
        const int kv = rem / (Hkv * (D / 8)), h = (rem / (D / 8)) % Hkv, c = rem % (D / 8);
        const int pg = page[i];
        if (pg < 0) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(rows + (((size_t)i * 2 + kv) * Hkv + h) * D + 8 * c);
        bf16* dst = (kv ? vc : kc) + (((size_t)pg * Hkv + h) * P + slot[i]) * D + 8 * c;
        *reinterpret_cast<uint4*>(dst) = v;
    }
}

MRSUM_API int mrsum_kv_scatter(const void* rows, int n, int Hkv, int D, const int* page, const int* slot, void* kc,
                               void* vc, int P, hipStream_t s) {
    if (n <= 0) return 0;
    if (D % 8 || Hkv < 1 || P < 1) return (int)hipErrorInvalidValue;
    const long vecs = (long)n * 2 * Hkv * (D / 8);
    const int grid = (int)std::min<long>((vecs + 255) / 256, 4096);
    kv_scatter_kernel<<<grid, 256, 0, s>>>((const bf16*)rows, n, Hkv, D, page, slot, (bf16*)kc, (bf16*)vc, P);
    return (int)hipGetLastError();
}
