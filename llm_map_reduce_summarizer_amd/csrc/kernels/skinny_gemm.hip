// Decode-shape GEMM on MFMA: out[M, N] = x[M, K] . W[N, K]^T with M <= 64
// (one row per decode sequence), W bf16 row-major (the nn.Linear layout).
//
// At decode batch sizes the op is a weight stream: every W byte is read
// exactly once per step and the whole step is bounded by HBM (15 GB of
// Llama-3-8B weights = 2.4 ms at 6.3 TB/s).  The kernel is built for that:
//
//  * swapped product  out^T[n, m] = W[n, :] . x[m, :]  on
//    v_mfma_f32_16x16x32_bf16: A = 16 W rows x 32 k (one 16-B load per lane
//    straight from HBM into the A fragment -- no LDS round trip for an operand
//    that is used once, cdna_hip_programming.md §5 "GEMV / M <= 16" row),
//    B = x^T fragments (x is tiny and stays in L2).
//  * workgroup = 4 waves over NT x 16 rows of W; the waves interleave over
//    128-wide k blocks (the workgroup reads 1 KiB contiguous per row per
//    round), next block's W loads issued before the current block's MFMAs
//    (two named register sets, no runtime-indexed arrays);
//  * optional split-K over S workgroups (grid.y) when N alone gives too few
//    workgroups for 256 CUs; partial slabs are fp32 and summed by the
//    CONSUMER kernel (add_rmsnorm_partials), not by atomics or an extra pass;
//  * fused epilogues: bf16 store | fp32 partial slab | SwiGLU (W rows laid
//    out as [8 gate | 8 up] blocks so one workgroup tile holds gate and up of
//    the same 8 features: act = silu(g) * u is written directly, the gate_up
//    activation never exists in HBM).
//  * deferred-RMSNorm operands (stream_gemm.hip header), one 16-row tile per workgroup, no split-K:
//    SWIGLU takes x = the un-normalised residual rows + the producer's per-tile sums of squares and
//    scales gate and up rows by rsqrt(mean(h^2) + eps) (the stream consumer's reduction order, so every
//    consumer of a row scales it by the same factor); RESID is a producer: residual += the tile (after
//    the TP push all-reduce when ``tp.world`` > 0, ar_common.h), per-tile row sums of squares to ssp.
//    A TP-shard row-parallel projection (K <= 2048) keeps this kernel's launch floor instead of the
//    stream kernel's ring ramp.
//    Progress of the TP push here: EVERY workgroup pushes its tile and then spins on its peers' copies
//    of the same tile (no split-K, so no "one spinner per tile" bound as in stream_gemm.hip).  A rank's
//    spinners wait only for tiles its peers' workgroups push BEFORE spinning, so the grid completes on
//    every rank iff each peer eventually dispatches every workgroup -- guaranteed when the whole grid is
//    resident at once (dispatch never waits for a spinner to retire).  The launcher therefore refuses a
//    TP-push grid larger than the device's resident capacity for this kernel (occupancy x CUs,
//    mrsum_skinny_resid_capacity; ops/__init__.py picks the stream producer then), and the 4 s wait bound
//    + the engine's collective reset / RCCL re-run (parallel/custom_ar.py) cover a stall anyway.
#include "ar_common.h"

namespace {
enum { EPI_BF16 = 0, EPI_F32_PARTIAL = 1, EPI_SWIGLU = 2, EPI_RESID = 3 };

struct SkinnyNorm {
    const float* ssq;  // SWIGLU consumer: [M][ssq_tiles] row sums of squares of x per producer tile (or null)
    int ssq_tiles;     // multiple of 32
    float inv_k, eps;
    bf16* resid;       // RESID producer: residual rows [M][ldr] (in / out)
    int ldr;
    float* ssp;        // RESID producer: [M][gridDim.x] row sums of squares of the new residual per tile
    mrsum_ar::TPPush tp;
};

// Deferred norm of row m, in stream_gemm.hip's order: partial p (< 8) of ssq_tiles / 8 consecutive tiles
// summed in float4 steps (thread 8 m + p; its loads issued in the kernel prologue, into registers, so they
// overlap the weight stream and nothing waits for them before the epilogue), then rsqrt(sum of the
// partials in order / K + eps).  ssq_tiles <= 32 * SS_C4.
constexpr int SS_C4 = 16;
struct SsLoads {
    float4 v[SS_C4];
};

__device__ __forceinline__ void deferred_issue(const SkinnyNorm& e, int m, int p, SsLoads& l) {
    const int C4 = e.ssq_tiles / 32;
    const float4* src = reinterpret_cast<const float4*>(e.ssq + (size_t)m * e.ssq_tiles) + p * C4;
#pragma unroll
    for (int q = 0; q < SS_C4; ++q) l.v[q] = q < C4 ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ float deferred_partial(const SsLoads& l) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < SS_C4; ++q) {
        a.x += l.v[q].x; a.y += l.v[q].y; a.z += l.v[q].z; a.w += l.v[q].w;
    }
    return (a.x + a.y) + (a.z + a.w);
}

__device__ __forceinline__ float deferred_row_scale(const SkinnyNorm& e, const float* s_part, int m) {
    float t = 0.f;
#pragma unroll
    for (int p = 0; p < 8; ++p) t += s_part[8 * m + p];
    return rsqrtf(t * e.inv_k + e.eps);
}
constexpr int KB = 128;  // k elements per wave round (4 MFMA k-steps of 32)

template <int NT>
struct AFrag {
    uint4 v[NT][4];
};

template <int NT>
__device__ __forceinline__ void load_a(AFrag<NT>& a, const bf16* __restrict__ W, int K, int n0, int kb, int lane) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const bf16* p = W + (size_t)(n0 + 16 * t + r) * K + kb + 8 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            a.v[t][i] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 32 * i)));
        }
    }
}

template <int MT>
struct BFrag {
    uint4 v[MT][4];
};

template <int MT>
__device__ __forceinline__ void load_b(BFrag<MT>& b, const bf16* __restrict__ x, int ldx, int M, int kb, int lane) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int row = min(16 * m + r, M - 1);
        const bf16* p = x + (size_t)row * ldx + kb + 8 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) b.v[m][i] = *reinterpret_cast<const uint4*>(p + 32 * i);
    }
}

// the per-wave partial sums of one output, waves in order (pairwise for 8, the 4-wave order unchanged)
template <int NW, typename R>
__device__ __forceinline__ float wsum(const R& red, int m, int n) {
    const float s4 = red[0][m][n] + red[1][m][n] + red[2][m][n] + red[3][m][n];
    if constexpr (NW == 8) return s4 + (red[4][m][n] + red[5][m][n] + red[6][m][n] + red[7][m][n]);
    return s4;
}

template <int NT, int MT>
__device__ __forceinline__ void mma_block(f32x4 (&acc)[NT][MT], const AFrag<NT>& a, const BFrag<MT>& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int m = 0; m < MT; ++m)
                acc[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a.v[t][i]),
                                                                    __builtin_bit_cast(bf16x8, b.v[m][i]),
                                                                    acc[t][m], 0, 0, 0);
}
}  // namespace

// RESID epilogue of one item (4 consecutive columns c .. c+3 of row m, product v): h = bf16(residual + v) (+
// the TP group's copies of the item, rank order, when e.tp.world > 0); returns the item's sum of h^2.
__device__ __forceinline__ float resid_item(const SkinnyNorm& e, int m, int c, int width, unsigned tp_epoch,
                                            const float (&v)[4]) {
    uint2* rp = reinterpret_cast<uint2*>(e.resid + (size_t)m * e.ldr + c);
    const uint2 rv = *rp;
    float4 a = make_float4(v[0], v[1], v[2], v[3]);
    if (e.tp.world > 0) {
        const long long off = mrsum_ar::tp_item_off(m, width, c);
        mrsum_ar::tp_push_item(e.tp, off, tp_epoch, a);
        a = mrsum_ar::tp_gather_item(e.tp, off, tp_epoch);
    }
    const uint2 hv = make_uint2(pack2(__uint_as_float(rv.x << 16) + a.x, __uint_as_float(rv.x & 0xffff0000u) + a.y),
                                pack2(__uint_as_float(rv.y << 16) + a.z, __uint_as_float(rv.y & 0xffff0000u) + a.w));
    *rp = hv;
    const float h0 = __uint_as_float(hv.x << 16), h1 = __uint_as_float(hv.x & 0xffff0000u);
    const float h2 = __uint_as_float(hv.y << 16), h3 = __uint_as_float(hv.y & 0xffff0000u);
    return (h0 * h0 + h1 * h1) + (h2 * h2 + h3 * h3);
}

// RESID tail: the 16-column tile's row sums of h^2 (the 4 items' sums in ``rows[m][0, 4, 8, 12]``) to
// ssp[m][tile], then the TP push epoch of the tile's granule.
template <typename Rows>
__device__ __forceinline__ void resid_tail(const SkinnyNorm& e, const Rows& rows, int M, int n0, unsigned tp_epoch) {
    __syncthreads();
    if (threadIdx.x < M) {
        const float* q = rows[threadIdx.x];
        e.ssp[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = ((q[0] + q[4]) + (q[8] + q[12]));
    }
    if (e.tp.world > 0 && threadIdx.x == 0) e.tp.epochs[n0 / mrsum_ar::GRAN] = tp_epoch;
}

// NW = waves per workgroup (4 or 8), interleaved over the k blocks: a grid of about one workgroup per CU
// (a TP shard's N / 16 tiles) keeps only NW x two blocks of W in flight per CU, so the 8-wave form doubles the
// bytes in flight where the grid cannot (Little's law: ~32 KiB per CU in flight is ~3 TB/s at decode latency).
template <int NT, int MT, int EPI, int NW = 4>
__global__ __launch_bounds__(64 * NW) void skinny_gemm_kernel(const bf16* __restrict__ x, int ldx,
                                                              const bf16* __restrict__ W, int K, int M,
                                                              void* __restrict__ out, int ldo, int kper,
                                                              const SkinnyNorm e) {
    constexpr int BN = 16 * NT, BM = 16 * MT;
    static_assert(EPI != EPI_RESID || (NT == 1 && MT == 1), "RESID: one 16-row tile, M <= 16");
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    __shared__ __attribute__((aligned(16))) float red[NW][BM][BN + 4];
    __shared__ float s_part[EPI == EPI_SWIGLU ? 8 * BM : 1];  // deferred-norm partials [m][8]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n0 = blockIdx.x * BN;
    const int ks = blockIdx.y * kper, ke = min(K, ks + kper);
    // TP push: this launch's epoch of the tile's granule, loaded long before it is needed
    const unsigned tp_epoch = EPI == EPI_RESID && e.tp.world > 0 ? e.tp.epochs[n0 / mrsum_ar::GRAN] + 1 : 0;
    const bool ss_mine = EPI == EPI_SWIGLU && e.ssq && threadIdx.x < 8 * M;
    SsLoads ssl;
    if constexpr (EPI == EPI_SWIGLU) {
        if (ss_mine) deferred_issue(e, threadIdx.x >> 3, threadIdx.x & 7, ssl);
    }

    f32x4 acc[NT][MT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};

    // wave w takes k blocks ks + (w + NW j) * KB.  Issue order per block: x fragments of THIS block,
    // then W of the NEXT block, then the MFMAs -- vmcnt retires loads in issue order, so waiting
    // for x must not also wait for the prefetched W (which would serialise the stream).  The steady
    // loop issues every next-block load unconditionally and the last one or two blocks run in
    // straight-line tails: with the next-block loads under a branch, the waitcnt pass merged the
    // branch's two vmcnt states into the smaller count and waited for the prefetched W before every
    // MFMA of the block, one exposed memory round trip per block.  Same-box A/B: TP=8 shard B=10 -1.4 %,
    // 70B fp8 B=1 -0.5 %, TP=1 B=1/10 unchanged -- the many resident waves had hidden most of it
    // (profiles/r3_skinny_prefetch_fix_ab.jsonl).
    constexpr int STEP = NW * KB;
    const int kb0 = ks + w * KB;
    const int nb = kb0 < ke ? (ke - kb0 + STEP - 1) / STEP : 0;  // this wave's k blocks
    AFrag<NT> a0, a1;
    BFrag<MT> b;
    if (nb > 0) load_a<NT>(a0, W, K, n0, kb0, lane);
    auto ldb = [&](int kb) { load_b<MT>(b, x, ldx, M, kb, lane); };
    int i = 0;
    for (; i + 2 < nb; i += 2) {  // blocks i and i + 1, each with a successor
        const int kb = kb0 + i * STEP;
        ldb(kb);
        load_a<NT>(a1, W, K, n0, kb + STEP, lane);
        mma_block<NT, MT>(acc, a0, b);
        ldb(kb + STEP);
        load_a<NT>(a0, W, K, n0, kb + 2 * STEP, lane);
        mma_block<NT, MT>(acc, a1, b);
    }
    if (nb - i == 2) {
        const int kb = kb0 + i * STEP;
        ldb(kb);
        load_a<NT>(a1, W, K, n0, kb + STEP, lane);
        mma_block<NT, MT>(acc, a0, b);
        ldb(kb + STEP);
        mma_block<NT, MT>(acc, a1, b);
    } else if (nb - i == 1) {
        ldb(kb0 + i * STEP);
        mma_block<NT, MT>(acc, a0, b);
    }

    // C layout (16x16x32): lane holds C[row 4(lane>>4)+j][col lane&15] = out^T[n][m]
    const int cn = 4 * (lane >> 4), cm = lane & 15;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int j = 0; j < 4; ++j) red[w][16 * m + cm][16 * t + cn + j] = acc[t][m][j];
    if constexpr (EPI == EPI_SWIGLU) {
        if (ss_mine) s_part[threadIdx.x] = deferred_partial(ssl);
    }
    __syncthreads();

    // each item = 4 consecutive n of one m
    constexpr int ITEMS = BM * (BN / 4);
    for (int it = threadIdx.x; it < ITEMS; it += 64 * NW) {
        const int m = it / (BN / 4), n4 = (it % (BN / 4)) * 4;
        if (m >= M) continue;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = wsum<NW>(red, m, n4 + j);
        if constexpr (EPI == EPI_BF16) {
            uint2 o;
            o.x = pack2(v[0], v[1]);
            o.y = pack2(v[2], v[3]);
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldo + n0 + n4) = o;
        } else if constexpr (EPI == EPI_F32_PARTIAL) {
            float* o = reinterpret_cast<float*>(out) + ((size_t)blockIdx.y * M + m) * ldo + n0 + n4;
            *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        } else if constexpr (EPI == EPI_RESID) {
            red[0][m][n4] = resid_item(e, m, n0 + n4, gridDim.x * BN, tp_epoch, v);  // own slot: reads are done
        } else {  // SWIGLU: tile rows [0, BN/2) gate, [BN/2, BN) up of features [blockIdx.x*BN/2, +BN/2)
            constexpr int H = BN / 2;
            if (n4 < H) {
                const float sc = e.ssq ? deferred_row_scale(e, s_part, m) : 1.f;
                float r[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float u = wsum<NW>(red, m, n4 + H + j) * sc;
                    const float g = v[j] * sc;
                    r[j] = g / (1.f + __expf(-g)) * u;
                }
                uint2 o;
                o.x = pack2(r[0], r[1]);
                o.y = pack2(r[2], r[3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldo + blockIdx.x * H + n4) = o;
            }
        }
    }
    if constexpr (EPI == EPI_RESID) resid_tail(e, red[0], M, n0, tp_epoch);
}

template <int NT, int EPI, int NW>
static int launch_mt(int mt, dim3 grid, hipStream_t s, const bf16* x, int ldx, const bf16* W, int K, int M,
                     void* out, int ldo, int kper, const SkinnyNorm& e) {
    const dim3 block(64 * NW);
    switch (mt) {
        case 1: skinny_gemm_kernel<NT, 1, EPI, NW><<<grid, block, 0, s>>>(x, ldx, W, K, M, out, ldo, kper, e); break;
        case 2: skinny_gemm_kernel<NT, 2, EPI, NW><<<grid, block, 0, s>>>(x, ldx, W, K, M, out, ldo, kper, e); break;
        case 3: skinny_gemm_kernel<NT, 3, EPI, NW><<<grid, block, 0, s>>>(x, ldx, W, K, M, out, ldo, kper, e); break;
        case 4: skinny_gemm_kernel<NT, 4, EPI, NW><<<grid, block, 0, s>>>(x, ldx, W, K, M, out, ldo, kper, e); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// Workgroups of the residual-update (TP push) instantiation with ``waves`` waves that can be resident on this
// device at once: occupancy per CU x CUs (header: a TP-push grid must fit, every workgroup spins on its peers).
MRSUM_API int mrsum_skinny_resid_capacity_w(int waves) {
    static int cap[2] = {-1, -1};
    const int i = waves == 8 ? 1 : 0;
    if (cap[i] < 0) {
        int dev = 0, cus = 0, per = 0;
        hipError_t st = hipGetDevice(&dev);
        if (st == hipSuccess) st = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (st == hipSuccess)
            st = i ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, skinny_gemm_kernel<1, 1, EPI_RESID, 8>, 512, 0)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, skinny_gemm_kernel<1, 1, EPI_RESID, 4>, 256, 0);
        if (st != hipSuccess) return 0;
        cap[i] = cus * per;
    }
    return cap[i];
}

MRSUM_API int mrsum_skinny_resid_capacity() { return mrsum_skinny_resid_capacity_w(4); }

// epi: 0 bf16 [M, ldo], 1 fp32 partial [S, M, ldo], 2 swiglu bf16 [M, ldo] (ldo >= N/2), 3 residual update
// (resid [M, ldr] bf16 += x W^T, ssp fp32 [M, N / 16] per-tile row sums of squares of the new residual;
// nt 1, splits 1, M <= 16; ``ar`` non-null: all-reduced over that custom all-reduce group first (TP push,
// M * N * 4 <= its slot bytes)).  nt: 16-row W tiles per workgroup (1 or 2; swiglu needs 1); splits: S (K/S
// multiple of 128).  ssq (swiglu only): deferred-RMSNorm input [M, ssq_tiles] fp32, ssq_tiles % 32 == 0.
// waves: 4 or 8 per workgroup (kernel header).
MRSUM_API int mrsum_skinny_gemm(const void* x, int ldx, const void* W, int N, int K, int M, void* out, int ldo,
                                int epi, int nt, int splits, const float* ssq, int ssq_tiles, float eps, void* resid,
                                int ldr, float* ssp, void* ar, int waves, hipStream_t s) {
    using namespace mrsum_ar;
    if (M <= 0) return 0;
    if (M > 64 || K % KB || splits < 1 || (K / KB) % splits || (nt != 1 && nt != 2) || N % (16 * nt) ||
        epi < EPI_BF16 || epi > EPI_RESID || (waves != 4 && waves != 8))
        return (int)hipErrorInvalidValue;
    if (epi != EPI_F32_PARTIAL && splits != 1) return (int)hipErrorInvalidValue;
    if (epi == EPI_SWIGLU && nt != 1) return (int)hipErrorInvalidValue;  // weight blocks of [8 gate | 8 up]
    if (ssq && (epi != EPI_SWIGLU || ssq_tiles <= 0 || ssq_tiles % 32 || ssq_tiles > 32 * SS_C4))
        return (int)hipErrorInvalidValue;
    if (epi == EPI_RESID && (nt != 1 || M > 16 || !resid || !ssp || ldr % 4)) return (int)hipErrorInvalidValue;
    if (ar) {
        auto h = (const ArHandle*)ar;
        if (epi != EPI_RESID || N / GRAN > MAX_GRAN || (size_t)M * N * 4 > h->max_bytes) return (int)hipErrorInvalidValue;
        for (int r = 0; r < h->world; ++r)
            if (!h->peers.base[r]) return (int)hipErrorInvalidValue;
    }
    if (ar && N / 16 > mrsum_skinny_resid_capacity_w(waves)) return (int)hipErrorInvalidValue;  // header: progress
    SkinnyNorm e;
    e.ssq = ssq; e.ssq_tiles = ssq_tiles; e.inv_k = 1.f / (float)K; e.eps = eps;
    e.resid = (bf16*)resid; e.ldr = ldr; e.ssp = ssp;
    e.tp = tp_push_of((const ArHandle*)ar);
    const int kper = K / splits;
    const int mt = (M + 15) / 16;
    dim3 grid(N / (16 * nt), splits);
    auto X = (const bf16*)x; auto Wp = (const bf16*)W;
#define BY_W(NT_, EPI_)                                                                       \
    return waves == 8 ? launch_mt<NT_, EPI_, 8>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper, e) \
                      : launch_mt<NT_, EPI_, 4>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper, e)
    if (nt == 1) {
        if (epi == EPI_BF16) BY_W(1, EPI_BF16);
        if (epi == EPI_F32_PARTIAL) BY_W(1, EPI_F32_PARTIAL);
        if (epi == EPI_SWIGLU) BY_W(1, EPI_SWIGLU);
        if (waves == 8) {
            skinny_gemm_kernel<1, 1, EPI_RESID, 8><<<grid, 512, 0, s>>>(X, ldx, Wp, K, M, out, ldo, kper, e);
        } else {
            skinny_gemm_kernel<1, 1, EPI_RESID, 4><<<grid, 256, 0, s>>>(X, ldx, Wp, K, M, out, ldo, kper, e);
        }
        return (int)hipGetLastError();
    } else {
        if (epi == EPI_BF16) BY_W(2, EPI_BF16);
        if (epi == EPI_F32_PARTIAL) BY_W(2, EPI_F32_PARTIAL);
    }
#undef BY_W
    return (int)hipErrorInvalidValue;
}


// ---------------------------------------------------------------------------------------------
// Medium-M variant (16 < M <= 64): x is shared by every W row, so at these M the per-wave x
// fragment loads of the kernel above dominate its instruction stream.  Here the workgroup stages
// each 128-wide k block of x ONCE into LDS (double-buffered, 16-B chunks XOR-swizzled by row&15
// for conflict-free ds_read_b128), and each of the 4 waves streams its own 16 W rows over the
// FULL k range (or the split's k range) straight from HBM into A fragments, prefetched one block
// ahead.  No cross-wave reduction: the epilogue goes straight from the accumulators (SwiGLU pairs
// gate/up across the lane halves with one xor-32 shuffle).
namespace {
__device__ __forceinline__ int xs_off(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }
}

// blockDim = 64 * wpb (wpb = 4..8 waves, each owning 16 W rows): the host picks wpb and the split
// count so the grid is a whole number of workgroups per CU -- with 448 four-wave tiles on 256 CUs a
// quarter of the CUs streams half as much as the rest and the kernel ends at ~4 TB/s.
template <int MT, int EPI, int PD>
__global__ __launch_bounds__(512) void skinny_lds_kernel(const bf16* __restrict__ x, int ldx,
                                                         const bf16* __restrict__ W, int K, int M,
                                                         void* __restrict__ out, int ldo, int kper) {
    constexpr int BM = 16 * MT;
    constexpr int XCH = BM * 16 / 256;  // 16-B x chunks per thread per k block at wpb = 4 (fewer above)
    __shared__ __attribute__((aligned(16))) char xl[2][BM * 256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, g = lane >> 4;
    const int nthr = blockDim.x;
    const int n0 = blockIdx.x * (nthr >> 2) + 16 * w;  // this wave's 16 W rows (16 * wpb rows per WG)
    const int ks = blockIdx.y * kper, ke = min(K, ks + kper);
    const int nkb = (ke - ks) / 128;

    // x staging: chunk id = tid + nthr i -> row = id / 16, chunk = id % 16 (ids past BM*16 idle)
    u32x4 xr[XCH];
#define LOAD_X(kb)                                                                                         \
    _Pragma("unroll") for (int i = 0; i < XCH; ++i) {                                                      \
        const int id = min(tid + nthr * i, BM * 16 - 1);                                                   \
        xr[i] = *reinterpret_cast<const u32x4*>(x + (size_t)min(id >> 4, M - 1) * ldx + (kb) + (id & 15) * 8); \
    }
#define STORE_X(buf)                                                                                       \
    _Pragma("unroll") for (int i = 0; i < XCH; ++i) {                                                      \
        const int id = tid + nthr * i;                                                                     \
        if (id < BM * 16) *reinterpret_cast<u32x4*>(&xl[buf][xs_off(id >> 4, id & 15)]) = xr[i];          \
    }
    const bf16* wrow = W + (size_t)(n0 + r) * K + 8 * g;
    u32x4 a0[4], a1[4], a2[4];
#define LOAD_A(dst, kb) \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) dst[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow + (kb) + 32 * i));
#define MMA(USE, CUR)                                                                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                                        \
        _Pragma("unroll") for (int m = 0; m < MT; ++m) {                                                   \
            const u32x4 bv = *reinterpret_cast<const u32x4*>(&xl[CUR][xs_off(16 * m + r, 4 * i + g)]);     \
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, USE[i]),           \
                                                             __builtin_bit_cast(bf16x8, bv), acc[m], 0, 0, 0); \
        }                                                                                                  \
    }

    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

    LOAD_X(ks);
    LOAD_A(a0, ks);
    if constexpr (PD == 2) LOAD_A(a1, ks + min(1, nkb - 1) * 128);
    STORE_X(0);
    __syncthreads();
    if constexpr (PD == 1) {
        // two k blocks per trip so the A register sets and LDS buffers have static roles (rule 20)
#define STEP(j, USE, PREF, CUR)                                                                            \
    {                                                                                                      \
        const int kn = ks + min((j) + 1, nkb - 1) * 128; /* unconditional prefetch (last block re-read) */ \
        LOAD_X(kn);                                                                                        \
        LOAD_A(PREF, kn);                                                                                  \
        MMA(USE, CUR);                                                                                     \
        STORE_X(CUR ^ 1);                                                                                  \
        __syncthreads();                                                                                   \
    }
        for (int j = 0; j < nkb; j += 2) {
            STEP(j, a0, a1, 0);
            if (j + 1 >= nkb) break;
            STEP(j + 1, a1, a0, 1);
        }
#undef STEP
    } else {
        // prefetch distance 2: W block j+2 is in flight while block j is consumed (x for block j+1 is
        // issued first, so waiting on it never waits on the newer W loads -- vmcnt is in order).
        // Three W register sets rotate with static roles; the LDS buffer index is a runtime value.
#define STEP2(j, USE, PREF)                                                                                \
    {                                                                                                      \
        LOAD_X(ks + min((j) + 1, nkb - 1) * 128);                                                          \
        LOAD_A(PREF, ks + min((j) + 2, nkb - 1) * 128);                                                    \
        const int cur = (j) & 1;                                                                           \
        MMA(USE, cur);                                                                                     \
        STORE_X(cur ^ 1);                                                                                  \
        __syncthreads();                                                                                   \
    }
        for (int j = 0; j < nkb; j += 3) {
            STEP2(j, a0, a2);
            if (j + 1 >= nkb) break;
            STEP2(j + 1, a1, a0);
            if (j + 2 >= nkb) break;
            STEP2(j + 2, a2, a1);
        }
#undef STEP2
    }
#undef MMA
#undef LOAD_X
#undef STORE_X
#undef LOAD_A

    // C: lane holds out^T[n = n0 + 4g + j][m = 16 mt + r]
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int mm = 16 * m + r;
        if constexpr (EPI == EPI_SWIGLU) {
            // rows 0-7 of the wave tile = gate (g 0,1), rows 8-15 = up (g 2,3) of features blockIdx.x*32 + 8w + ...
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
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)mm * ldo + (n0 >> 1) + 4 * g) = o;
            }
        } else if (mm < M) {
            if constexpr (EPI == EPI_BF16) {
                uint2 o;
                o.x = pack2(acc[m][0], acc[m][1]);
                o.y = pack2(acc[m][2], acc[m][3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)mm * ldo + n0 + 4 * g) = o;
            } else {
                float* o = reinterpret_cast<float*>(out) + ((size_t)blockIdx.y * M + mm) * ldo + n0 + 4 * g;
                *reinterpret_cast<float4*>(o) = make_float4(acc[m][0], acc[m][1], acc[m][2], acc[m][3]);
            }
        }
    }
}

// Same contract as mrsum_skinny_gemm; N % (16 wpb) == 0, 16 < M <= 64 (also valid for M <= 16).
// W is prefetched two 128-wide k blocks ahead (depth 1 measured slower; profiles/r1_decode_gemm_sweep.txt)
MRSUM_API int mrsum_skinny_lds(const void* x, int ldx, const void* W, int N, int K, int M, void* out, int ldo,
                               int epi, int splits, int wpb, hipStream_t s) {
    if (M <= 0) return 0;
    if (wpb < 4 || wpb > 8) return (int)hipErrorInvalidValue;
    if (M > 64 || K % KB || N % (16 * wpb) || splits < 1 || (K / KB) % splits) return (int)hipErrorInvalidValue;
    if (epi != EPI_F32_PARTIAL && splits != 1) return (int)hipErrorInvalidValue;
    const int kper = K / splits;
    const int mt = (M + 15) / 16;
    dim3 grid(N / (16 * wpb), splits), block(64 * wpb);
    auto X = (const bf16*)x; auto Wp = (const bf16*)W;
#define L(MT_, EPI_) skinny_lds_kernel<MT_, EPI_, 2><<<grid, block, 0, s>>>(X, ldx, Wp, K, M, out, ldo, kper)
#define BY_EPI(MT_) \
    if (epi == EPI_BF16) { L(MT_, EPI_BF16); } else if (epi == EPI_F32_PARTIAL) { L(MT_, EPI_F32_PARTIAL); } \
    else { L(MT_, EPI_SWIGLU); }
    switch (mt) {
        case 1: BY_EPI(1); break;
        case 2: BY_EPI(2); break;
        case 3: BY_EPI(3); break;
        default: BY_EPI(4); break;
    }
#undef BY_EPI
#undef L
    return (int)hipGetLastError();
}


// ---------------------------------------------------------------------------------------------
// FP8 weights (OCP e4m3fn, gfx950's format -- not MI300's fnuz) with one fp32 scale per output row:
//   out[m, n] = scale[n] * sum_k float(W8[n, k]) * x[m, k]          (W8A16: activations stay bf16)
// Same decomposition as skinny_gemm_kernel; a lane's 16-B load now carries 16 k-elements of its W
// row, converted exactly to bf16 with v_cvt_scalef32_pk_bf16_fp8 (2 per instruction) into the A
// fragments of two consecutive MFMA k-steps.  The k order inside a 64-wide chunk is permuted
// (lane group g holds k = 16g .. 16g+15 of the chunk) and the x (B) fragments are loaded with the
// same permutation, so the sum is unchanged.  Half the HBM bytes of the bf16 kernel per weight:
// this is the decode path of the fp8 Llama-3-70B aggregator.
namespace {
template <int NT>
struct A8Frag {
    u32x4 v[NT][2];
};

template <int NT>
__device__ __forceinline__ void load_a8(A8Frag<NT>& a, const uint8_t* __restrict__ W, int K, int n0, int kb,
                                        int lane) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint8_t* p = W + (size_t)(n0 + 16 * t + r) * K + kb + 16 * g;
#pragma unroll
        for (int c = 0; c < 2; ++c) a.v[t][c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 64 * c));
    }
}

__device__ __forceinline__ bf16x8 fp8x8_to_bf16(unsigned d0, unsigned d1) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, false);
    const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, true);
    const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, false);
    const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, true);
    return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

template <int MT>
__device__ __forceinline__ void load_b8(BFrag<MT>& b, const bf16* __restrict__ x, int ldx, int M, int kb, int lane) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int row = min(16 * m + r, M - 1);
        const bf16* p = x + (size_t)row * ldx + kb + 16 * g;
#pragma unroll
        for (int i = 0; i < 4; ++i) b.v[m][i] = *reinterpret_cast<const uint4*>(p + 64 * (i >> 1) + 8 * (i & 1));
    }
}

template <int NT, int MT>
__device__ __forceinline__ void mma_block8(f32x4 (&acc)[NT][MT], const A8Frag<NT>& a, const BFrag<MT>& b) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const u32x4 raw = a.v[t][i >> 1];
            const bf16x8 av = (i & 1) ? fp8x8_to_bf16(raw[2], raw[3]) : fp8x8_to_bf16(raw[0], raw[1]);
#pragma unroll
            for (int m = 0; m < MT; ++m)
                acc[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, __builtin_bit_cast(bf16x8, b.v[m][i]),
                                                                    acc[t][m], 0, 0, 0);
        }
}
}  // namespace

// XL (M = 1): the x row slice [ks, ke) is staged in LDS once per workgroup and the B fragments are read
// from there (a broadcast ds_read_b128 per k-step) -- otherwise every wave re-reads x from L2 for each
// weight block, 4 KiB of VMEM requests per 2 KiB of fp8 weights, twice the weight traffic itself.
// XL also takes a deferred-RMSNorm input (stream_gemm.hip header): x = the un-normalised residual row,
// ``ssq`` [1][ssq_tiles] its producer's per-tile sums of squares, reduced in the stream consumer's fixed
// order (8 partials of ssq_tiles / 8 tiles, float4 steps) so both consumers scale by the same factor.
// NW = 4 or 8 waves per workgroup (skinny_gemm_kernel header: bytes in flight per CU on small grids).
// EPI_RESID (one 16-row tile, M <= 16): the residual producer of skinny_gemm_kernel with fp8 weights --
// residual += x W^T (after the TP push when e.tp.world > 0), per-tile row sums of squares to e.ssp.
template <int NT, int MT, int EPI, bool XL, int NW = 4>
__global__ __launch_bounds__(64 * NW) void skinny_fp8_kernel(const bf16* __restrict__ x, int ldx,
                                                             const uint8_t* __restrict__ W,
                                                             const float* __restrict__ wscale, int K, int M,
                                                             void* __restrict__ out, int ldo, int kper,
                                                             const float* __restrict__ ssq, int ssq_tiles, float eps,
                                                             const SkinnyNorm e) {
    constexpr int BN = 16 * NT, BM = 16 * MT;
    static_assert(!XL || MT == 1, "the LDS x slice holds one row");
    static_assert(EPI != EPI_RESID || (NT == 1 && MT == 1), "RESID: one 16-row tile, M <= 16");
    __shared__ __attribute__((aligned(16))) float red[NW][BM][BN + 4];
    __shared__ float s_ss[8];
    extern __shared__ __attribute__((aligned(16))) char xs[];  // XL: kper bf16 of x row 0
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n0 = blockIdx.x * BN;
    const int ks = blockIdx.y * kper, ke = min(K, ks + kper);
    const unsigned tp_epoch = EPI == EPI_RESID && e.tp.world > 0 ? e.tp.epochs[n0 / mrsum_ar::GRAN] + 1 : 0;
    constexpr int STEP = NW * KB;
    const int kb0 = ks + w * KB;
    const int nb = kb0 < ke ? (ke - kb0 + STEP - 1) / STEP : 0;
    A8Frag<NT> a0, a1;
    // XL: the x slice's loads first, then the first weight block's, and only then the LDS writes of the
    // slice -- waiting for x (the older loads: vmcnt retires in order) never waits for W, so the weight
    // stream starts under the slice's round trip instead of after the barrier
    constexpr int XPRE = 4;  // 16-B x chunks per thread held in registers across the first weight loads
    const uint4* xsrc = reinterpret_cast<const uint4*>(x + ks);
    const int nx = kper / 8;
    uint4 xr[XL ? XPRE : 1];
    if constexpr (XL) {
#pragma unroll
        for (int j = 0; j < XPRE; ++j) xr[j] = xsrc[min((int)threadIdx.x + j * 64 * NW, nx - 1)];  // clamped
    }
    if (nb > 0) load_a8<NT>(a0, W, K, n0, kb0, lane);
    if constexpr (XL) {
#pragma unroll
        for (int j = 0; j < XPRE; ++j) {
            const int i = threadIdx.x + j * 64 * NW;
            if (i < nx) reinterpret_cast<uint4*>(xs)[i] = xr[j];
        }
        for (int i = threadIdx.x + XPRE * 64 * NW; i < nx; i += 64 * NW)  // slices beyond 4 chunks per thread
            reinterpret_cast<uint4*>(xs)[i] = xsrc[i];
        if (ssq && threadIdx.x < 8) {
            const int C = ssq_tiles / 8;
            const float4* sp = reinterpret_cast<const float4*>(ssq + threadIdx.x * C);
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int q = 0; q < C / 4; ++q) {
                const float4 v = sp[q];
                a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
            }
            s_ss[threadIdx.x] = (a.x + a.y) + (a.z + a.w);
        }
        // LDS writes visible to the workgroup; no vmcnt(0) here (the weight loads stay in flight)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
    auto load_b = [&](BFrag<MT>& b, int kb) {
        if constexpr (XL) {
            const char* p = xs + (kb - ks + 16 * (lane >> 4)) * 2;
#pragma unroll
            for (int i = 0; i < 4; ++i) b.v[0][i] = *reinterpret_cast<const uint4*>(p + (64 * (i >> 1) + 8 * (i & 1)) * 2);
        } else {
            load_b8<MT>(b, x, ldx, M, kb, lane);
        }
    };

    f32x4 acc[NT][MT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};

    // unconditional next-block loads in the steady loop, straight-line tails (as skinny_gemm_kernel)
    BFrag<MT> b;
    int i = 0;
    for (; i + 2 < nb; i += 2) {
        const int kb = kb0 + i * STEP;
        load_b(b, kb);
        load_a8<NT>(a1, W, K, n0, kb + STEP, lane);
        mma_block8<NT, MT>(acc, a0, b);
        load_b(b, kb + STEP);
        load_a8<NT>(a0, W, K, n0, kb + 2 * STEP, lane);
        mma_block8<NT, MT>(acc, a1, b);
    }
    if (nb - i == 2) {
        const int kb = kb0 + i * STEP;
        load_b(b, kb);
        load_a8<NT>(a1, W, K, n0, kb + STEP, lane);
        mma_block8<NT, MT>(acc, a0, b);
        load_b(b, kb + STEP);
        mma_block8<NT, MT>(acc, a1, b);
    } else if (nb - i == 1) {
        load_b(b, kb0 + i * STEP);
        mma_block8<NT, MT>(acc, a0, b);
    }

    const int cn = 4 * (lane >> 4), cm = lane & 15;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int j = 0; j < 4; ++j) red[w][16 * m + cm][16 * t + cn + j] = acc[t][m][j];
    __syncthreads();
    float rs = 1.f;  // deferred-norm row scale (XL: one row)
    if (XL && ssq) {
        float t = 0.f;
#pragma unroll
        for (int p = 0; p < 8; ++p) t += s_ss[p];
        rs = rsqrtf(t * (1.f / (float)K) + eps);
    }

    constexpr int ITEMS = BM * (BN / 4);
    for (int it = threadIdx.x; it < ITEMS; it += 64 * NW) {
        const int m = it / (BN / 4), n4 = (it % (BN / 4)) * 4;
        if (m >= M) continue;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            v[j] = wsum<NW>(red, m, n4 + j) * wscale[n0 + n4 + j] * rs;
        if constexpr (EPI == EPI_BF16) {
            uint2 o;
            o.x = pack2(v[0], v[1]);
            o.y = pack2(v[2], v[3]);
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldo + n0 + n4) = o;
        } else if constexpr (EPI == EPI_F32_PARTIAL) {
            float* o = reinterpret_cast<float*>(out) + ((size_t)blockIdx.y * M + m) * ldo + n0 + n4;
            *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        } else if constexpr (EPI == EPI_RESID) {
            red[0][m][n4] = resid_item(e, m, n0 + n4, gridDim.x * BN, tp_epoch, v);  // own slot: reads are done
        } else {  // SWIGLU, nt == 1: rows [0, 8) gate, [8, 16) up
            constexpr int H = BN / 2;
            if (n4 < H) {
                float rr[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float u = wsum<NW>(red, m, n4 + H + j) * wscale[n0 + n4 + H + j] * rs;
                    rr[j] = v[j] / (1.f + __expf(-v[j])) * u;
                }
                uint2 o;
                o.x = pack2(rr[0], rr[1]);
                o.y = pack2(rr[2], rr[3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldo + blockIdx.x * H + n4) = o;
            }
        }
    }
    if constexpr (EPI == EPI_RESID) resid_tail(e, red[0], M, n0, tp_epoch);
}

MRSUM_API int mrsum_skinny_fp8_resid_capacity();

// ssq (deferred-RMSNorm input, M = 1 with the x slice in LDS only): [1][ssq_tiles] fp32 row sums of squares
// of x per producer tile, ssq_tiles % 32 == 0; the product is scaled by rsqrt(sum / K + eps).  waves: 4 or 8.
// epi 3 (residual update, mrsum_skinny_gemm's contract): resid [M, ldr] bf16 += x W^T, ssp [M, N / 16]; nt 1,
// splits 1, M <= 16; ``ar``: TP push over that custom all-reduce group.
MRSUM_API int mrsum_skinny_fp8(const void* x, int ldx, const void* W, const float* wscale, int N, int K, int M,
                               void* out, int ldo, int epi, int nt, int splits, const float* ssq, int ssq_tiles,
                               float eps, void* resid, int ldr, float* ssp, void* ar, int waves, hipStream_t s) {
    using namespace mrsum_ar;
    if (M <= 0) return 0;
    if (M > 64 || K % KB || splits < 1 || (K / KB) % splits || (nt != 1 && nt != 2) || N % (16 * nt) ||
        (waves != 4 && waves != 8) || epi < EPI_BF16 || epi > EPI_RESID)
        return (int)hipErrorInvalidValue;
    if (epi != EPI_F32_PARTIAL && splits != 1) return (int)hipErrorInvalidValue;
    if (epi == EPI_SWIGLU && nt != 1) return (int)hipErrorInvalidValue;
    if (epi == EPI_RESID && (nt != 1 || M > 16 || !resid || !ssp || ldr % 4 || ssq)) return (int)hipErrorInvalidValue;
    if (ar) {
        auto h = (const ArHandle*)ar;
        if (epi != EPI_RESID || N / GRAN > MAX_GRAN || (size_t)M * N * 4 > h->max_bytes) return (int)hipErrorInvalidValue;
        for (int r = 0; r < h->world; ++r)
            if (!h->peers.base[r]) return (int)hipErrorInvalidValue;
        if (N / 16 > mrsum_skinny_fp8_resid_capacity()) return (int)hipErrorInvalidValue;  // every pusher resident
    }
    SkinnyNorm e{};
    e.resid = (bf16*)resid; e.ldr = ldr; e.ssp = ssp;
    e.tp = tp_push_of((const ArHandle*)ar);
    const int kper = K / splits;
    const int mt = (M + 15) / 16;
    dim3 grid(N / (16 * nt), splits);
    auto X = (const bf16*)x; auto Wp = (const uint8_t*)W;
    const bool xl = M == 1 && kper * 2 <= 56 * 1024;  // x slice in (default-limit) dynamic LDS
    if (ssq && (!xl || ssq_tiles <= 0 || ssq_tiles % 32)) return (int)hipErrorInvalidValue;
#define L(NT_, MT_, EPI_, NW_)                                                                                  \
    skinny_fp8_kernel<NT_, MT_, EPI_, false, NW_><<<grid, 64 * NW_, 0, s>>>(X, ldx, Wp, wscale, K, M, out, ldo, kper, \
                                                                          nullptr, 0, 0.f, e)
#define L1(NT_, EPI_, NW_)                                                                                      \
    if (xl) skinny_fp8_kernel<NT_, 1, EPI_, true, NW_><<<grid, 64 * NW_, kper * 2, s>>>(X, ldx, Wp, wscale, K, M, out, \
                                                                                      ldo, kper, ssq, ssq_tiles, eps, e); \
    else L(NT_, 1, EPI_, NW_)
#define BY_MT(NT_, EPI_, NW_)                   \
    switch (mt) {                               \
        case 1: L1(NT_, EPI_, NW_); break;      \
        case 2: L(NT_, 2, EPI_, NW_); break;    \
        case 3: L(NT_, 3, EPI_, NW_); break;    \
        default: L(NT_, 4, EPI_, NW_); break;   \
    }
#define BY_EPI(NW_)                                                           \
    if (nt == 1) {                                                            \
        if (epi == EPI_BF16) { BY_MT(1, EPI_BF16, NW_) }                      \
        else if (epi == EPI_F32_PARTIAL) { BY_MT(1, EPI_F32_PARTIAL, NW_) }   \
        else if (epi == EPI_SWIGLU) { BY_MT(1, EPI_SWIGLU, NW_) }             \
        else { L1(1, EPI_RESID, NW_); }                                       \
    } else {                                                                  \
        if (epi == EPI_BF16) { BY_MT(2, EPI_BF16, NW_) }                      \
        else { BY_MT(2, EPI_F32_PARTIAL, NW_) }                               \
    }
    if (waves == 8) { BY_EPI(8) } else { BY_EPI(4) }
#undef BY_EPI
#undef BY_MT
#undef L1
#undef L
    return (int)hipGetLastError();
}

// Workgroups of the fp8 residual producer resident at once (the smaller of the 4- / 8-wave, LDS-x / global-x
// forms; a TP-push grid of N / 16 workgroups must fit, as for mrsum_skinny_resid_capacity_w).
MRSUM_API int mrsum_skinny_fp8_resid_capacity() {
    static int cap = -1;
    if (cap < 0) {
        int dev = 0, cus = 0, lo = 1 << 30;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        int per = 0;
        // the LDS-x form is sized for the largest x slice it takes (56 KiB)
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, skinny_fp8_kernel<1, 1, EPI_RESID, true, 4>, 256,
                                                         56 * 1024) != hipSuccess) return 0;
        lo = std::min(lo, per);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, skinny_fp8_kernel<1, 1, EPI_RESID, true, 8>, 512,
                                                         56 * 1024) != hipSuccess) return 0;
        lo = std::min(lo, per);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, skinny_fp8_kernel<1, 1, EPI_RESID, false, 4>, 256, 0)
            != hipSuccess) return 0;
        lo = std::min(lo, per);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, skinny_fp8_kernel<1, 1, EPI_RESID, false, 8>, 512, 0)
            != hipSuccess) return 0;
        lo = std::min(lo, per);
        cap = cus * lo;
    }
    return cap;
}
