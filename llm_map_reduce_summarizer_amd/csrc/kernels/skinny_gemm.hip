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
#include "common.h"

namespace {
enum { EPI_BF16 = 0, EPI_F32_PARTIAL = 1, EPI_SWIGLU = 2 };
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

template <int NT, int MT, int EPI>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const bf16* __restrict__ x, int ldx,
                                                          const bf16* __restrict__ W, int K, int M,
                                                          void* __restrict__ out, int ldo, int kper) {
    constexpr int BN = 16 * NT, BM = 16 * MT;
    __shared__ __attribute__((aligned(16))) float red[4][BM][BN + 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n0 = blockIdx.x * BN;
    const int ks = blockIdx.y * kper, ke = min(K, ks + kper);

    f32x4 acc[NT][MT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[t][m] = f32x4{0.f, 0.f, 0.f, 0.f};

    // wave w takes k blocks ks + (w + 4j) * KB.  Issue order per block: x fragments of THIS block,
    // then W of the NEXT block, then the MFMAs -- vmcnt retires loads in issue order, so waiting
    // for x must not also wait for the prefetched W (which would serialise the stream).
    int kb = ks + w * KB;
    AFrag<NT> a0, a1;
    BFrag<MT> b;
    if (kb < ke) load_a<NT>(a0, W, K, n0, kb, lane);
    while (kb < ke) {
        const int kb1 = kb + 4 * KB;
        load_b<MT>(b, x, ldx, M, kb, lane);
        if (kb1 < ke) load_a<NT>(a1, W, K, n0, kb1, lane);
        mma_block<NT, MT>(acc, a0, b);
        if (kb1 >= ke) break;
        const int kb2 = kb1 + 4 * KB;
        load_b<MT>(b, x, ldx, M, kb1, lane);
        if (kb2 < ke) load_a<NT>(a0, W, K, n0, kb2, lane);
        mma_block<NT, MT>(acc, a1, b);
        kb = kb2;
    }

    // C layout (16x16x32): lane holds C[row 4(lane>>4)+j][col lane&15] = out^T[n][m]
    const int cn = 4 * (lane >> 4), cm = lane & 15;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int j = 0; j < 4; ++j) red[w][16 * m + cm][16 * t + cn + j] = acc[t][m][j];
    __syncthreads();

    // each item = 4 consecutive n of one m
    constexpr int ITEMS = BM * (BN / 4);
    for (int it = threadIdx.x; it < ITEMS; it += 256) {
        const int m = it / (BN / 4), n4 = (it % (BN / 4)) * 4;
        if (m >= M) continue;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = red[0][m][n4 + j] + red[1][m][n4 + j] + red[2][m][n4 + j] + red[3][m][n4 + j];
        if constexpr (EPI == EPI_BF16) {
            uint2 o;
            o.x = pack2(v[0], v[1]);
            o.y = pack2(v[2], v[3]);
            *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldo + n0 + n4) = o;
        } else if constexpr (EPI == EPI_F32_PARTIAL) {
            float* o = reinterpret_cast<float*>(out) + ((size_t)blockIdx.y * M + m) * ldo + n0 + n4;
            *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
        } else {  // SWIGLU: tile rows [0, BN/2) gate, [BN/2, BN) up of features [blockIdx.x*BN/2, +BN/2)
            constexpr int H = BN / 2;
            if (n4 < H) {
                float r[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float u = red[0][m][n4 + H + j] + red[1][m][n4 + H + j] + red[2][m][n4 + H + j] +
                                    red[3][m][n4 + H + j];
                    const float g = v[j];
                    r[j] = g / (1.f + __expf(-g)) * u;
                }
                uint2 o;
                o.x = pack2(r[0], r[1]);
                o.y = pack2(r[2], r[3]);
                *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + (size_t)m * ldo + blockIdx.x * H + n4) = o;
            }
        }
    }
}

template <int NT, int EPI>
static int launch_mt(int mt, dim3 grid, hipStream_t s, const bf16* x, int ldx, const bf16* W, int K, int M,
                     void* out, int ldo, int kper) {
    switch (mt) {
        case 1: skinny_gemm_kernel<NT, 1, EPI><<<grid, 256, 0, s>>>(x, ldx, W, K, M, out, ldo, kper); break;
        case 2: skinny_gemm_kernel<NT, 2, EPI><<<grid, 256, 0, s>>>(x, ldx, W, K, M, out, ldo, kper); break;
        case 3: skinny_gemm_kernel<NT, 3, EPI><<<grid, 256, 0, s>>>(x, ldx, W, K, M, out, ldo, kper); break;
        case 4: skinny_gemm_kernel<NT, 4, EPI><<<grid, 256, 0, s>>>(x, ldx, W, K, M, out, ldo, kper); break;
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}

// epi: 0 bf16 [M, ldo], 1 fp32 partial [S, M, ldo], 2 swiglu bf16 [M, ldo] (ldo >= N/2)
// nt: 16-row W tiles per workgroup (1 or 2; swiglu needs 1); splits: S (K/S multiple of 128)
MRSUM_API int mrsum_skinny_gemm(const void* x, int ldx, const void* W, int N, int K, int M, void* out, int ldo,
                                int epi, int nt, int splits, hipStream_t s) {
    if (M <= 0) return 0;
    if (M > 64 || K % KB || splits < 1 || (K / KB) % splits || (nt != 1 && nt != 2) || N % (16 * nt))
        return (int)hipErrorInvalidValue;
    if (epi != EPI_F32_PARTIAL && splits != 1) return (int)hipErrorInvalidValue;
    if (epi == EPI_SWIGLU && nt != 1) return (int)hipErrorInvalidValue;  // weight blocks of [8 gate | 8 up]
    const int kper = K / splits;
    const int mt = (M + 15) / 16;
    dim3 grid(N / (16 * nt), splits);
    auto X = (const bf16*)x; auto Wp = (const bf16*)W;
    if (nt == 1) {
        if (epi == EPI_BF16) return launch_mt<1, EPI_BF16>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper);
        if (epi == EPI_F32_PARTIAL) return launch_mt<1, EPI_F32_PARTIAL>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper);
        if (epi == EPI_SWIGLU) return launch_mt<1, EPI_SWIGLU>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper);
    } else {
        if (epi == EPI_BF16) return launch_mt<2, EPI_BF16>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper);
        if (epi == EPI_F32_PARTIAL) return launch_mt<2, EPI_F32_PARTIAL>(mt, grid, s, X, ldx, Wp, K, M, out, ldo, kper);
    }
    return (int)hipErrorInvalidValue;
}
