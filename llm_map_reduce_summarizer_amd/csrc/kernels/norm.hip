// RMSNorm and fused residual-add + RMSNorm.
//
//   rmsnorm:      out = x * rsqrt(mean(x^2) + eps) * w
//   add_rmsnorm:  residual = x + residual (stored bf16, the rounded value is
//                 what gets normalised); out = rmsnorm(residual) * w
//
// One 256-thread block per row; each lane holds VPT 16-byte vectors of the
// row in registers, so the row is read once and written once (memory bound:
// 2-3 x D x 2 bytes per row).  D % 8 == 0 and D <= 256*8*VPT.
//
// Q8 (the fp8 prefill GEMMs' input): the normalised row is quantised in the same pass -- row-wise
// dynamic OCP e4m3fn as quant.hip (scale = max|y| / 448, from the fp32 values) -- so neither the bf16
// normalised rows nor a separate quantisation pass over them exist.
// Q8 == 2 (two-term fp8, the QKV input of the fp8 model): the row is written as [hi | lo], 2 D bytes, on
// the same row scale: hi = e4m3(y / s), lo = e4m3((y / s - hi) x 16) -- the residual of the first rounding
// at 16x, inside e4m3's range since |y / s - hi| <= 16 (half an e4m3 step at 448).  The fp8 GEMM takes the
// pair as a 2K-deep product with the lo half scaled by 2^-4 through the MFMA's E8M0 block scale (gemm.hip),
// so x is carried to ~2^-8 relative precision: the attention scores computed from q / k stop amplifying
// e4m3's 2-3 % activation rounding (fp8 parity 24 % -> ~10 % rel L2, profiles/r4_fp8_activation_emulation.txt).
#include "common.h"

template <int VPT, bool ADD, int Q8 = 0>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16* __restrict__ x, bf16* __restrict__ residual,
                                                      const bf16* __restrict__ w, bf16* __restrict__ out,
                                                      int D, int x_stride, int out_stride, float eps,
                                                      float* __restrict__ qscale = nullptr) {
    __shared__ float red[16];
    const int row = blockIdx.x;
    const int nvec = D >> 3;
    const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * x_stride);
    uint4* rr = ADD ? reinterpret_cast<uint4*>(residual + (size_t)row * D) : nullptr;
    float v[VPT][8];
    const uint4* wr = reinterpret_cast<const uint4*>(w);
    uint4 wv[VPT];  // norm weights fetched up front, off the reduction's critical path
#pragma unroll
    for (int i = 0; i < VPT; ++i) wv[i] = wr[min((int)threadIdx.x + i * 256, nvec - 1)];
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + i * 256;
        if (c < nvec) {
            unpack8(xr[c], v[i]);
            if (ADD) {
                float r[8];
                unpack8(rr[c], r);
#pragma unroll
                for (int j = 0; j < 8; ++j) v[i][j] = (float)(bf16)(v[i][j] + r[j]);
                rr[c] = pack8(v[i]);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
        }
    }
    ss = block_sum(ss, red);
    const float inv = rsqrtf(ss / (float)D + eps);
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + i * 256;
        if (c < nvec) {
            float wf[8];
            unpack8(wv[i], wf);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] = v[i][j] * inv * wf[j];
            if constexpr (Q8) {
#pragma unroll
                for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
            } else {
                reinterpret_cast<uint4*>(out + (size_t)row * out_stride)[c] = pack8(v[i]);
            }
        }
    }
    if constexpr (Q8) {
        amax = wave_max(amax);
        __syncthreads();  // red[] of the sum above has been read by every wave
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
        __syncthreads();
        amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        const float sc = fmaxf(amax, 1e-12f) / 448.f, qi = 1.f / sc;
        if (threadIdx.x == 0) qscale[row] = sc;
        uint2* qr = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(out) + (size_t)row * out_stride);
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            const int c = threadIdx.x + i * 256;
            if (c < nvec) {
                float y[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) y[j] = v[i][j] * qi;
                int lo = 0, hi = 0;
                lo = __builtin_amdgcn_cvt_pk_fp8_f32(y[0], y[1], lo, false);
                lo = __builtin_amdgcn_cvt_pk_fp8_f32(y[2], y[3], lo, true);
                hi = __builtin_amdgcn_cvt_pk_fp8_f32(y[4], y[5], hi, false);
                hi = __builtin_amdgcn_cvt_pk_fp8_f32(y[6], y[7], hi, true);
                qr[c] = make_uint2((unsigned)lo, (unsigned)hi);
                if constexpr (Q8 == 2) {  // the second term: 16 x (y - e4m3(y)) on the same scale
                    float r[8];
                    const auto a0 = __builtin_amdgcn_cvt_pk_f32_fp8(lo, false), a1 = __builtin_amdgcn_cvt_pk_f32_fp8(lo, true);
                    const auto b0 = __builtin_amdgcn_cvt_pk_f32_fp8(hi, false), b1 = __builtin_amdgcn_cvt_pk_f32_fp8(hi, true);
                    r[0] = (y[0] - a0[0]) * 16.f; r[1] = (y[1] - a0[1]) * 16.f;
                    r[2] = (y[2] - a1[0]) * 16.f; r[3] = (y[3] - a1[1]) * 16.f;
                    r[4] = (y[4] - b0[0]) * 16.f; r[5] = (y[5] - b0[1]) * 16.f;
                    r[6] = (y[6] - b1[0]) * 16.f; r[7] = (y[7] - b1[1]) * 16.f;
                    int l2 = 0, h2 = 0;
                    l2 = __builtin_amdgcn_cvt_pk_fp8_f32(r[0], r[1], l2, false);
                    l2 = __builtin_amdgcn_cvt_pk_fp8_f32(r[2], r[3], l2, true);
                    h2 = __builtin_amdgcn_cvt_pk_fp8_f32(r[4], r[5], h2, false);
                    h2 = __builtin_amdgcn_cvt_pk_fp8_f32(r[6], r[7], h2, true);
                    qr[nvec + c] = make_uint2((unsigned)l2, (unsigned)h2);  // lo half starts at byte D
                }
            }
        }
    }
}

// Q8: ``out`` is e4m3fn [T, out_stride bytes] ([hi | lo], 2 D bytes, when Q8 == 2), ``qscale`` fp32 [T]
template <bool ADD, int Q8 = 0>
static int launch_rmsnorm(const void* x, void* residual, const void* w, void* out, int T, int D, int x_stride,
                          int out_stride, float eps, hipStream_t s, float* qscale = nullptr) {
    if (T <= 0) return 0;
    if (D % 8 || D > 256 * 8 * 8 || (Q8 && !qscale)) return (int)hipErrorInvalidValue;
    const int vpt = ceil_div(D / 8, 256);
    dim3 g(T), b(256);
    auto X = (const bf16*)x; auto R = (bf16*)residual; auto W = (const bf16*)w; auto O = (bf16*)out;
    if (vpt <= 1) rmsnorm_kernel<1, ADD, Q8><<<g, b, 0, s>>>(X, R, W, O, D, x_stride, out_stride, eps, qscale);
    else if (vpt <= 2) rmsnorm_kernel<2, ADD, Q8><<<g, b, 0, s>>>(X, R, W, O, D, x_stride, out_stride, eps, qscale);
    else if (vpt <= 4) rmsnorm_kernel<4, ADD, Q8><<<g, b, 0, s>>>(X, R, W, O, D, x_stride, out_stride, eps, qscale);
    else rmsnorm_kernel<8, ADD, Q8><<<g, b, 0, s>>>(X, R, W, O, D, x_stride, out_stride, eps, qscale);
    return (int)hipGetLastError();
}

// rmsnorm / residual-add + rmsnorm whose output rows are e4m3fn (q [T, ldq bytes]) with row scales [T];
// split: two-term rows [hi | lo] (2 D bytes, ldq >= 2 D)
MRSUM_API int mrsum_rmsnorm_fp8(const void* x, void* residual, const void* w, void* q, float* qscale, int T, int D,
                                int x_stride, int ldq, float eps, int split, hipStream_t s) {
    if (split) {
        if (ldq < 2 * D) return (int)hipErrorInvalidValue;
        if (residual) return launch_rmsnorm<true, 2>(x, residual, w, q, T, D, x_stride, ldq, eps, s, qscale);
        return launch_rmsnorm<false, 2>(x, nullptr, w, q, T, D, x_stride, ldq, eps, s, qscale);
    }
    if (residual) return launch_rmsnorm<true, 1>(x, residual, w, q, T, D, x_stride, ldq, eps, s, qscale);
    return launch_rmsnorm<false, 1>(x, nullptr, w, q, T, D, x_stride, ldq, eps, s, qscale);
}

MRSUM_API int mrsum_rmsnorm(const void* x, const void* w, void* out, int T, int D, int x_stride, int out_stride,
                            float eps, hipStream_t s) {
    return launch_rmsnorm<false>(x, nullptr, w, out, T, D, x_stride, out_stride, eps, s);
}

MRSUM_API int mrsum_add_rmsnorm(const void* x, void* residual, const void* w, void* out, int T, int D,
                                int x_stride, int out_stride, float eps, hipStream_t s) {
    return launch_rmsnorm<true>(x, residual, w, out, T, D, x_stride, out_stride, eps, s);
}

// residual += sum_s parts[s] (fp32 split-K slabs of the producing GEMM, [S, T, D]);
// out = rmsnorm(residual) * w.  The split-K reduction of the decode GEMMs
// (skinny_gemm EPI_F32_PARTIAL) is folded into this pass instead of costing
// its own kernel or atomics.
template <int VPT>
__global__ __launch_bounds__(256) void add_rmsnorm_parts_kernel(const float* __restrict__ parts, int S,
                                                                bf16* __restrict__ residual,
                                                                const bf16* __restrict__ w, bf16* __restrict__ out,
                                                                int T, int D, int out_stride, float eps) {
    __shared__ float red[16];
    const int row = blockIdx.x;
    const int nvec = D >> 3;
    uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * D);
    float v[VPT][8];
    float ss = 0.f;
    const uint4* wr = reinterpret_cast<const uint4*>(w);
    uint4 wv[VPT];  // norm weights fetched up front, off the reduction's critical path
#pragma unroll
    for (int i = 0; i < VPT; ++i) wv[i] = wr[min((int)threadIdx.x + i * 256, nvec - 1)];
    // every load of the first 4 slabs (and the residual) of all VPT vectors is issued before any is
    // consumed: one memory round trip for S <= 4 instead of one per vector
    uint4 rv[VPT];
    float4 a[VPT][4], bq[VPT][4];
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = min((int)threadIdx.x + i * 256, nvec - 1);
        rv[i] = rr[c];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4* p = reinterpret_cast<const float4*>(parts + ((size_t)min(u, S - 1) * T + row) * D + c * 8);
            a[i][u] = p[0];
            bq[i][u] = p[1];
        }
    }
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + i * 256;
        unpack8(rv[i], v[i]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (u < S) {
                v[i][0] += a[i][u].x; v[i][1] += a[i][u].y; v[i][2] += a[i][u].z; v[i][3] += a[i][u].w;
                v[i][4] += bq[i][u].x; v[i][5] += bq[i][u].y; v[i][6] += bq[i][u].z; v[i][7] += bq[i][u].w;
            }
        }
        if (c < nvec) {
            // slabs beyond the first 4 in batches of 4, all loads of a batch in flight together
            for (int s0 = 4; s0 < S; s0 += 4) {
                float4 x0[4], x1[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4* p = reinterpret_cast<const float4*>(
                        parts + ((size_t)min(s0 + u, S - 1) * T + row) * D + c * 8);
                    x0[u] = p[0];
                    x1[u] = p[1];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (s0 + u < S) {
                        v[i][0] += x0[u].x; v[i][1] += x0[u].y; v[i][2] += x0[u].z; v[i][3] += x0[u].w;
                        v[i][4] += x1[u].x; v[i][5] += x1[u].y; v[i][6] += x1[u].z; v[i][7] += x1[u].w;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] = (float)(bf16)v[i][j];
            rr[c] = pack8(v[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
        }
    }
    ss = block_sum(ss, red);
    const float inv = rsqrtf(ss / (float)D + eps);
    uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * out_stride);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + i * 256;
        if (c < nvec) {
            float wf[8];
            unpack8(wv[i], wf);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[i][j] = v[i][j] * inv * wf[j];
            orow[c] = pack8(v[i]);
        }
    }
}

MRSUM_API int mrsum_add_rmsnorm_parts(const void* parts, int S, void* residual, const void* w, void* out, int T,
                                      int D, int out_stride, float eps, hipStream_t s) {
    if (T <= 0) return 0;
    if (D % 8 || D > 256 * 8 * 8 || S < 1) return (int)hipErrorInvalidValue;
    const int vpt = ceil_div(D / 8, 256);
    auto P = (const float*)parts; auto R = (bf16*)residual; auto W = (const bf16*)w; auto O = (bf16*)out;
    if (vpt <= 1) add_rmsnorm_parts_kernel<1><<<T, 256, 0, s>>>(P, S, R, W, O, T, D, out_stride, eps);
    else if (vpt <= 2) add_rmsnorm_parts_kernel<2><<<T, 256, 0, s>>>(P, S, R, W, O, T, D, out_stride, eps);
    else if (vpt <= 4) add_rmsnorm_parts_kernel<4><<<T, 256, 0, s>>>(P, S, R, W, O, T, D, out_stride, eps);
    else add_rmsnorm_parts_kernel<8><<<T, 256, 0, s>>>(P, S, R, W, O, T, D, out_stride, eps);
    return (int)hipGetLastError();
}
