// Row-wise dynamic FP8 (OCP e4m3fn) quantisation of bf16 activations for the fp8 prefill GEMMs
// (gemm.hip's v_mfma_scale_f32_16x16x128_f8f6f4 path, per-row activation scales x per-output-row
// weight scales applied in its epilogue), and the matching row-wise weight quantiser used at load.
//
//   scale[r] = max(|x[r, :]|, tiny) / 448;  q[r, k] = e4m3fn(x[r, k] / scale[r])
//
// One 256-thread block per row, the row held in registers (16-B loads, VPT vectors per lane), so
// the row is read once: amax (block reduction) -> scale -> convert (v_cvt_pk_fp8_f32) -> 8-B store.
#include "common.h"

template <int VPT>
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16* __restrict__ x, int ldx,
                                                             uint8_t* __restrict__ q, float* __restrict__ scale,
                                                             int K) {
    __shared__ float red[16];
    const int row = blockIdx.x;
    const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * ldx);
    const int nvec = K >> 3;
    float v[VPT][8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + 256 * i;
        if (c < nvec) {
            unpack8(xr[c], v[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
        }
    }
    // block max
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float s = fmaxf(amax, 1e-12f) / 448.f;
    const float inv = 1.f / s;
    if (threadIdx.x == 0) scale[row] = s;
    uint2* qr = reinterpret_cast<uint2*>(q + (size_t)row * K);
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
        const int c = threadIdx.x + 256 * i;
        if (c < nvec) {
            int lo = 0, hi = 0;
            lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][0] * inv, v[i][1] * inv, lo, false);
            lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][2] * inv, v[i][3] * inv, lo, true);
            hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][4] * inv, v[i][5] * inv, hi, false);
            hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[i][6] * inv, v[i][7] * inv, hi, true);
            qr[c] = make_uint2((unsigned)lo, (unsigned)hi);
        }
    }
}

MRSUM_API int mrsum_quant_fp8_rows(const void* x, int ldx, void* q, float* scale, int T, int K, hipStream_t s) {
    if (T <= 0) return 0;
    if (K % 8 || K > 256 * 8 * 16) return (int)hipErrorInvalidValue;
    const int vpt = ceil_div(K / 8, 256);
    auto X = (const bf16*)x; auto Q = (uint8_t*)q;
    if (vpt <= 1) quant_fp8_rows_kernel<1><<<T, 256, 0, s>>>(X, ldx, Q, scale, K);
    else if (vpt <= 2) quant_fp8_rows_kernel<2><<<T, 256, 0, s>>>(X, ldx, Q, scale, K);
    else if (vpt <= 4) quant_fp8_rows_kernel<4><<<T, 256, 0, s>>>(X, ldx, Q, scale, K);
    else if (vpt <= 8) quant_fp8_rows_kernel<8><<<T, 256, 0, s>>>(X, ldx, Q, scale, K);
    else quant_fp8_rows_kernel<16><<<T, 256, 0, s>>>(X, ldx, Q, scale, K);
    return (int)hipGetLastError();
}
