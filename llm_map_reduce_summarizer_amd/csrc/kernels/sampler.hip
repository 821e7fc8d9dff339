// Token sampler: Gumbel-max sampling at temperature
// tau (greedy argmax when tau <= 0) fused with the decode bookkeeping.
//
// sample:  grid (segments, B).  Each workgroup scans one vocabulary segment
//          of row b (16-B bf16 loads), adds Gumbel noise
//          g = -log(-log(u)), u = hash(seed_b, position_b, token) -- a
//          counter-based hash, so a sequence's samples do not depend on how
//          it was batched -- and folds (value, token) into one 64-bit key
//          (order-preserving float bits << 32 | ~token: ties -> lowest id)
//          that is atomicMax'ed into result[b].  Equivalent to sampling from
//          softmax(logits / tau) without a softmax or a sort.
// finish:  one lane per row: decode the winner, reset result[b] to 0 for
//          the next launch, append the token to out_tokens, feed it as the
//          next input id, advance the position, and retire the row on EOS or
//          max_new.  The stop ids are read from device memory at EVERY launch
//          (EOS_SLOTS ints, -1 = unused slot), never passed by value: a
//          captured decode graph then follows whatever stop set the engine
//          holds when it is replayed (generate(ignore_eos=True) writes -1s),
//          not the one it held when the graph was captured.  A retired row keeps its position, so a captured decode
//          graph can keep running it harmlessly until the host drops it.
// Tensor parallel (vocab-parallel LM head): each rank scans its vocab shard with
// tok_offset = rank * V_local -- the noise is a function of the GLOBAL token id, so the
// per-rank winners max-reduced across ranks (8 bytes per row, parallel/custom_ar.py) give the
// same token as one GPU scanning the whole row, without gathering the logits.
#include "common.h"

constexpr int EOS_SLOTS = 4;  // engine DecodeState.eos: 4 device ints, -1 = unused

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31;
    return x;
}

__device__ __forceinline__ unsigned int order_key(float v) {
    const unsigned int b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__global__ __launch_bounds__(256) void sample_kernel(const bf16* __restrict__ logits, int ld, int V, int tok_offset,
                                                     const float* __restrict__ temps,
                                                     const long long* __restrict__ seeds,
                                                     const int* __restrict__ positions,
                                                     unsigned long long* __restrict__ result, int seg_len) {
    __shared__ unsigned long long red[4];
    const int b = blockIdx.y;
    const float tau = temps[b];
    const float inv_tau = tau > 0.f ? 1.f / tau : 0.f;
    const unsigned long long key0 =
        mix64((unsigned long long)seeds[b] * 0x9E3779B97F4A7C15ULL + (unsigned long long)(positions[b] + 1));
    const int c0 = blockIdx.x * seg_len;
    const int c1 = min(V, c0 + seg_len);
    const bf16* row = logits + (size_t)b * ld;
    unsigned long long best = 0;
    for (int c = c0 + threadIdx.x * 8; c < c1; c += 256 * 8) {
        float f[8];
        if (c + 8 <= c1) {
            unpack8(*reinterpret_cast<const uint4*>(row + c), f);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = c + j < c1 ? (float)row[c + j] : -INFINITY;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int tok = tok_offset + c + j;
            float v = f[j];
            if (tau > 0.f) {
                const unsigned long long h = mix64(key0 ^ ((unsigned long long)tok * 0xD1B54A32D192ED03ULL));
                const float u = ((float)(h >> 40) + 0.5f) * (1.f / 16777216.f);
                v = v * inv_tau - __logf(-__logf(u));
            }
            const unsigned long long k =
                ((unsigned long long)order_key(v) << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned int)tok);
            if (c + j < c1 && k > best) best = k;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o, 64);
        best = other > best ? other : best;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = red[0];
        for (int i = 1; i < 4; ++i) m = red[i] > m ? red[i] : m;
        atomicMax(result + b, m);
    }
}

__global__ void sample_finish_kernel(unsigned long long* __restrict__ result, int* __restrict__ next_ids,
                                     int* __restrict__ positions, int* __restrict__ gen_count,
                                     const int* __restrict__ max_new, int* __restrict__ out_tokens, int out_stride,
                                     int* __restrict__ done, const int* __restrict__ eos, int B) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const unsigned long long r = result[b];
    result[b] = 0ULL;
    if (done[b]) return;
    const int tok = (int)(0xFFFFFFFFu - (unsigned int)(r & 0xFFFFFFFFULL));
    const int g = gen_count[b];
    out_tokens[(size_t)b * out_stride + g] = tok;
    gen_count[b] = g + 1;
    next_ids[b] = tok;
    bool stop = g + 1 >= max_new[b];
#pragma unroll
    for (int i = 0; i < EOS_SLOTS; ++i) stop |= tok == eos[i];  // tok >= 0 never matches a -1 slot
    if (stop) done[b] = 1;
    else positions[b] += 1;
}

static int launch_keys(const void* logits, int ld, int B, int V, int tok_offset, const float* temps,
                       const long long* seeds, const int* positions, void* result, hipStream_t s) {
    const int nseg = 32;
    int seg_len = ceil_div(V, nseg);
    seg_len = (seg_len + 7) & ~7;
    sample_kernel<<<dim3(nseg, B), 256, 0, s>>>((const bf16*)logits, ld, V, tok_offset, temps, seeds, positions,
                                                (unsigned long long*)result, seg_len);
    return (int)hipGetLastError();
}

// Gumbel-max keys of a (shard of the) vocabulary, max-folded into result[b] (which must be 0 or an
// earlier partial key).  Tensor-parallel callers max-reduce result across ranks, then finish.
MRSUM_API int mrsum_sample_keys(const void* logits, int ld, int B, int V, int tok_offset, const float* temps,
                                const long long* seeds, const int* positions, void* result, hipStream_t s) {
    if (B <= 0) return 0;
    return launch_keys(logits, ld, B, V, tok_offset, temps, seeds, positions, result, s);
}

MRSUM_API int mrsum_sample_finish(void* result, int* next_ids, int* positions_rw, int* gen_count, const int* max_new,
                                  int* out_tokens, int out_stride, int* done, const int* eos, int B,
                                  hipStream_t s) {
    if (B <= 0) return 0;
    sample_finish_kernel<<<ceil_div(B, 64), 64, 0, s>>>((unsigned long long*)result, next_ids, positions_rw,
                                                        gen_count, max_new, out_tokens, out_stride, done, eos, B);
    return (int)hipGetLastError();
}

MRSUM_API int mrsum_sample(const void* logits, int ld, int B, int V, const float* temps, const long long* seeds,
                           const int* positions, void* result, int* next_ids, int* positions_rw, int* gen_count,
                           const int* max_new, int* out_tokens, int out_stride, int* done, const int* eos,
                           hipStream_t s) {
    if (B <= 0) return 0;
    int e = launch_keys(logits, ld, B, V, 0, temps, seeds, positions, result, s);
    if (e) return e;
    sample_finish_kernel<<<ceil_div(B, 64), 64, 0, s>>>((unsigned long long*)result, next_ids, positions_rw,
                                                        gen_count, max_new, out_tokens, out_stride, done, eos, B);
    return (int)hipGetLastError();
}
