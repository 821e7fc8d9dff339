// Large-M bf16 GEMM, four-wave form:  C[M, N] = X[M, K] . W[N, K]^T  (prefill projections).
//
// The layout hipBLASLt picks for these shapes on gfx950 (profiles/r4_hipblaslt_kernel_choice.jsonl:
// MT256x256x64, MI16x16, 256-thread workgroups) re-derived in HIP: one 256 x 256 output tile per
// workgroup of 4 waves, one wave per SIMD, each wave 128 x 128 outputs = 8 x 8 blocks of
// v_mfma_f32_16x16x32_bf16 (256 accumulator registers: the AGPR file).  Per 32-k step a wave reads 8 X
// and 8 W fragments (ds_read_b128) for 64 MFMAs -- 0.25 reads per MFMA against gemm.hip's 0.375 -- and
// the workgroup passes ONE barrier, where gemm.hip's 8-wave schedule passes two per phase.
//
//   * LDS ring of NS slots, one 32-k step each: X rows 0-255 then W rows 0-255, 64 B per row (32 KiB).
//     Steps arrive by LDS-DMA (buffer_load ... lds, 16 B per lane, 1 KiB = 16 rows per wave instruction,
//     8 per lane per step) from tile-local buffer descriptors (rows past M / N dropped by the range check).
//     Bank swizzle on the SOURCE address: 16-B chunk c of row r sits at position c ^ (((r >> 2) & 1) << 1),
//     which makes every fragment read conflict-free (each 16-lane group of a ds_read_b128 covers the 16
//     slots of a bank row; found by exhaustive search over the lane groups of MI355X_MICROARCH.md §LDS).
//   * step t: wait until step t + 1 has landed (counted vmcnt, never 0 in the steady state) and this
//     wave's reads of step t are retired (lgkmcnt(0)); barrier -- now every wave is done with slot t and
//     step t + 1 is visible; restage slot t with step t + NS (NS - 1 steps = NS - 1 x 64 MFMA issues of
//     prefetch distance); then 64 MFMAs on step t's fragments (registers) interleaved with the 16
//     fragment reads of step t + 1 into the other register set (sched_group_barrier).
//   * epilogue: transposed tile (A = W fragment), so a lane holds 4 consecutive output columns of one row;
//     LDS-staged whole-row stores; SwiGLU of the [8 gate | 8 up] rows in the store pass.
#include "common.h"

namespace {
constexpr int SLOT = 2 * 256 * 64;  // one 32-k step: X rows 0-255, W rows 0-255, 64 B each

struct G4Args {
    const char* x;
    const char* w;
    void* c;
    int ldx_b, ldw_b, ldc;  // X / W row strides in bytes, C row stride in elements
    int M, N, nk;           // nk = 32-k steps
    int tiles_m, tiles_n, group_m;
};

typedef __attribute__((address_space(3))) void* lds_ptr4_t;

__device__ __forceinline__ void dma16w(__amdgpu_buffer_rsrc_t r, char* dst, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr4_t)dst, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void vmw() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void vmw_rt(int steps) {  // wait until at most ``steps`` staged steps are in flight
    if (steps >= 3) vmw<24>();  // (more allowed is never assumed: fewer in flight is always safe)
    else if (steps == 2) vmw<16>();
    else if (steps == 1) vmw<8>();
    else vmw<0>();
}

__device__ __forceinline__ void bar4() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// bijective XCD remap then a grouped raster (gemm.hip tile_of)
__device__ __forceinline__ void tile_of4(int bid, int nwg, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
    const int xcd = bid & 7, local = bid >> 3, q = nwg >> 3, r = nwg & 7;
    const int p = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
    const int gsz = group_m * tiles_n;
    const int g = p / gsz, first = g * group_m;
    const int gm = min(tiles_m - first, group_m);
    const int within = p - g * gsz;
    tm = first + within % gm;
    tn = within / gm;
}
}  // namespace

// G4_LAG: MFMAs between a fragment register's last reader and the LDS read that refills it (0 or 4)
template <int EPI, int NS, bool LEPI, int G4_LAG>
__global__ __launch_bounds__(256, 1) void gemm4w_kernel(const G4Args a) {
    static_assert(NS >= 4 && NS * SLOT <= 160 * 1024, "LDS ring");
    __shared__ __attribute__((aligned(1024))) char lds[NS * SLOT];
    // an AGPR named in inline asm keeps the compiler from inferring "no AGPRs" for this kernel, so the MFMAs
    // are selected with their C / D in the AGPR file (256 accumulators); with the VGPR form the 256 acc + 128
    // fragment registers do not fit the 256 VGPRs and spill to scratch
    asm volatile("" ::: "a255");
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 1, wc = w & 1;
    int tm, tn;
    tile_of4(blockIdx.x, gridDim.x, a.tiles_m, a.tiles_n, a.group_m, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int xrows = min(a.M - m0, 256), wrows = min(a.N - n0, 256);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.x + (size_t)m0 * a.ldx_b), (short)0, xrows * a.ldx_b, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.w + (size_t)n0 * a.ldw_b), (short)0, wrows * a.ldw_b, 0x00020000);
    const int nk = a.nk;

    // staging: wave w fills X rows and W rows 64 w .. 64 w + 63, four 16-row pieces each; lane = (row 0..15 of
    // the piece, LDS position lane & 3), whose source chunk is position ^ f(row)
    const int prow = lane >> 2;
    const int sch = ((lane & 3) ^ (((prow >> 2) & 1) << 1)) << 4;
    const int vx = (64 * w + prow) * a.ldx_b + sch, vw = (64 * w + prow) * a.ldw_b + sch;
    const int px = 16 * a.ldx_b, pw = 16 * a.ldw_b;
    auto stage = [&](int t) {
        char* s = lds + (t % NS) * SLOT + 64 * w * 64;
        const int soff = t * 64;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            dma16w(rx, s + j * 1024, vx + j * px, soff);
            dma16w(rw, s + 16384 + j * 1024, vw + j * pw, soff);
        }
    };

    // fragment reads: 16-row block at row r0 of a slot image, lane = (row lane & 15, k chunk lane >> 4)
    const int r16 = lane & 15;
    const int lo = r16 * 64 + (((lane >> 4) ^ (((r16 >> 2) & 1) << 1)) << 4);
    const int xoff = (128 * wr) * 64 + lo, woff = 16384 + (128 * wc) * 64 + lo;

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[i][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 xf[8], wf[8];  // ONE fragment set, refilled in place (two sets made the allocator rotate the accumulators)

    // prologue: steps 0 .. NS-2 in flight, wait for step 0, read its fragments
#pragma unroll
    for (int t = 0; t < NS - 1; ++t)
        if (t < nk) stage(t);
    vmw_rt(min(NS - 1, nk) - 1);  // step 0 landed
    bar4();
    // (in the order the loop refills them: the waitcnt pass then sees one outstanding-read order at the loop head)
#pragma unroll
    for (int j = 0; j < 4; ++j) xf[j] = *reinterpret_cast<const u32x4*>(lds + xoff + j * 1024);
#pragma unroll
    for (int j = 0; j < 8; ++j) wf[j] = *reinterpret_cast<const u32x4*>(lds + woff + j * 1024);
#pragma unroll
    for (int j = 4; j < 8; ++j) xf[j] = *reinterpret_cast<const u32x4*>(lds + xoff + j * 1024);

    // step t: wait for step t + 1 (the steps staged after it may stay in flight), barrier, restage the slot of step
    // t - 1 (its fragments were consumed by step t - 1's MFMAs) with step t + NS - 1, then the 64 MFMAs of step t,
    // each fragment register refilled with step t + 1's fragment right after its last MFMA issued.  Order: X blocks
    // 0-3 against all W blocks first (X 0-3 refilled early), then W-major over X blocks 4-7 (each W block refilled
    // as it finishes, X 4-7 at the end) -- the next step starts on X 0-3 and W 0.., which were refilled 7 or more
    // MFMAs earlier, and the in-order LDS counter lets its first MFMAs wait only for those.  The last step reads a
    // stale slot into registers nothing uses.
#define G4_MFMA(i, b) acc[i][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[i]),       \
                                                                        __builtin_bit_cast(bf16x8, xf[b]), acc[i][b], 0, 0, 0);
#define G4_STEP(T)                                                                                          \
    {                                                                                                      \
        const int t_ = (T);                                                                                \
        vmw_rt(min(t_ + NS - 2, nk - 1) - (t_ + 1));                                                       \
        bar4();                                                                                            \
        if (t_ + NS - 1 < nk) stage(t_ + NS - 1);                                                          \
        const char* s = lds + ((t_ + 1) % NS) * SLOT;                                                      \
        _Pragma("unroll") for (int b = 0; b < 4; ++b) {                                                    \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) { G4_MFMA(i, b) }                                \
            xf[b] = *reinterpret_cast<const u32x4*>(s + xoff + b * 1024);                                  \
        }                                                                                                  \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                    \
            _Pragma("unroll") for (int b = 4; b < 8; ++b) { G4_MFMA(i, b) }                                \
            wf[i] = *reinterpret_cast<const u32x4*>(s + woff + i * 1024);                                  \
        }                                                                                                  \
        _Pragma("unroll") for (int b = 4; b < 8; ++b)                                                      \
            xf[b] = *reinterpret_cast<const u32x4*>(s + xoff + b * 1024);                                  \
        /* keep the refills between the MFMAs (hipcc otherwise sinks all 16 reads below the last MFMA); with  \
           G4_LAG = 4 each refill issues 4 MFMAs after the last MFMA that reads the register it overwrites */  \
        if constexpr (G4_LAG == 4) {                                                                       \
            __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);                                            \
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                             \
            _Pragma("unroll") for (int b = 1; b < 4; ++b) {                                                \
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                                         \
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
            }                                                                                              \
            _Pragma("unroll") for (int k = 0; k < 7; ++k) {                                                \
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                         \
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
            }                                                                                              \
            __builtin_amdgcn_sched_group_barrier(0x100, 5, 0);                                             \
        } else {                                                                                           \
            _Pragma("unroll") for (int b = 0; b < 4; ++b) {                                                \
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                                         \
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
            }                                                                                              \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) {                                                \
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);                                         \
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                         \
            }                                                                                              \
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                                             \
        }                                                                                                  \
    }
    for (int t = 0; t < nk; ++t) G4_STEP(t)
#undef G4_STEP
#undef G4_MFMA

    // epilogue: every wave writes its 128 x 128 bf16 results into a [256 rows][512 B] LDS image of the tile
    // (16-B unit u of row r at u ^ (r & 7): conflict-free), then each wave stores 64 whole rows.  SwiGLU is applied
    // in the store pass from the image's [8 gate | 8 up] units -- gate and up are rounded to bf16 first (gemm.hip
    // applies it to the fp32 accumulators; an in-register lane exchange here kept all 256 accumulators live and
    // spilled).  LEPI: 16-B stores; else the 8-B aligned output takes two 8-B stores per unit.
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    constexpr int RB = 512;
    const int g4 = lane >> 4;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int rl = 128 * wr + 16 * b + (lane & 15);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int cbyte = (128 * wc + 16 * i + 4 * g4) * 2;
            const f32x4 v = acc[i][b];
            const uint2 pk = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
            *reinterpret_cast<uint2*>(lds + rl * RB + (((cbyte >> 4) ^ (rl & 7)) << 4) + (cbyte & 15)) = pk;
        }
    }
    __syncthreads();
    constexpr int UNITS = EPI == 1 ? 16 : 32;  // output 16-B units per tile row
    constexpr int RPI = 64 / UNITS;           // rows per wave instruction
    const int u = lane % UNITS;
    const int col = (EPI == 1 ? (n0 >> 1) : n0) + 8 * u;  // first output column of the unit
    const bool cok = (EPI == 1 ? 2 * col : col) < a.N;
#pragma unroll
    for (int it0 = 0; it0 < 64 / RPI; it0 += 8) {  // 8 rows in flight, then their stores
        u32x4 val[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int rl = 64 * w + RPI * (it0 + j) + lane / UNITS;
            if constexpr (EPI == 1) {
                const u32x4 gv = *reinterpret_cast<const u32x4*>(lds + rl * RB + (((2 * u) ^ (rl & 7)) << 4));
                const u32x4 uv = *reinterpret_cast<const u32x4*>(lds + rl * RB + (((2 * u + 1) ^ (rl & 7)) << 4));
                float g[8], up[8], r[8];
                unpack8(make_uint4(gv[0], gv[1], gv[2], gv[3]), g);
                unpack8(make_uint4(uv[0], uv[1], uv[2], uv[3]), up);
#pragma unroll
                for (int e = 0; e < 8; ++e) r[e] = g[e] / (1.f + __expf(-g[e])) * up[e];
                const uint4 o = pack8(r);
                val[j] = u32x4{o.x, o.y, o.z, o.w};
            } else {
                val[j] = *reinterpret_cast<const u32x4*>(lds + rl * RB + ((u ^ (rl & 7)) << 4));
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int m = m0 + 64 * w + RPI * (it0 + j) + lane / UNITS;
            if (!cok || m >= a.M) continue;
            bf16* o = reinterpret_cast<bf16*>(a.c) + (size_t)m * a.ldc + col;
            if constexpr (LEPI) {
                *reinterpret_cast<u32x4*>(o) = val[j];
            } else {
                reinterpret_cast<uint2*>(o)[0] = make_uint2(val[j][0], val[j][1]);
                reinterpret_cast<uint2*>(o)[1] = make_uint2(val[j][2], val[j][3]);
            }
        }
    }
}

// Same contract as mrsum_gemm's bf16 path (epi 0 plain, 1 SwiGLU of the [8 gate | 8 up] rows): x [M, K] (ldx
// elements), w [N, K] (ldw), c (ldc).  K % 64 == 0 (an even count of 32-k steps), N % 16 == 0, 16-byte aligned rows.  ns: LDS ring steps (4 or 5) | 256 for the lagged refill schedule.
MRSUM_API int mrsum_gemm4w(const void* x, int ldx, const void* w, int ldw, void* c, int ldc, int M, int N, int K,
                           int epi, int group_m, int ns, hipStream_t s) {
    const int lag = (ns >> 8) & 1 ? 4 : 0;  // bit 8: refills 4 MFMAs after their registers' last reader
    ns &= 255;
    if (M <= 0 || N <= 0) return 0;
    if (K % 64 || N % 16 || ldx % 8 || ldw % 8 || ldc % 4 || (epi != 0 && epi != 1) || (ns != 4 && ns != 5))
        return (int)hipErrorInvalidValue;
    if ((size_t)256 * ldx * 2 >= (1u << 31) || (size_t)256 * ldw * 2 >= (1u << 31)) return (int)hipErrorInvalidValue;
    G4Args a;
    a.x = (const char*)x; a.w = (const char*)w; a.c = c;
    a.ldx_b = ldx * 2; a.ldw_b = ldw * 2; a.ldc = ldc;
    a.M = M; a.N = N; a.nk = K / 32;
    a.tiles_m = ceil_div(M, 256); a.tiles_n = ceil_div(N, 256);
    a.group_m = group_m > 0 ? group_m : 4;
    const dim3 grid(a.tiles_m * a.tiles_n), block(256);
    const bool lepi = ldc % 8 == 0 && (uintptr_t)c % 16 == 0;
#define G4_LAUNCH(E, NS_, L)                                                    \
    if (lepi) gemm4w_kernel<E, NS_, true, L><<<grid, block, 0, s>>>(a);          \
    else gemm4w_kernel<E, NS_, false, L><<<grid, block, 0, s>>>(a);
#define G4_BY_LAG(E, NS_) if (lag) { G4_LAUNCH(E, NS_, 4) } else { G4_LAUNCH(E, NS_, 0) }
    if (ns == 4) {
        if (epi == 1) { G4_BY_LAG(1, 4) } else { G4_BY_LAG(0, 4) }
    } else {
        if (epi == 1) { G4_BY_LAG(1, 5) } else { G4_BY_LAG(0, 5) }
    }
#undef G4_BY_LAG
#undef G4_LAUNCH
    return (int)hipGetLastError();
}
