// Large-M GEMM on the matrix cores (prefill projections, LM head over many rows):
//
//     C[M, N] = X[M, K] . W[N, K]^T            X = activations, W = weights, both K-contiguous
//
//   * bf16 x bf16 on v_mfma_f32_16x16x32_bf16, or
//   * OCP e4m3fn x e4m3fn on v_mfma_scale_f32_16x16x128_f8f6f4 with unit block scales (E8M0 127): the
//     block-scaled form runs at twice the bf16 rate (MI355X_MICROARCH.md "Matrix cores"), so the plain
//     per-row quantisation (activation row scale sx[m] x weight row scale sw[n]) is applied in the
//     epilogue and the MX block scales stay 1.0.  (Per-32 E8M0 activation scales measured WORSE than the
//     fp32 row scale: power-of-two scales waste up to a bit of e4m3's range -- 2.67 vs 2.29 % element
//     error, 25.6 vs 24.3 % on the fp8 parity logits, profiles/r4_fp8_activation_emulation.txt.)
//   * two-term fp8 activations (norm.hip Q8 == 2, the fp8 model's QKV input): X rows hold [hi | lo] over
//     2K bytes, W keeps K; the K-tiles kt >= kbw (the lo half) re-read W's tile kt - kbw and run with the
//     X block scale E8M0 123 = 2^-4, so one launch computes hi W^T + lo W^T / 16.
//
// Structure (cdna_hip_programming.md §5 "The 256^2 8-phase template", re-derived for this layout):
//   * one 256 x 256 output tile per 512-thread workgroup (8 waves, one workgroup per CU), K-tiles of 128
//     bytes per row (64 bf16 | 128 e4m3); the XCD-aware bijective tile remap + grouped raster keeps
//     the ~32 tiles an XCD runs at a time on 4 X row-panels x 8 W row-panels (L2 reuse).
//   * LDS: 2 buffers x 4 half-tile images of 128 rows x 128 B (X rows 0-127, W rows 0-127, W rows
//     128-255, X rows 128-255 -- the order the phases first read them) = 128 KiB in ONE __shared__
//     array.  Half-tiles arrive by LDS-DMA (buffer_load ... lds, 16 B per lane, one 1 KiB piece = 8
//     rows per wave instruction) from a tile-local buffer descriptor: rows past M / N are dropped by
//     the descriptor's range check (their LDS rows hold stale bytes that only feed masked outputs).
//     The bank swizzle is applied on the SOURCE address (rule 21): 16-B chunk c of row r sits at
//     chunk position c ^ ((r >> 1) & 7), which makes every ds_read_b128 fragment read conflict-free
//     (each 16-lane group covers the 16 slots of a bank row).
//   * wave (wr, wc) owns 128 x 64 outputs split into four 64 x 32 quadrants; quadrant (qm, qn) reads
//     X half qm and W half qn, so the four phases of a K-tile need the half-tiles in the order
//     X0 W0 | W1 | X1 | -- and a half-tile can be staged LOOK = 6 half-tiles (1.5 K-tiles) ahead of
//     the phase that first reads it.  Per phase: R = fragment ds_reads + stage one half-tile (2 DMA
//     per lane) + counted s_waitcnt vmcnt(8) (never 0 in the main loop), raw s_barrier, M = 16 bf16 (8
//     fp8) MFMAs between s_setprio(1/0), raw s_barrier.  Waves 4-7 run one barrier (half a phase)
//     behind waves 0-3 (stagger), so one wave of each SIMD reads LDS while its partner computes.
//   * hazards (derived for the staggered schedule, which is the stricter one): the wait at the end of
//     R_P covers every half-tile phase P+1 reads, before the barrier the lagging group passes ahead
//     of its R_P; a half-tile is restaged >= 2 phases after the last phase that read its region
//     (reads are retired by the lgkmcnt wait ahead of that phase's MFMAs, which precede the barrier
//     the restaging wave passes).
//   * the MFMA computes the transposed tile (A = W fragment, B = X fragment) so each lane ends with 4
//     consecutive output columns of one row: 8-byte bf16 stores, and the fused SwiGLU epilogue of the
//     [8 gate | 8 up]-interleaved gate_up weight is a lane-xor-32 exchange.
//   * M32 variant: the same ring, phases and quadrants on 32x32 MFMA tiles (v_mfma_f32_32x32x16_bf16 /
//     v_mfma_scale_f32_32x32x64_f8f6f4); a lane then holds 4 register groups of 4 consecutive columns,
//     and the SwiGLU gate / up halves of a 16-column group sit in adjacent groups of the same lane.
#include "common.h"

#include <type_traits>

namespace {
constexpr int HALF = 16384;
constexpr int TILE = 4 * HALF;
constexpr int LOOK = 6;

enum { GEPI_BF16 = 0, GEPI_SWIGLU = 1 };

typedef int i32x8 __attribute__((ext_vector_type(8)));

struct GemmArgs {
    const char* x;
    const char* w;
    void* c;
    const float* sx;  // fp8: per-row activation scale [M]
    const float* sw;  // fp8: per-row weight scale [N]
    int ldx_b, ldw_b, ldc;  // X / W row strides in bytes, C row stride in elements
    int M, N, kb;           // kb = K-tiles (128 bytes of every row each)
    int kbw;                // W's K-tiles: kb, or kb / 2 for two-term X (X tiles kt >= kbw re-read W tile kt - kbw)
    int tiles_m, tiles_n, group_m;
#ifdef MRSUM_CLOCK_STAMPS
    unsigned long long* stamps;  // diagnostic build only (tools/gemm_clock.py): [grid][2] shader / 100 MHz ticks
#endif
};

template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void vm_wait_rt(int n) {
    if (n >= 12) vm_wait<12>();
    else if (n >= 10) vm_wait<10>();
    else if (n >= 8) vm_wait<8>();
    else if (n >= 6) vm_wait<6>();
    else if (n >= 4) vm_wait<4>();
    else if (n >= 2) vm_wait<2>();
    else vm_wait<0>();
}

__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* dst, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, voff, soff, 0, 0);
}

// bijective XCD remap (blocks b, b+8, ... share an XCD) then a grouped raster of group_m tile rows
__device__ __forceinline__ void tile_of(int bid, int nwg, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
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

template <bool FP8, int EPI, int NS, bool LEPI, bool M32>
__global__ __launch_bounds__(512, 1) void gemm_kernel(const GemmArgs a) {
    // NS = half-tile slots of the LDS ring: half-tile h (K-tile h / 4, part h % 4) lives in slot h % NS.
    // NS = 8 (128 KiB, 2 K-tiles): staged LK = 6 ahead; NS = 10 (160 KiB): LK = 8 ahead.  A slot is
    // restaged at phase h + NS - LK >= 2 phases after the last phase that read half-tile h (<= h).
    constexpr int LK = NS - 2;
    static_assert(NS * HALF <= 160 * 1024 && NS * HALF >= 2 * TILE, "LDS ring size");
#ifdef MRSUM_CLOCK_STAMPS
    const unsigned long long clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    __shared__ __attribute__((aligned(1024))) char lds[NS * HALF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    int tm, tn;
    tile_of(blockIdx.x, gridDim.x, a.tiles_m, a.tiles_n, a.group_m, tm, tn);
    const int m0 = tm * 256, n0 = tn * 256;
    const int xrows = min(a.M - m0, 256), wrows = min(a.N - n0, 256);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.x + (size_t)m0 * a.ldx_b), (short)0, xrows * a.ldx_b, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.w + (size_t)n0 * a.ldw_b), (short)0, wrows * a.ldw_b, 0x00020000);

    // staging: this lane's source offsets for the 2 pieces (8 rows each) of every half-tile it fills
    const int srow = 16 * w + (lane >> 3);
    const int ch0 = ((lane & 7) ^ ((lane >> 4) & 7)) << 4;
    const int ch1 = ((lane & 7) ^ ((4 + (lane >> 4)) & 7)) << 4;
    const int vx0 = srow * a.ldx_b + ch0, vx1 = (srow + 8) * a.ldx_b + ch1;
    const int vw0 = srow * a.ldw_b + ch0, vw1 = (srow + 8) * a.ldw_b + ch1;
    const int xh = 128 * a.ldx_b, wh = 128 * a.ldw_b;
    const int nk = a.kb, htot = 4 * nk;

    auto stage = [&](int part, int kt) {
        char* dst = lds + ((4 * kt + part) % NS) * HALF + w * 2048;
        const int soff = kt * 128;
        if (part == 0 || part == 3) {
            const int o = part == 3 ? xh : 0;
            dma16(rx, dst, vx0 + o, soff);
            dma16(rx, dst + 1024, vx1 + o, soff);
        } else {
            const int o = part == 2 ? wh : 0;
            const int sw = (kt >= a.kbw ? kt - a.kbw : kt) * 128;
            dma16(rw, dst, vw0 + o, sw);
            dma16(rw, dst + 1024, vw1 + o, sw);
        }
    };

    // fragment reads.  16x16 MFMA: row (lane & 15) of a 16-row block, chunk (lane >> 4) (k-step 0) or
    // 4 + (lane >> 4).  32x32 MFMA (M32): row (lane & 31) of a 32-row block, read r = chunk 2 r + (lane >> 5);
    // any k order shared by the A and B operands gives the same dot product, and each ds_read_b128 lane
    // group still covers 16 distinct slots of a bank row (rows r, r + 1 share the swizzle, 8 slots apart).
    int lo[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
        lo[r] = M32 ? (lane & 31) * 128 + (((2 * r + (lane >> 5)) ^ ((lane >> 1) & 7)) << 4)
                    : (lane & 15) * 128 + (((4 * (r & 1) + (lane >> 4)) ^ ((lane >> 1) & 7)) << 4);
    const int xbase = (64 * wr) * 128, wbase = (32 * wc) * 128;

    // per quadrant: 16x16 -- [x block b 0..3][w block i 0..1] f32x4; 32x32 -- [x block b 0..1] f32x16
    f32x4 acc[2][4][2][2];
    f32x16 acc32[2][2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    if constexpr (M32) { if (b < 2 && k == 0) acc32[i][b][j] = f32x16{}; }
                    else acc[i][b][j][k] = f32x4{0.f, 0.f, 0.f, 0.f};
                }
    // xf[2 b + ks] (16x16) | xf[4 b + r] (32x32); wf[2 i + ks] | wf[r]
    u32x4 xf[8], wf0[4], wf1[4];

    // prologue: half-tiles 0 .. LK-1 in flight, wait for the phase 0 reads (h <= 1 | h <= 2)
#pragma unroll
    for (int h = 0; h < LK; ++h)
        if (h < htot) stage(h & 3, h >> 2);
    vm_wait_rt(2 * (min(LK - 1, htot - 1) - 1));
    bar();
    if (wr == 1) bar();  // stagger: waves 4-7 run one barrier (half a phase) behind waves 0-3

    // 16x16: block b (16 rows) read ks at b * 2048 + lo[ks];  32x32: block b (32 rows) read r at b * 4096 + lo[r]
    auto read_x = [&](const char* base) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            xf[j] = *reinterpret_cast<const u32x4*>(base + xbase + (M32 ? (j >> 2) * 4096 + lo[j & 3]
                                                                        : (j >> 1) * 2048 + lo[j & 1]));
    };
    auto read_w = [&](const char* base, u32x4 (&wf)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            wf[j] = *reinterpret_cast<const u32x4*>(base + wbase + (M32 ? lo[j] : (j >> 1) * 2048 + lo[j & 1]));
    };
    auto cat8 = [](const u32x4& p, const u32x4& q) -> i32x8 {
        return i32x8{(int)p[0], (int)p[1], (int)p[2], (int)p[3], (int)q[0], (int)q[1], (int)q[2], (int)q[3]};
    };
    auto mfma_q = [&](int qm, int qn, const u32x4 (&wf)[4], int xsc) {
        __builtin_amdgcn_s_setprio(1);
        if constexpr (M32) {
            if constexpr (FP8) {
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc32[qm][b][qn] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                            cat8(wf[2 * s], wf[2 * s + 1]), cat8(xf[4 * b + 2 * s], xf[4 * b + 2 * s + 1]),
                            acc32[qm][b][qn], 0, 0, 0, 127, 0, xsc);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc32[qm][b][qn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                            __builtin_bit_cast(bf16x8, wf[r]), __builtin_bit_cast(bf16x8, xf[4 * b + r]),
                            acc32[qm][b][qn], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    if constexpr (FP8) {
                        acc[qm][b][qn][i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                            cat8(wf[2 * i], wf[2 * i + 1]), cat8(xf[2 * b], xf[2 * b + 1]), acc[qm][b][qn][i],
                            0, 0, 0, 127, 0, xsc);
                    } else {
#pragma unroll
                        for (int ks = 0; ks < 2; ++ks)
                            acc[qm][b][qn][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                __builtin_bit_cast(bf16x8, wf[2 * i + ks]), __builtin_bit_cast(bf16x8, xf[2 * b + ks]),
                                acc[qm][b][qn][i], 0, 0, 0);
                    }
                }
        }
        __builtin_amdgcn_s_setprio(0);
    };
    // stage the half-tile LK ahead of phase P = 4 kt + p, then wait for what phase P + 1 reads.  In the
    // steady state (TAIL false: kt < nk - LK / 4) the stage always exists and the wait is vmcnt(2 (LK - 2)).
    auto stage_and_wait = [&](int kt, int p, auto tail) {
        const int P = 4 * kt + p, h = P + LK;
        if constexpr (decltype(tail)::value) {
            if (h < htot) stage(h & 3, h >> 2);
            const int rem = htot - 1 - P;
            vm_wait_rt(rem >= LK ? 2 * (LK - 2) : 2 * (rem - 2));
        } else {
            stage(h & 3, h >> 2);
            vm_wait<2 * (LK - 2)>();
        }
    };
    auto slot = [&](int kt, int part) -> const char* { return lds + ((4 * kt + part) % NS) * HALF; };
    auto ktile = [&](int kt, auto tail) {
        const int xsc = FP8 && kt >= a.kbw ? 123 : 127;  // E8M0 2^-4 on the lo half of two-term X
        // phase 0: quadrant (0, 0) -- X0, W0
        read_x(slot(kt, 0));
        read_w(slot(kt, 1), wf0);
        stage_and_wait(kt, 0, tail);
        bar();
        mfma_q(0, 0, wf0, xsc);
        bar();
        // phase 1: quadrant (0, 1) -- W1
        read_w(slot(kt, 2), wf1);
        stage_and_wait(kt, 1, tail);
        bar();
        mfma_q(0, 1, wf1, xsc);
        bar();
        // phase 2: quadrant (1, 1) -- X1
        read_x(slot(kt, 3));
        stage_and_wait(kt, 2, tail);
        bar();
        mfma_q(1, 1, wf1, xsc);
        bar();
        // phase 3: quadrant (1, 0) -- registers only
        stage_and_wait(kt, 3, tail);
        bar();
        mfma_q(1, 0, wf0, xsc);
        bar();
    };
    // steady state while every phase's stage exists: P + LK < htot for P <= 4 kt + 3
    int kt = 0;
    for (; kt < nk - (LK + 3) / 4; ++kt) ktile(kt, std::false_type{});
    for (; kt < nk; ++kt) ktile(kt, std::true_type{});
    if (wr == 0) bar();

    // epilogue: lane holds C[m][n .. n+3] of every 16 x 16 block, m = .. + (lane & 15), n = .. + 4 (lane >> 4).
    // LEPI: every wave writes its bf16 results into a [256 rows][RB bytes] LDS image of the whole tile
    // (16-B unit u of row r at u ^ (r & 7): 2-way ds_write_b64, conflict-free ds_read_b128), then each
    // wave stores 32 whole rows with 16-B lanes (full-row segments instead of 32-B pieces per row).
    constexpr int RB = EPI == GEPI_SWIGLU ? 256 : 512;
    // fp8: v *= activation row scale x weight row scales of tile columns c4 .. c4+3
    auto scale4 = [&](f32x4& v, float rs, int c4) {
        if constexpr (FP8) {
            const float4 s4 = *reinterpret_cast<const float4*>(a.sw + min(n0 + c4, a.N - 4));
            v[0] *= rs * s4.x; v[1] *= rs * s4.y; v[2] *= rs * s4.z; v[3] *= rs * s4.w;
        }
    };
    auto silu_mul = [](const f32x4& g, const f32x4& u) {
        f32x4 r;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
        return r;
    };
    // 4 bf16 outputs of tile row rl at byte cbyte of the output tile row; gcol = first weight column of
    // the 16-column group they come from (N % 16 == 0, so the group is wholly in or out of range)
    auto store4 = [&](int rl, int cbyte, const f32x4& v, int gcol) {
        const uint2 pk = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
        if constexpr (LEPI) {
            *reinterpret_cast<uint2*>(lds + rl * RB + (((cbyte >> 4) ^ (rl & 7)) << 4) + (cbyte & 15)) = pk;
        } else if (m0 + rl < a.M && n0 + gcol < a.N) {
            char* o = reinterpret_cast<char*>(a.c) + ((size_t)(m0 + rl) * a.ldc) * 2 +
                      (EPI == GEPI_SWIGLU ? n0 : 2 * n0) + cbyte;
            *reinterpret_cast<uint2*>(o) = pk;
        }
    };
    if constexpr (M32) {
        // lane holds C[m][n .. n+3] of every 32 x 32 block: m = .. + (lane & 31), register group gi covers
        // n = .. + 8 gi + 4 (lane >> 5).  SwiGLU: groups 0 / 2 are gate, 1 / 3 the matching up columns.
        const int h = lane >> 5;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int rl = 128 * qm + 64 * wr + 32 * b + (lane & 31);
                float rs = 1.f;
                if constexpr (FP8) rs = a.sx[min(m0 + rl, a.M - 1)];
#pragma unroll
                for (int qn = 0; qn < 2; ++qn) {
                    const int cb = 128 * qn + 32 * wc;
                    f32x4 v[4];
#pragma unroll
                    for (int gi = 0; gi < 4; ++gi) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) v[gi][t] = acc32[qm][b][qn][4 * gi + t];
                        scale4(v[gi], rs, cb + 8 * gi + 4 * h);
                    }
                    if constexpr (EPI == GEPI_SWIGLU) {
#pragma unroll
                        for (int gp = 0; gp < 2; ++gp) {
                            const int gcol = cb + 16 * gp;
                            store4(rl, ((gcol >> 1) + 4 * h) * 2, silu_mul(v[2 * gp], v[2 * gp + 1]), gcol);
                        }
                    } else {
#pragma unroll
                        for (int gi = 0; gi < 4; ++gi) {
                            const int c4 = cb + 8 * gi + 4 * h;
                            store4(rl, c4 * 2, v[gi], c4);
                        }
                    }
                }
            }
    } else {
        // lane holds C[m][n .. n+3] of every 16 x 16 block, m = .. + (lane & 15), n = .. + 4 (lane >> 4).
        // SwiGLU: the up columns 8-15 of a 16-column group sit in lane xor 32.
        const int g4 = lane >> 4;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int rl = 128 * qm + 64 * wr + 16 * b + (lane & 15);
                float rs = 1.f;
                if constexpr (FP8) rs = a.sx[min(m0 + rl, a.M - 1)];
#pragma unroll
                for (int qn = 0; qn < 2; ++qn)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        const int cb = 128 * qn + 32 * wc + 16 * i;  // 16-column block within the tile
                        f32x4 v = acc[qm][b][qn][i];
                        scale4(v, rs, cb + 4 * g4);
                        if constexpr (EPI == GEPI_SWIGLU) {
                            f32x4 up;
#pragma unroll
                            for (int j = 0; j < 4; ++j) up[j] = __shfl_xor(v[j], 32, 64);
                            if (g4 < 2) store4(rl, ((cb >> 1) + 4 * g4) * 2, silu_mul(v, up), cb);
                        } else {
                            store4(rl, (cb + 4 * g4) * 2, v, cb);
                        }
                    }
            }
    }
    if constexpr (LEPI) {
        __syncthreads();
        constexpr int UPR = RB / 16, RPI = 1024 / RB;
#pragma unroll
        for (int it = 0; it < 32 / RPI; ++it) {
            const int rl = 32 * w + RPI * it + lane / UPR, u = lane % UPR;
            const u32x4 val = *reinterpret_cast<const u32x4*>(lds + rl * RB + ((u ^ (rl & 7)) << 4));
            const int m = m0 + rl;
            const int col = (EPI == GEPI_SWIGLU ? (n0 >> 1) : n0) + 8 * u;  // output column of the unit
            const bool ok = m < a.M && (EPI == GEPI_SWIGLU ? 2 * col : col) < a.N;
            if (ok) *reinterpret_cast<u32x4*>(reinterpret_cast<bf16*>(a.c) + (size_t)m * a.ldc + col) = val;
        }
    }
#ifdef MRSUM_CLOCK_STAMPS
    // in-kernel clock = shader ticks / 100 MHz ticks (MI355X_MICROARCH.md, DVFS give-back item 6); lane 0's
    // vector store to a buffer no other code reads
    __syncthreads();
    if (tid == 0) {
        const unsigned long long clk = __builtin_amdgcn_s_memtime() - clk0, rt = __builtin_amdgcn_s_memrealtime() - rt0;
        a.stamps[2 * blockIdx.x] = clk;
        a.stamps[2 * blockIdx.x + 1] = rt;
    }
#endif
}

#ifdef MRSUM_CLOCK_STAMPS
static unsigned long long* g_stamps = nullptr;
static int g_nstamps = 0;
// copies the last launch's [grid][2] stamps to host memory; returns the count of u64 words (diagnostic build)
MRSUM_API int mrsum_gemm_stamps(unsigned long long* host, int max_words) {
    const int n = std::min(max_words, g_nstamps);
    if (!g_stamps || n <= 0 || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(host, g_stamps, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return n;
}
#endif

// x [M, K] (row stride ldx elements), w [N, K] (ldw), c [M, N] bf16 (ldc) -- or [M, N / 2] for
// epi 1 (SwiGLU of the [8 gate | 8 up]-interleaved gate_up rows).  fp8: x, w are e4m3fn bytes,
// sx [M] / sw [N] fp32 row scales; split: x is two-term [hi | lo] of 2K bytes per row over w's K.
// Requirements (checked by the Python wrapper too): K % 64 (bf16) / K % 128 (fp8), N % 16, 16-byte
// aligned rows.
MRSUM_API int mrsum_gemm(const void* x, int ldx, const void* w, int ldw, void* c, int ldc, int M, int N, int K,
                         int fp8, int epi, const float* sx, const float* sw, int group_m, int split, hipStream_t s) {
    if (M <= 0 || N <= 0) return 0;
    const int es = fp8 ? 1 : 2;
    if ((K * es) % 128 || N % 16 || (ldx * es) % 16 || (ldw * es) % 16 || ldc % 4) return (int)hipErrorInvalidValue;
    if ((size_t)256 * ldx * es >= (1u << 31) || (size_t)256 * ldw * es >= (1u << 31)) return (int)hipErrorInvalidValue;
    if (fp8 && (!sx || !sw)) return (int)hipErrorInvalidValue;
    GemmArgs a;
    a.x = (const char*)x; a.w = (const char*)w; a.c = c; a.sx = sx; a.sw = sw;
    a.ldx_b = ldx * es; a.ldw_b = ldw * es; a.ldc = ldc;
    a.M = M; a.N = N; a.kb = K * es / 128;
    if (split && (!fp8 || ldx < 2 * K)) return (int)hipErrorInvalidValue;
    a.kbw = a.kb;
    if (split) a.kb *= 2;  // X K-tiles: hi then lo
    a.tiles_m = ceil_div(M, 256); a.tiles_n = ceil_div(N, 256);
    // group_m bits 0-7: tile rows per raster group (0 = 4); bit 8: 32x32 MFMA tiles instead of 16x16.
    // Measured (profiles/r3_gemm_mfma32_experiment.jsonl, same box, interleaved): 32x32 is 0-9 % slower on
    // the 8B bf16 projections and about equal on the 70B fp8 qkv / o / down, so 16x16 stays the default;
    // the fp8 gate_up + SwiGLU GEMM gains 1.7-3.8 % at M = 4k-32k and takes it (ops/hip.py gemm_fp8).
    const bool m32 = (group_m >> 8) & 1;
    group_m &= 255;
    a.group_m = group_m > 0 ? group_m : 4;
    const dim3 grid(a.tiles_m * a.tiles_n), block(512);
#ifdef MRSUM_CLOCK_STAMPS
    static unsigned long long* stamps = nullptr;
    static size_t nstamps = 0;
    if (nstamps < 2 * grid.x) {
        if (stamps) (void)hipFree(stamps);
        nstamps = 2 * grid.x;
        if (hipMalloc(&stamps, nstamps * 8) != hipSuccess) return (int)hipErrorOutOfMemory;
    }
    a.stamps = stamps;
    g_stamps = stamps;
    g_nstamps = 2 * (int)grid.x;
#endif
    // measured (profiles/r2_gemm_variants_ab.jsonl, r2_gemm_ring10_ab.jsonl): the staggered 8-slot ring
    // (LOOK 6) with the LDS-staged epilogue is the fastest; the 2-phase / 10-slot rings and the
    // unstaggered schedule lost 5-25 %.  The register epilogue remains for outputs that are not 16-B
    // aligned (strided views).
    const bool lepi = ldc % 8 == 0 && (uintptr_t)c % 16 == 0;
#define GEMM_LAUNCH(F, E)                                                          \
    if (m32) {                                                                     \
        if (lepi) gemm_kernel<F, E, 8, true, true><<<grid, block, 0, s>>>(a);      \
        else gemm_kernel<F, E, 8, false, true><<<grid, block, 0, s>>>(a);          \
    } else {                                                                       \
        if (lepi) gemm_kernel<F, E, 8, true, false><<<grid, block, 0, s>>>(a);     \
        else gemm_kernel<F, E, 8, false, false><<<grid, block, 0, s>>>(a);         \
    }
    if (fp8) {
        if (epi == GEPI_SWIGLU) { GEMM_LAUNCH(true, GEPI_SWIGLU) } else { GEMM_LAUNCH(true, GEPI_BF16) }
    } else {
        if (epi == GEPI_SWIGLU) { GEMM_LAUNCH(false, GEPI_SWIGLU) } else { GEMM_LAUNCH(false, GEPI_BF16) }
    }
#undef GEMM_LAUNCH
    return (int)hipGetLastError();
}
