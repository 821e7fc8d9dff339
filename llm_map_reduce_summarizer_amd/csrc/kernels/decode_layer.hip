// Persistent post-attention decode layer (one GPU, decode rows M <= 16): ONE launch runs
//
//     o projection + residual  ->  gate_up + SwiGLU  ->  down projection + residual  ->  next layer's QKV
//
// with the RMSNorms deferred into the consumers (stream_gemm.hip header) -- four launches of the
// stream GEMM (and their dispatch / first-byte / drain latency, docs/decode_latency.md) become one.
//
// Geometry: 256 workgroups = one per CU (all co-resident: every workgroup only waits on work of
// stages it has already finished itself, so any co-resident set makes progress; spins are bounded and
// set an error word instead of hanging).  Each stage gives every workgroup one (column tile, k split):
//   o       [4096 x 4096]   128-row tiles x 8 splits (512 k)    residual update (split-K last arriver)
//   gate_up [28672 x 4096]  112-row tiles x 1 split             SwiGLU, deferred norm of o's residual
//   down    [4096 x 14336]  128-row tiles x 8 splits (1792 k)   residual update
//   qkv     [6144 x 4096]    96-row tiles x 4 splits (1024 k)   fp32 split-K slabs, deferred norm
//
// Workgroup = 8 STREAM waves + 1 CONTROL wave.  Stream waves only issue LDS-DMA (weights and x pieces
// into a 4-slot ring), read LDS and run MFMAs; they never issue an ordinary global load or store, so
// their in-order vmcnt only ever waits on ring pieces and the weight stream runs straight across the
// stage seams: the next stage's weight pieces are issued as ring slots free up, its x pieces (the
// previous stage's output) only once the control wave has passed the seam.  The control wave does all
// other memory traffic: it stores the tile the stream waves staged in LDS (write-through), drains,
// takes the split-K ticket, reduces the tile as the last arriver (residual + sums of squares), signals
// the seam counters, polls them (bounded), and turns the producer's sums of squares into the row
// scales of the deferred norm.  Seam counters: S_O (32 tile arrivals), S_GU + split (32 gate_up tiles
// feed each down k split), S_DN (32 tile arrivals); all re-armed by the last workgroup to exit.
#include "common.h"

namespace {
constexpr int NWG = 256;           // workgroups (= CUs)
constexpr int NSW = 8;             // stream waves
constexpr int NTHR = 64 * (NSW + 1);
constexpr int KB = 128;            // k per ring slot (256 B per weight row)
constexpr int D = 4;               // ring slots
constexpr int WIMG = 128 * 256;    // weight image: up to 128 rows x 256 B
constexpr int XIMG = 16 * 256;     // x image: 16 rows
constexpr int SLOT = WIMG + XIMG;
constexpr int STAGE_B = 16 * 128 * 4;  // epilogue tile staging: [16 rows][128 cols] fp32
constexpr int LDS_B = D * SLOT + STAGE_B + 256;
static_assert(LDS_B <= 160 * 1024, "LDS budget");

enum { ST_O = 0, ST_GU = 1, ST_DN = 2, ST_QKV = 3 };
enum { SEM_O = 0, SEM_GU = 1, SEM_DN = 9, SEM_EXIT = 10, NSEM = 16 };
constexpr unsigned long long WAIT_TICKS = 20000000ull;  // 0.2 s at 100 MHz

struct LayerArgs {
    const bf16* a;       // attention output [M, 4096] (o's x)
    int lda;
    const bf16* wo;      // [4096, 4096]
    const bf16* wgu;     // [28672, 4096] ([8 gate | 8 up] row blocks)
    const bf16* wd;      // [4096, 14336]
    const bf16* wqkv;    // [6144, 4096] or null (last layer: 3 stages)
    bf16* resid;         // residual rows [M, 4096] (in / out)
    bf16* act;           // SwiGLU features [M, 14336]
    float* parts;        // split-K scratch [8, M, 4096] (o, then down)
    float* ssp_o;        // [M, 32] row sums of squares of the residual after o, per tile
    float* ssp_d;        // [M, 32] ... after down
    float* qkv_out;      // [4, M, 6144] slabs
    int* tickets;        // [64]: o tiles 0-31, down tiles 32-63 (zero between launches)
    int* sem;            // [NSEM] seam counters (zero between launches)
    int* err;            // sticky error word
    int M;
    float eps;
};

template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void vm_wait_rt(int n) {
    switch (n) {
        case 0: vm_wait<0>(); break;   case 1: vm_wait<1>(); break;   case 2: vm_wait<2>(); break;
        case 3: vm_wait<3>(); break;   case 4: vm_wait<4>(); break;   case 5: vm_wait<5>(); break;
        case 6: vm_wait<6>(); break;   case 7: vm_wait<7>(); break;   case 8: vm_wait<8>(); break;
        case 9: vm_wait<9>(); break;   case 10: vm_wait<10>(); break; case 11: vm_wait<11>(); break;
        case 12: vm_wait<12>(); break; case 13: vm_wait<13>(); break; case 14: vm_wait<14>(); break;
        default: vm_wait<15>(); break;
    }
}

__device__ __forceinline__ void bar() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* dst, int voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, voff, 0, 0, 0);
}

// the stream_gemm.hip image: a 1 KiB piece = 8 rows x 128 B (one k half); 16-B chunk slot = chunk ^ (row & 7)
__device__ __forceinline__ int img_off(int row, int chunk) {
    return (((row >> 3) << 1) + (chunk >> 3)) * 1024 + ((row & 7) << 7) + ((((chunk & 7) ^ (row & 7))) << 4);
}

struct Stage {
    const bf16* w;  // this workgroup's weight rows (row n0 of the stage matrix)
    const bf16* x;  // x rows, k offset of this split applied
    int ldw, ldx;   // row strides (elements)
    int rows;       // tile rows (16 per active stream wave)
    int nkb;        // k blocks of this split
    int rows_valid; // rows of the matrix left from n0 (masking)
};

__device__ __forceinline__ void stage_geom(const LayerArgs& a, int s, int bid, Stage& g, int& tile, int& sp) {
    switch (s) {
        case ST_O:
            tile = bid >> 3; sp = bid & 7;
            g.w = a.wo + (size_t)(tile * 128) * 4096 + sp * 512; g.ldw = 4096;
            g.x = a.a + sp * 512; g.ldx = a.lda; g.rows = 128; g.nkb = 4; break;
        case ST_GU:
            tile = bid; sp = 0;
            g.w = a.wgu + (size_t)(tile * 112) * 4096; g.ldw = 4096;
            g.x = a.resid; g.ldx = 4096; g.rows = 112; g.nkb = 32; break;
        case ST_DN:
            tile = bid >> 3; sp = bid & 7;
            g.w = a.wd + (size_t)(tile * 128) * 14336 + sp * 1792; g.ldw = 14336;
            g.x = a.act + sp * 1792; g.ldx = 14336; g.rows = 128; g.nkb = 14; break;
        default:
            tile = bid >> 2; sp = bid & 3;
            g.w = a.wqkv + (size_t)(tile * 96) * 4096 + sp * 1024; g.ldw = 4096;
            g.x = a.resid + sp * 1024; g.ldx = 4096; g.rows = 96; g.nkb = 8; break;
    }
    g.rows_valid = g.rows;
}

// control wave: bounded poll of a seam counter, then an agent-scope acquire (invalidates this CU's L1
// and the XCD's L2 lines, so the stream waves' later x pieces read the producers' write-through data)
__device__ __forceinline__ void seam_wait(int* c, int target, int* err, int lane) {
    if (lane == 0) {
        if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target &&
            !__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > WAIT_TICKS) {
                    atomicOr(err, 1);
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void st_wt(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt_u32(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// control wave: row scales of the deferred norm from the producer's [M][32] per-tile sums of squares
__device__ __forceinline__ void row_scales(const float* ssp, int M, float eps, int lane, float* s_scale) {
    if (lane < M) {
        const float4* p = reinterpret_cast<const float4*>(ssp + lane * 32);
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = p[i];
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) t += (v[i].x + v[i].y) + (v[i].z + v[i].w);
        s_scale[lane] = rsqrtf(t * (1.f / 4096.f) + eps);
    }
}

// control wave, residual-update stage: publish this split's fp32 partial tile [M][128] (staged in LDS),
// take the tile's ticket, and as the last of the 8 splits: residual += sum of partials (split order,
// residual first: the add_rmsnorm_parts arithmetic), per-row sums of squares of the rounded residual
// -> ssp[m][tile], re-arm the ticket, signal the seam.
__device__ void resid_epilogue(const LayerArgs& a, int tile, int sp, const float* stg, int lane, int* ticket,
                               float* ssp, int* sem) {
    const int M = a.M;
    float* pp = a.parts + (size_t)sp * M * 4096 + tile * 128;
    for (int i = lane; i < M * 32; i += 64) {  // item: (row, 4 columns)
        const int m = i >> 5, c = (i & 31) * 4;
        const float4 v = *reinterpret_cast<const float4*>(stg + m * 128 + c);
        float* d = pp + (size_t)m * 4096 + c;
        st_wt(d, v.x); st_wt(d + 1, v.y); st_wt(d + 2, v.z); st_wt(d + 3, v.w);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) last = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 7;
    last = __shfl(last, 0, 64);
    if (!last) return;
    if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    // lane owns columns 2 lane, 2 lane + 1 of the tile for every row
    const int c = tile * 128 + 2 * lane;
    for (int m = 0; m < M; ++m) {
        float s0[8], s1[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float2 v = *reinterpret_cast<const float2*>(a.parts + ((size_t)q * M + m) * 4096 + c);
            s0[q] = v.x; s1[q] = v.y;
        }
        unsigned* rp = reinterpret_cast<unsigned*>(a.resid + (size_t)m * 4096 + c);
        const unsigned rv = *rp;
        float h0 = __uint_as_float(rv << 16), h1 = __uint_as_float(rv & 0xffff0000u);
#pragma unroll
        for (int q = 0; q < 8; ++q) { h0 += s0[q]; h1 += s1[q]; }
        const unsigned hv = pack2(h0, h1);
        st_wt_u32(rp, hv);
        h0 = __uint_as_float(hv << 16); h1 = __uint_as_float(hv & 0xffff0000u);
        const float ss = wave_sum(h0 * h0 + h1 * h1);
        if (lane == 0) st_wt(ssp + m * 32 + tile, ss);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(sem, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

__global__ __launch_bounds__(NTHR, 1) void decode_layer_kernel(const LayerArgs a) {
    // ONE LDS object (a second one made hipcc wait vmcnt(0) before every ring read): the DMA ring, the
    // epilogue staging [16][128] fp32 and 16 row scales.  hipcc drains vmcnt before the staging writes
    // (it cannot tell them from the ring), so the next stage's weight pieces are issued right AFTER the
    // staging writes, never before them.
    __shared__ __attribute__((aligned(1024))) char lds[LDS_B];
    float* stg = reinterpret_cast<float*>(lds + D * SLOT);
    float* s_scale = reinterpret_cast<float*>(lds + D * SLOT + STAGE_B);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // 0..7 stream, 8 control
    const int bid = blockIdx.x, M = a.M;
    const int nst = a.wqkv ? 4 : 3;

    // stage k-block bases in the global slot sequence
    // global ring-slot sequence: o slots [0, 4), gate_up [4, 36), down [36, 50), qkv [50, 58)
    const int J = nst == 4 ? 58 : 50;

    if (wv < NSW) {
        // ---------------------------------------------------------------- stream waves
        const int prow = lane >> 3, pslot = lane & 7;
        int issued = 0, need0 = 0, need1 = 0, need2 = 0, need3 = 0;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        // stage geometry is recomputed where needed (uniform scalar math): an array of per-stage
        // structs indexed by the runtime stage went to scratch
        // issue the weight pieces of slot j (this wave's 16 rows, if the stage uses this wave)
#define STAGE_OF(J_) ((J_) < 4 ? 0 : (J_) < 36 ? 1 : (J_) < 50 ? 2 : 3)
#define BASE_OF(S_) ((S_) == 0 ? 0 : (S_) == 1 ? 4 : (S_) == 2 ? 36 : (S_) == 3 ? 50 : 58)
#define ISSUE_W(J_)                                                                                       \
        {                                                                                                 \
            const int s_ = STAGE_OF(J_), kb_ = (J_) - BASE_OF(s_);                                           \
            Stage G_;                                                                                     \
            int t_, p_;                                                                                   \
            stage_geom(a, s_, bid, G_, t_, p_);                                                           \
            if (wv * 16 < G_.rows) {                                                                      \
                const __amdgpu_buffer_rsrc_t r_ = __builtin_amdgcn_make_buffer_rsrc(                      \
                    (void*)(G_.w + (size_t)(16 * wv) * G_.ldw + kb_ * KB), (short)0, 0x7fffffff, 0x00020000); \
                char* dst_ = lds + ((J_) % D) * SLOT + wv * 4096;                                         \
                _Pragma("unroll") for (int p = 0; p < 4; ++p) {                                           \
                    const int row_ = 8 * (p >> 1) + prow;                                                 \
                    dma16(r_, dst_ + p * 1024, row_ * G_.ldw * 2 + 16 * (8 * (p & 1) + (pslot ^ prow)));  \
                }                                                                                         \
                issued += 4;                                                                              \
            }                                                                                             \
        }
        // the x piece of slot j: waves 0-3, piece = wave (rows 8 (wv >> 1) + prow, k half wv & 1); rows
        // past M re-read row M - 1 (their products are never stored)
#define ISSUE_X(J_)                                                                                       \
        {                                                                                                 \
            if (wv < 4) {                                                                                 \
                const int s_ = STAGE_OF(J_), kb_ = (J_) - BASE_OF(s_);                                       \
                Stage G_;                                                                                 \
                int t_, p_;                                                                               \
                stage_geom(a, s_, bid, G_, t_, p_);                                                       \
                const int row_ = min(8 * (wv >> 1) + prow, M - 1);                                       \
                const __amdgpu_buffer_rsrc_t r_ = __builtin_amdgcn_make_buffer_rsrc(                      \
                    (void*)(G_.x + kb_ * KB), (short)0, 0x7fffffff, 0x00020000);                          \
                dma16(r_, lds + ((J_) % D) * SLOT + WIMG + wv * 1024,                                     \
                      row_ * G_.ldx * 2 + 16 * (8 * (wv & 1) + (pslot ^ prow)));                         \
                issued += 1;                                                                              \
            }                                                                                             \
        }
#define SET_NEED(J_) { const int i_ = (J_) & 3; if (i_ == 0) need0 = issued; else if (i_ == 1) need1 = issued; \
                       else if (i_ == 2) need2 = issued; else need3 = issued; }
#define GET_NEED(J_) (((J_) & 3) == 0 ? need0 : ((J_) & 3) == 1 ? need1 : ((J_) & 3) == 2 ? need2 : need3)
        // prologue: slots 0 .. D-2 (stage 0 has 4 >= D-1 slots: W and x; o's x is the attention output)
#pragma unroll
        for (int j = 0; j < D - 1; ++j) {
            ISSUE_W(j)
            ISSUE_X(j)
            SET_NEED(j)
        }
        const int r = lane & 15, q4 = lane >> 4;
        for (int j = 0; j < J; ++j) {
            const int s = STAGE_OF(j);
            if (s > 0 && j == BASE_OF(s)) {
                bar();  // B2: the control wave passed the seam into stage s (row scales in LDS)
                // x pieces of the stage-s slots whose weights are already in flight
                for (int jj = j; jj < min(j + D - 1, BASE_OF(s + 1)); ++jj) {
                    ISSUE_X(jj)
                    SET_NEED(jj)
                }
            }
            vm_wait_rt(issued - GET_NEED(j));
            bar();  // B1: slot j landed for every wave; every wave finished slot j-1 (its buffer is free)
            const int jn = j + D - 1;
            if (jn < J && STAGE_OF(jn) == s) {  // next-stage slots: issued after this stage's epilogue
                ISSUE_W(jn)
                ISSUE_X(jn)
                SET_NEED(jn)
            }
            Stage G;
            int tile_, sp_;
            stage_geom(a, s, bid, G, tile_, sp_);
            if (wv * 16 < G.rows) {
                const char* wl = lds + (j % D) * SLOT;
                const char* xl = wl + WIMG;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const u32x4 av = *reinterpret_cast<const u32x4*>(wl + img_off(16 * wv + r, 4 * i + q4));
                    const u32x4 bv = *reinterpret_cast<const u32x4*>(xl + img_off(r, 4 * i + q4));
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                                  __builtin_bit_cast(bf16x8, bv), acc, 0, 0, 0);
                }
            }
            if (j == BASE_OF(s + 1) - 1) {
                // epilogue: lane holds out^T[n = 16 wv + 4 q4 + jj][m = r] of the tile -> LDS staging
                if (wv * 16 < G.rows && r < M) {
                    if (s == ST_GU || s == ST_QKV) {
                        const float sc = s_scale[r];
                        acc[0] *= sc; acc[1] *= sc; acc[2] *= sc; acc[3] *= sc;
                    }
                    if (s == ST_GU) {
                        // [8 gate | 8 up] rows: lanes q4 < 2 hold gate features 8 wv + 4 q4 + jj, q4 + 2 the ups
                        f32x4 up;
#pragma unroll
                        for (int jj = 0; jj < 4; ++jj) up[jj] = __shfl_xor(acc[jj], 32, 64);
                        if (q4 < 2) {
                            float* o = stg + r * 128 + 8 * wv + 4 * q4;
#pragma unroll
                            for (int jj = 0; jj < 4; ++jj) o[jj] = acc[jj] / (1.f + __expf(-acc[jj])) * up[jj];
                        }
                    } else {
                        *reinterpret_cast<float4*>(stg + r * 128 + 16 * wv + 4 * q4) =
                            make_float4(acc[0], acc[1], acc[2], acc[3]);
                    }
                }
                acc = f32x4{0.f, 0.f, 0.f, 0.f};
                // the next stage's first D-1 slots: weight pieces now (their buffers were freed by slots
                // j-2 .. j), x pieces once the control wave has passed the seam
                for (int jj = BASE_OF(s + 1); jj < min(j + D, J); ++jj) {
                    ISSUE_W(jj)
                    SET_NEED(jj)
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                bar();  // B3: tile staged -> control wave
                bar();  // B4: control wave took the staged tile (staging reusable)
            }
        }
#undef ISSUE_W
#undef ISSUE_X
#undef SET_NEED
#undef GET_NEED
    } else {
        // ---------------------------------------------------------------- control wave
        int* sem = a.sem;
        for (int j = 0; j < J; ++j) {
            const int s = STAGE_OF(j);
            if (s > 0 && j == BASE_OF(s)) {
                // seam into stage s, then the deferred-norm row scales of gate_up / qkv
                int tile, sp;
                Stage gg;
                stage_geom(a, s, bid, gg, tile, sp);
                if (s == ST_GU) seam_wait(sem + SEM_O, 32, a.err, lane);
                else if (s == ST_DN) seam_wait(sem + SEM_GU + sp, 32, a.err, lane);
                else seam_wait(sem + SEM_DN, 32, a.err, lane);
                if (s == ST_GU) row_scales(a.ssp_o, M, a.eps, lane, s_scale);
                if (s == ST_QKV) row_scales(a.ssp_d, M, a.eps, lane, s_scale);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                bar();  // B2
            }
            bar();  // B1
            if (j == BASE_OF(s + 1) - 1) {
                bar();  // B3: the stream waves staged the tile
                int tile, sp;
                Stage gg;
                stage_geom(a, s, bid, gg, tile, sp);
                if (s == ST_O || s == ST_DN) {
                    // copy the partial tile out of the staging buffer first (B4 releases it)
                    resid_epilogue(a, tile, sp, stg, lane, a.tickets + (s == ST_O ? 0 : 32) + tile,
                                   s == ST_O ? a.ssp_o : a.ssp_d, sem + (s == ST_O ? SEM_O : SEM_DN));
                } else if (s == ST_GU) {
                    // SwiGLU features [M][56] -> act columns 56 tile .. (write-through), then signal the
                    // down k split that consumes them (features 1792 sp' .. : tiles 32 sp' .. 32 sp' + 31)
                    for (int i = lane; i < M * 28; i += 64) {
                        const int m = i / 28, c = (i % 28) * 2;
                        st_wt_u32(reinterpret_cast<unsigned*>(a.act + (size_t)m * 14336 + tile * 56 + c),
                                  pack2(stg[m * 128 + c], stg[m * 128 + c + 1]));
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0)
                        __hip_atomic_fetch_add(sem + SEM_GU + (tile >> 5), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    // QKV slabs [4][M][6144] (read by the next launch: plain stores)
                    for (int i = lane; i < M * 24; i += 64) {
                        const int m = i / 24, c = (i % 24) * 4;
                        *reinterpret_cast<float4*>(a.qkv_out + ((size_t)sp * M + m) * 6144 + tile * 96 + c) =
                            *reinterpret_cast<const float4*>(stg + m * 128 + c);
                    }
                }
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                bar();  // B4
            }
        }
        // exit: the last workgroup out re-arms the seam counters for the next launch
        if (lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (__hip_atomic_fetch_add(sem + SEM_EXIT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NWG - 1) {
                for (int i = 0; i < NSEM; ++i) __hip_atomic_store(sem + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
#undef STAGE_OF
#undef BASE_OF
}

// One post-attention decode layer of a Llama-3-8B-shaped model on one GPU (hidden 4096, ffn 14336,
// 32 q / 8 kv heads x 128), M <= 16 rows.  wqkv null: the last layer (o, gate_up, down only).
// Scratch: act [M, 14336] bf16, parts [8, M, 4096] fp32, ssp_o / ssp_d [M, 32] fp32, tickets [64] and
// sem [16] ints zero on the first call (every launch leaves them zero), err a sticky int.
MRSUM_API int mrsum_decode_layer(const void* attn, int lda, const void* wo, const void* wgu, const void* wd,
                                 const void* wqkv, void* resid, void* act, void* parts, void* ssp_o, void* ssp_d,
                                 void* qkv_out, int* tickets, int* sem, int* err, int M, float eps, hipStream_t s) {
    if (M < 1 || M > 16 || lda % 8) return (int)hipErrorInvalidValue;
    if (!attn || !wo || !wgu || !wd || !resid || !act || !parts || !ssp_o || !ssp_d || !tickets || !sem || !err)
        return (int)hipErrorInvalidValue;
    if (wqkv && !qkv_out) return (int)hipErrorInvalidValue;
    LayerArgs a;
    a.a = (const bf16*)attn; a.lda = lda;
    a.wo = (const bf16*)wo; a.wgu = (const bf16*)wgu; a.wd = (const bf16*)wd; a.wqkv = (const bf16*)wqkv;
    a.resid = (bf16*)resid; a.act = (bf16*)act; a.parts = (float*)parts;
    a.ssp_o = (float*)ssp_o; a.ssp_d = (float*)ssp_d; a.qkv_out = (float*)qkv_out;
    a.tickets = tickets; a.sem = sem; a.err = err; a.M = M; a.eps = eps;
    decode_layer_kernel<<<NWG, NTHR, 0, s>>>(a);
    return (int)hipGetLastError();
}
