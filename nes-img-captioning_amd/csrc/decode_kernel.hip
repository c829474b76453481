// decode_kernel.hip -- population greedy decode of the fc_caption LSTM on gfx950.
//
// Replaces, for a whole population at once, the per-worker CPU path
//   NESWorker.fitness -> PolicyNet.evolve -> CaptPolicy.rollout -> FCModel._sample
//   (/root/reference/src/algorithm/nic_nes/nic_nes_worker.py:142-154,
//    /root/reference/src/algorithm/nets.py:101-113,
//    /root/reference/src/captioning/nets.py:98-134,183-245)
//
// One workgroup = one population member (both antithetic signs) x one slab of <=128 unique
// images. 8 waves: wave w decodes sign (w>>2) for batch rows 32*(w&3) .. +31 of the slab.
// Every dense product is computed TRANSPOSED (weights = MFMA A operand from LDS, activations =
// B operand held in registers) with v_mfma_f32_32x32x2_f32, so the 32x32 accumulator of one
// product is already the B operand of the next (k order: include/nicnes_math.h nn_kperm).
// Perturbed weights are never materialised in HBM: each 32x128 weight tile is formed in LDS
// as fp32(W0 +/- fp32(sigma * z[idx + offset])) from the base theta and the member's noise
// slice, once for both signs.
//
// Addressing: every global access goes through a buffer resource (wave-uniform 128-bit
// descriptor + 32-bit lane offset) so no 64-bit VGPR address pairs are kept live.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nicnes_math.h"
#include "decode_kernel.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

#define NTHREADS 512
#define LDS_ROW 132                                   // 128 k + 4 pad: conflict-free b128 reads
#define SIGN_FLOATS (32 * LDS_ROW)
#define STAGE_FLOATS (2 * SIGN_FLOATS + 64)           // W+ | W- | bias+ (32) | bias- (32)
#define LOG2E 1.44269504088896340736f
#define NEG_INF (-__builtin_inff())
#ifndef DECODE_ABLATE
#define DECODE_ABLATE 0    // timing-only builds (scripts/ablate.py): 1 no logit epilogue, 2 no logit
#endif                     // staging, 4 no LSTM cell, 8 no logit-loop barrier -- wrong results
#ifndef DECODE_SCHED
#define DECODE_SCHED 0
#endif
#ifndef DECODE_PROF
#define DECODE_PROF 0      // timing-only build: per-wave section cycles written over seq (wrong tokens)
#endif
#if DECODE_PROF
#define PROF_STAMP(sec)                                                                          \
    do {                                                                                         \
        unsigned long long t_;                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                 \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        const uint32_t d_ = (uint32_t)(t_ - prof_t0);                                            \
        _Pragma("unroll") for (int k_ = 0; k_ < 16; ++k_) prof_acc[k_] += prof_cur == k_ ? d_ : 0u;  \
        prof_t0 = t_;                                                                            \
        prof_cur = (sec);                                                                        \
    } while (0)
#else
#define PROF_STAMP(sec) do { } while (0)
#endif
#ifndef DECODE_IEPI
#define DECODE_IEPI 0      // 1: logit epilogue folded into the MFMA stream of each wave (no sign stagger)
#endif
#ifndef DECODE_CELL
#define DECODE_CELL 1      // 1: two-pass cell, 32-row tiles; 2: fused single pass; 3: two-pass, 64-row stages, folded gates
#endif

// lane id recomputed at the point of use (volatile: never hoisted or kept live across the logit
// loop), so lane-derived LDS / buffer offsets are cheap VALU instead of registers the compiler
// would spill and reload behind the in-flight staging loads (vmcnt is in-order)
__device__ __forceinline__ int lane_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// ---- buffer helpers ------------------------------------------------------------------------
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 ld4(rsrc_t r, uint32_t byte_off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 0));
}
__device__ __forceinline__ float ld1(rsrc_t r, uint32_t byte_off, uint32_t soff = 0) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, (int)soff, 0));
}
__device__ __forceinline__ void st1(rsrc_t r, uint32_t byte_off, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)byte_off, (int)soff, 0);
}

struct TileDesc {
    uint32_t w_off;    // theta offset (floats) of the weight matrix
    int32_t ld;        // row length of the matrix in theta (floats)
    int32_t row0;      // first matrix row of the tile
    int32_t nvalid;    // rows >= nvalid are padding (zero weights, pad bias)
    int32_t k0;        // first column of the 128-wide k window
    uint32_t b_off;    // theta offset of the bias vector
    float pad_bias;
};

struct StageRegs {
    f32x4 w[2], z[2];
    float bw, bz;
};

// ---- LDS staging of one perturbed 32 x 128 tile (both signs) ------------------------------
// theta_r covers theta[0, D); noise_r covers the member's slice noise[idx, idx + D)
__device__ __forceinline__ void stage_load(rsrc_t theta_r, rsrc_t noise_r, const TileDesc& d, int tid, StageRegs& s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = tid + NTHREADS * u, row = f >> 5, q = f & 31;
        const int rc = row < d.nvalid ? row : max(d.nvalid - 1, 0);  // clamp, zero after the load
        const uint32_t off = 4u * (d.w_off + (uint32_t)((d.row0 + rc) * d.ld + d.k0 + 4 * q));
        const f32x4 w = ld4(theta_r, off), z = ld4(noise_r, off);
        const bool ok = row < d.nvalid;
        s.w[u] = ok ? w : f32x4{0.f, 0.f, 0.f, 0.f};
        s.z[u] = ok ? z : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    {   // every thread loads bias row (tid & 31): no divergent branch in the staging code
        const int r = tid & 31;
        const int rc = r < d.nvalid ? r : 0;
        const uint32_t off = 4u * (d.b_off + (uint32_t)(d.row0 + rc));
        s.bw = ld1(theta_r, off);
        s.bz = ld1(noise_r, off);
    }
}

__device__ __forceinline__ void stage_store(float* buf, const TileDesc& d, float sigma, int tid, const StageRegs& s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = tid + NTHREADS * u, row = f >> 5, q = f & 31;
        const int T = q >> 3, hh = q & 1, a = (q & 7) >> 1;
        const int o = row * LDS_ROW + T * 32 + hh * 16 + 4 * a;
        const f32x4 delta = sigma * s.z[u];           // fp32(sigma * z), nets.py:102
        const f32x4 plus = s.w[u] + delta;            // nets.py:113
        const f32x4 minus = s.w[u] - delta;           // nic_nes_worker.py:151
        *reinterpret_cast<f32x4*>(buf + o) = plus;
        *reinterpret_cast<f32x4*>(buf + SIGN_FLOATS + o) = minus;
    }
    {   // slot (tid & 63): bias+ rows 0..31, bias- rows 32..63; every wave writes the same
        // values to the same 64 slots (benign, branch-free)
        const int r = tid & 31;
        const float delta = sigma * s.bz;
        const float v = (tid & 32) ? s.bw - delta : s.bw + delta;
        buf[2 * SIGN_FLOATS + (tid & 63)] = r < d.nvalid ? v : d.pad_bias;
    }
}

// ---- one 32x32 output tile: acc += W_tile(32 x 128, LDS) . B(128 x 32, registers) -----------
__device__ __forceinline__ f32x16 bias_init(const float* bias, int hh) {
    f32x16 acc;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + 8 * a + 4 * hh);
        acc[4 * a + 0] = bb[0];
        acc[4 * a + 1] = bb[1];
        acc[4 * a + 2] = bb[2];
        acc[4 * a + 3] = bb[3];
    }
    return acc;
}

__device__ __forceinline__ f32x16 mfma_tile(f32x16 acc, const float* w, const float (&Bop)[64], int lane) {
    const float* row = w + (lane & 31) * LDS_ROW + (lane >> 5) * 16;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = *reinterpret_cast<const f32x4*>(row + T * 32 + 4 * c);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[jj >> 2][jj & 3], Bop[16 * T + jj], acc, 0, 0, 0);
    }
    return acc;
}

// same product with the A fragments of sub-chunk T+1 read while sub-chunk T's MFMAs run
__device__ __forceinline__ f32x16 mfma_tile_pf(f32x16 acc, const float* w, const float (&Bop)[64], int lane) {
    const float* row = w + (lane & 31) * LDS_ROW + (lane >> 5) * 16;
    f32x4 a[4], an[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = *reinterpret_cast<const f32x4*>(row + 4 * c);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        if (T < 3) {
#pragma unroll
            for (int c = 0; c < 4; ++c) an[c] = *reinterpret_cast<const f32x4*>(row + (T + 1) * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[jj >> 2][jj & 3], Bop[16 * T + jj], acc, 0, 0, 0);
        if (T < 3) {
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] = an[c];
        }
    }
#if DECODE_SCHED >= 3
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 1);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        if (T < 3) __builtin_amdgcn_sched_group_barrier(0x100, 4, 1);
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 1);
    }
#endif
    return acc;
}

// img_embed variant: the B operand (fc row chunk) is read per 32-k sub-chunk from global
__device__ __forceinline__ f32x16 mfma_tile_fc(f32x16 acc, const float* w, rsrc_t fc_r, uint32_t frow_off, int lane) {
    const float* row = w + (lane & 31) * LDS_ROW + (lane >> 5) * 16;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a[4], bq[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a[c] = *reinterpret_cast<const f32x4*>(row + T * 32 + 4 * c);
            bq[c] = ld4(fc_r, frow_off + 4u * (32 * T + 8 * c));
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[jj >> 2][jj & 3], bq[jj >> 2][jj & 3], acc, 0, 0, 0);
    }
    return acc;
}

// ---- per-row greedy state over the vocabulary (log_softmax + first argmax, nets.py:202,208) --
struct RowState {
    float m;              // running max logit (== newest record)
    float s;              // sum exp(L - m) over this lane's vocab subset
    float r1v; int r1i;   // newest left-to-right record (the running max, first index)
    float r0v; int r0i;   // previous record
    float ev;             // largest evicted record
};

__device__ __forceinline__ void row_state_init(RowState& st) {
    st.m = -1.0e30f; st.s = 0.f;   // finite, and m * log2e stays finite: exp2 args never NaN
    st.r1v = NEG_INF; st.r1i = 0x7fffffff;
    st.r0v = NEG_INF; st.r0i = 0x7fffffff;
    st.ev = NEG_INF;
}

// Lane holds logits for vocab vbase + (r&3) + 8(r>>2), increasing in r.
// The greedy token is the earliest record (left-to-right maximum) inside the log_softmax tie
// window of the final max; each lane half keeps its last two records, and remembers the
// largest record it evicted so an overflowing row can be detected.
__device__ __forceinline__ void logit_epilogue(RowState& st, const f32x16& acc, int vbase) {
    float tmax = acc[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) tmax = fmaxf(tmax, acc[r]);
    const float mnew = fmaxf(st.m, tmax);
    st.s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
    st.m = mnew;
    float ts = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) ts += __builtin_amdgcn_exp2f((acc[r] - st.m) * LOG2E);
    st.s += ts;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float L = acc[r];
        const int v = vbase + (r & 3) + 8 * (r >> 2);
        const bool c = L > st.r1v;
        st.ev = c ? st.r0v : st.ev;
        st.r0v = c ? st.r1v : st.r0v;
        st.r0i = c ? st.r1i : st.r0i;
        st.r1v = c ? L : st.r1v;
        st.r1i = c ? v : st.r1i;
    }
}

// One logit tile with a hand-placed schedule: the 64 dependent MFMAs of tile n, and between
// consecutive MFMAs a slice of (a) the epilogue of tile n-1 and (b) the LDS store of the staged
// tile n+1. In-order issue puts every slice in the shadow of the MFMA ahead of it (the next
// dependent MFMA waits for that one anyway); sched_barrier(0) pins the order.
// Epilogue slots: 0-6 tile max + rescale, 8-23 sum of exp2, 24-39 record updates;
// staging slots 44-51 (row u=0), 52-59 (u=1), 60 bias.
__device__ __forceinline__ void epi_slot(int j, RowState& st, const f32x16& P, int vbase, float (&x)[5],
                                         float& ml) {
    if (j < 5) {
        x[j] = fmaxf(fmaxf(P[3 * j], P[3 * j + 1]), P[3 * j + 2]);
    } else if (j == 5) {
        x[0] = fmaxf(fmaxf(x[0], x[1]), x[2]);
    } else if (j == 6) {
        const float tmax = fmaxf(fmaxf(x[0], x[3]), fmaxf(x[4], P[15]));
        const float mnew = fmaxf(st.m, tmax);
        st.s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
        st.m = mnew;
        ml = mnew * LOG2E;
    } else if (j >= 8 && j < 24) {
        const int r = j - 8;
        st.s += __builtin_amdgcn_exp2f(__builtin_fmaf(P[r], LOG2E, -ml));
    } else if (j >= 24 && j < 40) {
        const int r = j - 24;
        const float L = P[r];
        const int v = vbase + (r & 3) + 8 * (r >> 2);
        const bool c = L > st.r1v;
        st.ev = c ? st.r0v : st.ev;
        st.r0v = c ? st.r1v : st.r0v;
        st.r0i = c ? st.r1i : st.r0i;
        st.r1v = c ? L : st.r1v;
        st.r1i = c ? v : st.r1i;
    }
}

__device__ __forceinline__ void store_slot(int j, float* buf, const TileDesc& d, float sigma, int tid,
                                           const StageRegs& s) {
    if (j >= 44 && j < 60) {
        const int u = (j - 44) >> 3, part = (j - 44) & 7;
        const int f = tid + NTHREADS * u, row = f >> 5, q = f & 31;
        const int o = row * LDS_ROW + (q >> 3) * 32 + (q & 1) * 16 + 4 * ((q & 7) >> 1);
        if (part == 0) {
            const f32x4 delta = sigma * s.z[u];
            *reinterpret_cast<f32x4*>(buf + o) = s.w[u] + delta;
            *reinterpret_cast<f32x4*>(buf + SIGN_FLOATS + o) = s.w[u] - delta;
        }
    } else if (j == 60) {
        const int r = tid & 31;
        const float delta = sigma * s.bz;
        const float v = (tid & 32) ? s.bw - delta : s.bw + delta;
        buf[2 * SIGN_FLOATS + (tid & 63)] = r < d.nvalid ? v : d.pad_bias;
    }
}

__device__ __forceinline__ f32x16 logit_tile_sched(const float* w, const float* bias, const float (&Bop)[64], int lane,
                                                   RowState& st, const f32x16& prev, int vbase_prev, float* nbuf,
                                                   const TileDesc& nd, float sigma, int tid, const StageRegs& s) {
    const int hh = lane >> 5;
    const float* row = w + (lane & 31) * LDS_ROW + hh * 16;
    f32x16 acc = bias_init(bias, hh);
    f32x4 a[4], an[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = *reinterpret_cast<const f32x4*>(row + 4 * c);
    float x[5], ml = 0.f;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        if (T < 3) {
#pragma unroll
            for (int c = 0; c < 4; ++c) an[c] = *reinterpret_cast<const f32x4*>(row + (T + 1) * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int j = 16 * T + jj;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[jj >> 2][jj & 3], Bop[j], acc, 0, 0, 0);
            epi_slot(j, st, prev, vbase_prev, x, ml);
            store_slot(j, nbuf, nd, sigma, tid, s);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (T < 3) {
#pragma unroll
            for (int c = 0; c < 4; ++c) a[c] = an[c];
        }
    }
    return acc;
}

// ---- 64-row logit stages ---------------------------------------------------------------------
#define STAGE64_FLOATS (2 * 64 * LDS_ROW + 128)       // W+ (64 rows) | W- | bias+ (64) | bias- (64)

struct Stage64Regs {
    f32x4 w[4], z[4];
    float bw, bz;
};

__device__ __forceinline__ f32x4 ld4s(rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
#ifndef LOGIT_Z_AUX
#define LOGIT_Z_AUX 0      // cache policy of the member's noise-slice loads in the logit stages
#endif
#ifndef LOGIT_W_AUX
#define LOGIT_W_AUX 0
#endif
template <int AUX>
__device__ __forceinline__ f32x4 ld4p(rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, AUX));
}

// thread tid loads floats 4*tid + 2048*u .. +3 of the stage (row (tid>>5) + 16u, k 4*(tid&31)):
// one lane offset (16*tid) for every load, the stage / chunk offsets ride in the scalar offset
__device__ __forceinline__ void stage64_load(rsrc_t lw, rsrc_t lz, rsrc_t lbw, rsrc_t lbz, int s, int tid,
                                             Stage64Regs& r) {
    const uint32_t vo = 16u * (uint32_t)tid;
    const uint32_t so = 32768u * (uint32_t)s;
    const uint32_t vb = (vo >> 2) & 252u;               // 4 * (tid & 63), recomputed, never spilled
    r.bw = ld1(lbw, vb, 256u * (uint32_t)s);
    r.bz = ld1(lbz, vb, 256u * (uint32_t)s);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        r.w[u] = ld4p<LOGIT_W_AUX>(lw, vo, so + 8192u * u);
        r.z[u] = ld4p<LOGIT_Z_AUX>(lz, vo, so + 8192u * u);
    }
}

__device__ __forceinline__ void stage64_store(float* buf, int s, int V1, float sigma, int tid, const Stage64Regs& r) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int f = tid + NTHREADS * u, row = f >> 5, q = f & 31;
        const int o = row * LDS_ROW + (q >> 3) * 32 + (q & 1) * 16 + 4 * ((q & 7) >> 1);
        const f32x4 delta = sigma * r.z[u];           // fp32(sigma * z), nets.py:102
        *reinterpret_cast<f32x4*>(buf + o) = r.w[u] + delta;                    // nets.py:113
        *reinterpret_cast<f32x4*>(buf + 64 * LDS_ROW + o) = r.w[u] - delta;     // nic_nes_worker.py:151
    }
    const int row = tid & 63, sg = (tid >> 6) & 1;     // every pair of waves writes all 128 slots
    const float delta = sigma * r.bz;
    const float v = sg ? r.bw - delta : r.bw + delta;
    buf[2 * 64 * LDS_ROW + 64 * sg + row] = (64 * s + row < V1) ? v : NEG_INF;
}

// two independent accumulator chains (rows 0-31 and 32-63 of the stage) over the same B
__device__ __forceinline__ void mfma_stage64(const float* w, const float* bias, const float (&Bop)[64], int lane,
                                             f32x16& acc0, f32x16& acc1) {
    const int hh = lane >> 5;
    const float* row0 = w + (lane & 31) * LDS_ROW + hh * 16;
    const float* row1 = row0 + 32 * LDS_ROW;
    acc0 = bias_init(bias, hh);
    acc1 = bias_init(bias + 32, hh);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a0[c] = *reinterpret_cast<const f32x4*>(row0 + T * 32 + 4 * c);
            a1[c] = *reinterpret_cast<const f32x4*>(row1 + T * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], acc1, 0, 0, 0);
        }
    }
}

// the same two chains continuing from given accumulators (no bias initialisation)
__device__ __forceinline__ void mfma_stage64_acc(const float* w, const float (&Bop)[64], int lane, f32x16& acc0,
                                                 f32x16& acc1) {
    const int hh = lane >> 5;
    const float* row0 = w + (lane & 31) * LDS_ROW + hh * 16;
    const float* row1 = row0 + 32 * LDS_ROW;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a0[c] = *reinterpret_cast<const f32x4*>(row0 + T * 32 + 4 * c);
            a1[c] = *reinterpret_cast<const f32x4*>(row1 + T * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], acc1, 0, 0, 0);
        }
    }
}

// ---- logit stages staged by LDS-DMA (DECODE_GLDS) ----------------------------------------------
// One stage buffer: region 0 = 64 rows x 128 (raw w, then W+), region 1 (raw z, then W-), then
// bias+ (64) | bias- (64). Rows are unpadded; 16-byte chunk `pre` of row r sits at chunk
// pre ^ (r & 15) (conflict-free A reads). The DMA writes lane-linearly, so the permutation is on
// the per-lane SOURCE offset. Each lane later reads back exactly the chunks its own DMA wrote and
// forms W+/W- in place: no registers carry the stage across the MFMA phase.
#define GST_FLOATS (2 * 64 * 128 + 128)
#ifndef DECODE_GLDS
#define DECODE_GLDS 0
#endif
typedef __attribute__((address_space(3))) void* lds_vptr;

__device__ __forceinline__ uint32_t glds_src_off(int j, int lane) {
    const int row = 2 * j + (lane >> 5), pos = lane & 31, pre = pos ^ (row & 15);
    const int q = 8 * (pre >> 3) + 2 * (pre & 3) + ((pre >> 2) & 1);      // natural 4-float chunk
    return 4u * (uint32_t)(row * 128 + 4 * q);
}

__device__ __forceinline__ void glds_issue(rsrc_t lw, rsrc_t lz, rsrc_t lbw, rsrc_t lbz, float* buf, int s, int wave) {
    const int lane = lane_fresh();
    const uint32_t so = 32768u * (uint32_t)s;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = 4 * wave + u;
        const uint32_t vo = glds_src_off(j, lane);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(lw, (lds_vptr)(buf + 256 * j), 16, vo, so, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(lz, (lds_vptr)(buf + 64 * 128 + 256 * j), 16, vo, so, 0, 0);
    }
    if (wave == 0) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(lbw, (lds_vptr)(buf + 2 * 64 * 128), 4, 4u * (uint32_t)lane, 256u * (uint32_t)s, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(lbz, (lds_vptr)(buf + 2 * 64 * 128 + 64), 4, 4u * (uint32_t)lane, 256u * (uint32_t)s, 0, 0);
    }
}

// after this wave's DMAs landed: W+ = fp32(w + fp32(sigma z)), W- = fp32(w - fp32(sigma z)) in place
__device__ __forceinline__ void glds_form(float* buf, int s, int V1, float sigma, int wave) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int lane = lane_fresh();
    float* pw = buf + 256 * (4 * wave) + 4 * lane;
    f32x4 w[4], z[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {                                  // all reads first: one LDS round trip
        w[u] = *reinterpret_cast<const f32x4*>(pw + 256 * u);
        z[u] = *reinterpret_cast<const f32x4*>(pw + 256 * u + 64 * 128);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const f32x4 delta = sigma * z[u];                           // nets.py:102
        *reinterpret_cast<f32x4*>(pw + 256 * u) = w[u] + delta;    // nets.py:113
        *reinterpret_cast<f32x4*>(pw + 256 * u + 64 * 128) = w[u] - delta;   // nic_nes_worker.py:151
    }
    if (wave == 0) {
        float* pb = buf + 2 * 64 * 128 + lane;
        const float bw = pb[0], bz = pb[64];
        const float delta = sigma * bz;
        const bool ok = 64 * s + lane < V1;
        pb[0] = ok ? bw + delta : NEG_INF;
        pb[64] = ok ? bw - delta : NEG_INF;
    }
}

// general stage of two 32-row tiles of a [*, 128] matrix: stage rows 0..31 = matrix rows ra..,
// 32..63 = rb.. (waves 0-3 stage tile a, waves 4-7 tile b); w_r / z_r address the matrix (base +
// byte soffset `mat`), b_r / bz_r its bias vector (element offset `bofs`)
__device__ __forceinline__ void glds_issue2(rsrc_t w_r, rsrc_t z_r, rsrc_t b_r, rsrc_t bz_r, uint32_t mat, uint32_t bofs,
                                            float* buf, uint32_t ra, uint32_t rb, int wave) {
    const int lane = lane_fresh();
    const uint32_t so = mat + 512u * (wave < 4 ? ra : rb);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = 4 * wave + u;
        const uint32_t vo = glds_src_off(j & 15, lane);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(w_r, (lds_vptr)(buf + 256 * j), 16, vo, so, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(z_r, (lds_vptr)(buf + 64 * 128 + 256 * j), 16, vo, so, 0, 0);
    }
    if (wave == 0) {
        const uint32_t rm = min(ra, rb);
        const uint32_t vb = 4u * ((lane < 32 ? ra - rm : rb - rm) + (uint32_t)(lane & 31));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_r, (lds_vptr)(buf + 2 * 64 * 128), 4, vb, 4u * (bofs + rm), 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bz_r, (lds_vptr)(buf + 2 * 64 * 128 + 64), 4, vb, 4u * (bofs + rm), 0, 0);
    }
}

// the same two chains continuing from given accumulators (DMA-staged layout)
__device__ __forceinline__ void mfma_stage64_g_acc(const float* region, const float (&Bop)[64], int lane, f32x16& acc0,
                                                   f32x16& acc1) {
    const int r = lane & 31, hh = lane >> 5;
    const uint32_t lb = (uint32_t)(r * 512) | (uint32_t)(16 * ((4 * hh) ^ (r & 15)));
    const char* base = reinterpret_cast<const char*>(region);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t o = lb ^ (uint32_t)(128 * T + 16 * c);
            a0[c] = *reinterpret_cast<const f32x4*>(base + o);
            a1[c] = *reinterpret_cast<const f32x4*>(base + o + 32 * 512);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], acc1, 0, 0, 0);
        }
    }
}

// two chains over one sign region of a DMA-staged stage (swizzled chunk reads)
__device__ __forceinline__ void mfma_stage64_g(const float* region, const float* bias, const float (&Bop)[64], int lane,
                                               f32x16& acc0, f32x16& acc1) {
    const int r = lane & 31, hh = lane >> 5;
    const uint32_t lb = (uint32_t)(r * 512) | (uint32_t)(16 * ((4 * hh) ^ (r & 15)));   // bytes
    const char* base = reinterpret_cast<const char*>(region);
    acc0 = bias_init(bias, hh);
    acc1 = bias_init(bias + 32, hh);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t o = lb ^ (uint32_t)(128 * T + 16 * c);
            a0[c] = *reinterpret_cast<const f32x4*>(base + o);
            a1[c] = *reinterpret_cast<const f32x4*>(base + o + 32 * 512);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], acc1, 0, 0, 0);
        }
    }
}

__device__ __forceinline__ void records16(RowState& st, const f32x16& P, int vbase) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float L = P[r];
        const int v = vbase + (r & 3) + 8 * (r >> 2);
        const bool c = L > st.r1v;
        st.ev = c ? st.r0v : st.ev;
        st.r0v = c ? st.r1v : st.r0v;
        st.r0i = c ? st.r1i : st.r0i;
        st.r1v = c ? L : st.r1v;
        st.r1i = c ? v : st.r1i;
    }
}

#ifndef DECODE_REC
#define DECODE_REC 1       // 2: newest record + previous record's value only (index as a scalar key)
#endif
// REC 2: per element one compare and three selects. The index is kept as the wave-uniform key
// kbase + (r&3) + 8(r>>2) (vocab index minus this lane half's 4*hh); the previous record keeps
// only its value -- if it lands in the tie window the row takes the exact pass.
__device__ __forceinline__ void records16_k(RowState& st, const f32x16& P, int kbase) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float L = P[r];
        const bool c = L > st.r1v;
        st.r0v = c ? st.r1v : st.r0v;
        st.r1v = c ? L : st.r1v;
        st.r1i = c ? kbase + (r & 3) + 8 * (r >> 2) : st.r1i;
    }
}

// epilogue of one stage: P0 holds vocab vbase + (r&3) + 8(r>>2), P1 the same + 32.
// Record scans run only in the (wave-uniform) case that some lane sees a new running max.
__device__ __forceinline__ void epilogue64(RowState& st, const f32x16& P0, const f32x16& P1, int vbase) {
    float t0 = fmaxf(fmaxf(P0[0], P0[1]), P0[2]);
    float t1 = fmaxf(fmaxf(P1[0], P1[1]), P1[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) {
        t0 = fmaxf(fmaxf(t0, P0[r]), P0[r + 1]);
        t1 = fmaxf(fmaxf(t1, P1[r]), P1[r + 1]);
    }
    const float tmax = fmaxf(fmaxf(t0, P0[15]), fmaxf(t1, P1[15]));
    const float mnew = fmaxf(st.m, tmax);
    const float ml = mnew * LOG2E;
    float s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
#pragma unroll
    for (int r = 0; r < 16; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(P0[r], LOG2E, -ml));
#pragma unroll
    for (int r = 0; r < 16; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(P1[r], LOG2E, -ml));
    st.s = s;
    st.m = mnew;
    if (__any(tmax > st.r1v)) {
#if DECODE_REC == 2
        const int kbase = __builtin_amdgcn_readfirstlane(vbase) & ~7;    // vbase = 64 (s-1) + 4 hh
        records16_k(st, P0, kbase);
        records16_k(st, P1, kbase + 32);
#else
        records16(st, P0, vbase);
        records16(st, P1, vbase + 32);
#endif
    }
}

// online-softmax piece over 8 of the previous stage's logits (chunk T: rows 4T..4T+3 of P0, P1)
__device__ __forceinline__ void softmax_piece(RowState& st, const f32x16& P0, const f32x16& P1, int T) {
    const float t0 = fmaxf(fmaxf(P0[4 * T], P0[4 * T + 1]), fmaxf(P0[4 * T + 2], P0[4 * T + 3]));
    const float t1 = fmaxf(fmaxf(P1[4 * T], P1[4 * T + 1]), fmaxf(P1[4 * T + 2], P1[4 * T + 3]));
    const float mnew = fmaxf(st.m, fmaxf(t0, t1));
    const float ml = mnew * LOG2E;
    float s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
#pragma unroll
    for (int r = 0; r < 4; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(P0[4 * T + r], LOG2E, -ml));
#pragma unroll
    for (int r = 0; r < 4; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(P1[4 * T + r], LOG2E, -ml));
    st.s = s;
    st.m = mnew;
}

// the stage's two MFMA chains with the previous stage's softmax folded in between them (one
// piece per 32-k sub-chunk), so the epilogue VALU issues inside this wave's own MFMA stream;
// the (rare) record scan follows the chains
__device__ __forceinline__ void mfma_stage64_iepi(const float* w, const float* bias, const float (&Bop)[64], int lane,
                                                  f32x16& acc0, f32x16& acc1, RowState& st, const f32x16& P0,
                                                  const f32x16& P1, int vbase) {
    const int hh = lane >> 5;
    const float* row0 = w + (lane & 31) * LDS_ROW + hh * 16;
    const float* row1 = row0 + 32 * LDS_ROW;
    acc0 = bias_init(bias, hh);
    acc1 = bias_init(bias + 32, hh);
    const float m_before = st.r1v;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a0[c] = *reinterpret_cast<const f32x4*>(row0 + T * 32 + 4 * c);
            a1[c] = *reinterpret_cast<const f32x4*>(row1 + T * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], acc1, 0, 0, 0);
        }
        softmax_piece(st, P0, P1, T);
#if DECODE_IEPI >= 2
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);      // A fragments
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // 4 MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // ~4 VALU of the piece
        }
#endif
    }
    if (__any(st.m > m_before)) {            // a new running maximum: scan the records
        records16(st, P0, vbase);
        records16(st, P1, vbase + 32);
    }
}

// exact mode (fallback): first v with fp32((L - m) - lse) == -lse
__device__ __forceinline__ void logit_epilogue_exact(int& best, const f32x16& acc, int vbase, float m, float lse) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int v = vbase + (r & 3) + 8 * (r >> 2);
        const float lp = (acc[r] - m) - lse;
        if (lp == -lse && v < best) best = v;
    }
}

__device__ __forceinline__ bool in_window(float v, float m, float lse) { return ((v - m) - lse) == -lse; }

// ---- the kernel --------------------------------------------------------------------------
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_kernel(DecodeParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sgn = wave >> 2, grp = wave & 3, hh = lane >> 5, li = lane & 31;
    const int member = blockIdx.x, slab = blockIdx.y;
    const int b = slab * 128 + grp * 32 + li;
    const bool row_valid = b < p.B;
    const int bc = row_valid ? b : 0;
    const uint64_t nidx = p.noise_idx[member];
    const float sigma = p.sigma;
    const uint32_t Dbytes = 4u * (uint32_t)p.D;

    const rsrc_t theta_r = make_rsrc(p.theta, Dbytes);
    const rsrc_t noise_r = make_rsrc(p.noise + nidx, Dbytes);
    const rsrc_t fc_r = make_rsrc(p.fc, 4u * (uint32_t)p.B * (uint32_t)p.F);
    // lane-private spill slots (c | h' | 20 partial gate tiles), [slot][lane] per wave
    float* wscr = p.scratch + ((size_t)(member * gridDim.y + slab) * 8 + wave) * (SCR_SLOTS * 64);
    const rsrc_t scr_r = make_rsrc(wscr, SCR_SLOTS * 64 * 4);
    // logit weight / bias views bounded to V1 rows: padding rows of the last stage read 0
    const rsrc_t lw_r = make_rsrc(p.theta + p.off_log_w, 4u * 128u * (uint32_t)p.V1);
    const rsrc_t lz_r = make_rsrc(p.noise + nidx + p.off_log_w, 4u * 128u * (uint32_t)p.V1);
    const rsrc_t lbw_r = make_rsrc(p.theta + p.off_log_b, 4u * (uint32_t)p.V1);
    const rsrc_t lbz_r = make_rsrc(p.noise + nidx + p.off_log_b, 4u * (uint32_t)p.V1);
    const uint32_t lo = 4u * lane;
#define C_SLOT(s) (4u * 64u * (uint32_t)(s))
#define H_SLOT(s) (4u * 64u * (uint32_t)(64 + (s)))
#define P_SLOT(s) (4u * 64u * (uint32_t)(128 + (s)))

    float xB[64], hB[64];
    StageRegs sr;
#if DECODE_PROF
    uint32_t prof_acc[16] = {0};
    int prof_cur = 0;
    unsigned long long prof_t0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(prof_t0)::"memory");
#endif

    // ========== t = 0: x = img_embed(fc) (nets.py:194-195) ==================================
    {
        f32x16 accU[4];
        const int nK = p.F >> 7;
        const int ntile = nK * 4;
        auto desc = [&](int n) {
            TileDesc d;
            d.w_off = (uint32_t)p.off_img_w; d.ld = p.F; d.row0 = 32 * (n & 3); d.nvalid = 32; d.k0 = 128 * (n >> 2);
            d.b_off = (uint32_t)p.off_img_b; d.pad_bias = 0.f;
            return d;
        };
        stage_load(theta_r, noise_r, desc(0), tid, sr);
        stage_store(lds, desc(0), sigma, tid, sr);
        __syncthreads();
        for (int kc = 0; kc < nK; ++kc) {
            const uint32_t frow = 4u * (uint32_t)(bc * p.F + 128 * kc + 4 * hh);
#pragma unroll
            for (int U = 0; U < 4; ++U) {
                const int n = kc * 4 + U;
                if (n + 1 < ntile) stage_load(theta_r, noise_r, desc(n + 1), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_FLOATS;
                if (kc == 0) accU[U] = bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh);
                accU[U] = mfma_tile_fc(accU[U], buf + sgn * SIGN_FLOATS, fc_r, frow, lane);
                if (n + 1 < ntile) stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), sigma, tid, sr);
                __syncthreads();
            }
        }
#pragma unroll
        for (int U = 0; U < 4; ++U)
#pragma unroll
            for (int r = 0; r < 16; ++r) xB[16 * U + r] = accU[U][r];
    }

    int it = 0;
    bool unfinished = true;
    for (int t = 0; t <= p.T; ++t) {
        PROF_STAMP(1);
        // ========== x = embed(it) (nets.py:196-199) =========================================
        if (t > 0) {
            const uint32_t eo = 4u * ((uint32_t)p.off_emb_w + (uint32_t)it * 128u + 4u * hh);
#pragma unroll
            for (int T = 0; T < 4; ++T)
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const f32x4 w = ld4(theta_r, eo + 4u * (32 * T + 8 * a));
                    const f32x4 z = ld4(noise_r, eo + 4u * (32 * T + 8 * a));
                    const f32x4 delta = sigma * z;
                    const f32x4 x = sgn ? (w - delta) : (w + delta);
#pragma unroll
                    for (int c = 0; c < 4; ++c) xB[16 * T + 4 * a + c] = x[c];
                }
        }
        // ========== LSTM cell (nets.py:98-134) ==============================================
        // gate sum s = ((b_i2h + Wi.x) + b_h2h) + Wh.h : one fma chain per gate (the oracle's
        // definition; i2h then h2h as LSTMCore adds them, nets.py:109-111). Tiles 0..19 run the
        // i2h products into 20 lane-private gate-sum slots (slot 5U+q: gate chunk q, units
        // 32U..32U+31); tiles 20..39 add b_h2h + Wh.h in place, so x and h are never live in
        // registers together; then nn_lstm_cell (the oracle's own function) runs per unit.
#if !(DECODE_ABLATE & 4) && DECODE_CELL == 2
        // fused form: one 64-row stage = [Wi rows | Wh rows] of gate tile (q, U); the chain
        // b_i + Wi.x, + b_h, + Wh.h runs in one accumulator, and the gates of a 32-unit block U are
        // folded as they complete (order g1, g2, i, f, o), so only one running value is held.
        {
            auto cell_load = [&](int n, Stage64Regs& r) {
                const int U = n / 5, q = (n % 5 + 3) % 5;        // q order 3, 4, 0, 1, 2
                const uint32_t rowbase = (uint32_t)(q * 128 + 32 * U);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int f = tid + NTHREADS * u, row = (f >> 5) & 31, q4 = f & 31;
                    const uint32_t base = u < 2 ? (uint32_t)p.off_i2h_w : (uint32_t)p.off_h2h_w;
                    const uint32_t off = 4u * (base + (rowbase + (uint32_t)row) * 128u + 4u * (uint32_t)q4);
                    r.w[u] = ld4(theta_r, off);
                    r.z[u] = ld4(noise_r, off);
                }
                const int br = tid & 63;
                const uint32_t bbase = br < 32 ? (uint32_t)p.off_i2h_b : (uint32_t)p.off_h2h_b;
                const uint32_t boff = 4u * (bbase + rowbase + (uint32_t)(br & 31));
                r.bw = ld1(theta_r, boff);
                r.bz = ld1(noise_r, boff);
            };
            Stage64Regs cr;
            cell_load(0, cr);
            stage64_store(lds, 0, 64, sigma, tid, cr);
            __syncthreads();
            f32x16 hold;
            for (int n = 0; n < 20; ++n) {
                cell_load(min(n + 1, 19), cr);
                const float* buf = lds + (n & 1) * STAGE64_FLOATS;
                const float* wsg = buf + sgn * (64 * LDS_ROW);
                const float* bsg = buf + 2 * 64 * LDS_ROW + 64 * sgn;
                f32x16 acc = mfma_tile(bias_init(bsg, hh), wsg, xB, lane);
                acc = acc + bias_init(bsg + 32, hh);
                if (t > 0) acc = mfma_tile(acc, wsg + 32 * LDS_ROW, hB, lane);   // h = 0 at t = 0
                const int U = n / 5, j = n % 5;
                if (j == 0) {                                   // g1
                    hold = acc;
                } else if (j == 1) {                            // g = max(g1, g2)
#pragma unroll
                    for (int r = 0; r < 16; ++r) hold[r] = hold[r] > acc[r] ? hold[r] : acc[r];
                } else if (j == 2) {                            // ig * g
#pragma unroll
                    for (int r = 0; r < 16; ++r) hold[r] = nn_sigmoidf(acc[r]) * hold[r];
                } else if (j == 3) {                            // c' = f * c + ig * g
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float cold = (t == 0) ? 0.f : ld1(scr_r, lo, C_SLOT(16 * U + r));
                        const float fc = nn_sigmoidf(acc[r]) * cold;
                        const float cn = fc + hold[r];
                        st1(scr_r, lo, C_SLOT(16 * U + r), cn);
                        hold[r] = cn;
                    }
                } else {                                        // h' = o * tanh(c')
#pragma unroll
                    for (int r = 0; r < 16; ++r) st1(scr_r, lo, H_SLOT(16 * U + r), nn_sigmoidf(acc[r]) * nn_tanhf(hold[r]));
                }
                stage64_store(lds + ((n + 1) & 1) * STAGE64_FLOATS, 0, 64, sigma, tid, cr);
                __syncthreads();
            }
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = ld1(scr_r, lo, H_SLOT(i));
        }
#elif !(DECODE_ABLATE & 4) && DECODE_CELL == 4
        // cell 3's two passes, with every stage brought in by LDS-DMA and formed in place
        {
            PROF_STAMP(2);
            auto tile_q = [](int m) { const int j = m % 5; return j < 2 ? j + 3 : j - 2; };   // 3,4,0,1,2
            auto rows_of = [&](int j, uint32_t& ra, uint32_t& rb) {
                const int ma = 2 * j, mb = 2 * j + 1;
                ra = (uint32_t)(tile_q(ma) * 128 + 32 * (ma / 5));
                rb = (uint32_t)(tile_q(mb) * 128 + 32 * (mb / 5));
            };
            auto issue = [&](uint32_t w_off, uint32_t b_off, int j, float* buf) {
                uint32_t ra, rb;
                rows_of(j, ra, rb);
                glds_issue2(theta_r, noise_r, theta_r, noise_r, 4u * w_off, b_off, buf, ra, rb, wave);
            };
            // ---- pass 1: b_i + Wi.x -> lane scratch
            issue((uint32_t)p.off_i2h_w, (uint32_t)p.off_i2h_b, 0, lds);
            glds_form(lds, 0, 64, sigma, wave);
            __syncthreads();
            for (int j = 0; j < 10; ++j) {
                float* nbuf = lds + ((j + 1) & 1) * GST_FLOATS;
                if (j < 9) issue((uint32_t)p.off_i2h_w, (uint32_t)p.off_i2h_b, j + 1, nbuf);
                const float* buf = lds + (j & 1) * GST_FLOATS;
                f32x16 a0, a1;
                mfma_stage64_g(buf + sgn * (64 * 128), buf + 2 * 64 * 128 + 64 * sgn, xB, lane_fresh(), a0, a1);
                const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
                const int qa = tile_q(2 * j), qb = tile_q(2 * j + 1), ua = (2 * j) / 5, ub = (2 * j + 1) / 5;
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(scr_r, lo_, P_SLOT(16 * (5 * ua + qa) + r), a0[r]);
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(scr_r, lo_, P_SLOT(16 * (5 * ub + qb) + r), a1[r]);
                if (j < 9) glds_form(nbuf, 0, 64, sigma, wave);
                __syncthreads();
            }
            PROF_STAMP(3);
            // ---- pass 2: + b_h + Wh.h, folded per unit block
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = (t == 0) ? 0.f : ld1(scr_r, lo, H_SLOT(i));
            issue((uint32_t)p.off_h2h_w, (uint32_t)p.off_h2h_b, 0, lds);
            glds_form(lds, 0, 64, sigma, wave);
            __syncthreads();
            f32x16 hold;
            auto fold = [&](int m, const f32x16& acc, uint32_t lo_) {
                const int U = m / 5, j5 = m % 5;
                if (j5 == 0) {                                   // g1
                    hold = acc;
                } else if (j5 == 1) {                            // g = max(g1, g2)
#pragma unroll
                    for (int r = 0; r < 16; ++r) hold[r] = hold[r] > acc[r] ? hold[r] : acc[r];
                } else if (j5 == 2) {                            // ig * g
#pragma unroll
                    for (int r = 0; r < 16; ++r) hold[r] = nn_sigmoidf(acc[r]) * hold[r];
                } else if (j5 == 3) {                            // c' = f * c + ig * g
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float cold = (t == 0) ? 0.f : ld1(scr_r, lo_, C_SLOT(16 * U + r));
                        const float fcv = nn_sigmoidf(acc[r]) * cold;
                        const float cn = fcv + hold[r];
                        st1(scr_r, lo_, C_SLOT(16 * U + r), cn);
                        hold[r] = cn;
                    }
                } else {                                         // h' = o * tanh(c')
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        st1(scr_r, lo_, H_SLOT(16 * U + r), nn_sigmoidf(acc[r]) * nn_tanhf(hold[r]));
                }
            };
            for (int j = 0; j < 10; ++j) {
                const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
                const int ma = 2 * j, mb = 2 * j + 1;
                // scratch partials (and c) are ordinary loads: take them before this stage's DMA
                // is issued, so their waits do not drain it
                f32x16 a0, a1, cpre;
#pragma unroll
                for (int r = 0; r < 16; ++r) a0[r] = ld1(scr_r, lo_, P_SLOT(16 * (5 * (ma / 5) + tile_q(ma)) + r));
#pragma unroll
                for (int r = 0; r < 16; ++r) a1[r] = ld1(scr_r, lo_, P_SLOT(16 * (5 * (mb / 5) + tile_q(mb)) + r));
                const int mf = (ma % 5 == 3) ? ma : mb;          // the f gate of this stage, if any
                const bool has_f = (ma % 5 == 3) || (mb % 5 == 3);
                if (has_f && t > 0) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) cpre[r] = ld1(scr_r, lo_, C_SLOT(16 * (mf / 5) + r));
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                float* nbuf = lds + ((j + 1) & 1) * GST_FLOATS;
                if (j < 9) issue((uint32_t)p.off_h2h_w, (uint32_t)p.off_h2h_b, j + 1, nbuf);
                const float* buf = lds + (j & 1) * GST_FLOATS;
                const float* bsg = buf + 2 * 64 * 128 + 64 * sgn;
                const int hh_ = lane_fresh() >> 5;
                a0 = a0 + bias_init(bsg, hh_);
                a1 = a1 + bias_init(bsg + 32, hh_);
                if (t > 0) mfma_stage64_g_acc(buf + sgn * (64 * 128), hB, lane_fresh(), a0, a1);   // h = 0 at t = 0
                // fold (c for the f gate comes from cpre, not a load behind the DMA)
                auto fold2 = [&](int m, const f32x16& acc) {
                    if (m % 5 == 3) {
                        const int U = m / 5;
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const float cold = (t == 0) ? 0.f : cpre[r];
                            const float fcv = nn_sigmoidf(acc[r]) * cold;
                            const float cn = fcv + hold[r];
                            st1(scr_r, lo_, C_SLOT(16 * U + r), cn);
                            hold[r] = cn;
                        }
                    } else {
                        fold(m, acc, lo_);
                    }
                };
                fold2(ma, a0);
                fold2(mb, a1);
                if (j < 9) glds_form(nbuf, 0, 64, sigma, wave);
                __syncthreads();
            }
            PROF_STAMP(4);
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = ld1(scr_r, lo, H_SLOT(i));
        }
#elif !(DECODE_ABLATE & 4) && DECODE_CELL == 3
        // two passes over 64-row stages (two 32-row gate tiles, two MFMA chains per wave):
        //   pass 1: b_i + Wi.x for every tile -> lane scratch (h not live)
        //   pass 2: partial + b_h + Wh.h, folded per 32-unit block U as the gates complete in
        //           the order g1, g2, i, f, o (x not live): g = max(g1, g2); ig*g; c' = f*c + ig*g;
        //           h' = o*tanh(c') -- the operations of nn_lstm_cell, in its order
        {
            PROF_STAMP(2);
            auto tile_q = [](int m) { const int j = m % 5; return j < 2 ? j + 3 : j - 2; };   // 3,4,0,1,2
            auto cell_load = [&](uint32_t w_off, uint32_t b_off, int j, Stage64Regs& r) {
                const int ma = 2 * j, mb = 2 * j + 1;
                const uint32_t ra = (uint32_t)(tile_q(ma) * 128 + 32 * (ma / 5));
                const uint32_t rb = (uint32_t)(tile_q(mb) * 128 + 32 * (mb / 5));
                const int l = lane_fresh();
                const uint32_t vo = 16u * (uint32_t)(wave * 64 + l);
                const uint32_t sa = 4u * (w_off + ra * 128u), sb = 4u * (w_off + rb * 128u);
                // lane offsets stay non-negative (the buffer range check is on the lane offset)
                const uint32_t rm = min(ra, rb);
                const uint32_t vb = 4u * (uint32_t)(l & 31) + 4u * ((l & 32) ? rb - rm : ra - rm);
                r.bw = ld1(theta_r, vb, 4u * (b_off + rm));
                r.bz = ld1(noise_r, vb, 4u * (b_off + rm));
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t so = (u < 2 ? sa : sb) + 8192u * (uint32_t)(u & 1);
                    r.w[u] = ld4s(theta_r, vo, so);
                    r.z[u] = ld4s(noise_r, vo, so);
                }
            };
            Stage64Regs cr;
            // ---- pass 1
            cell_load((uint32_t)p.off_i2h_w, (uint32_t)p.off_i2h_b, 0, cr);
            stage64_store(lds, 0, 64, sigma, wave * 64 + lane_fresh(), cr);
            __syncthreads();
            for (int j = 0; j < 10; ++j) {
                cell_load((uint32_t)p.off_i2h_w, (uint32_t)p.off_i2h_b, min(j + 1, 9), cr);
                const float* buf = lds + (j & 1) * STAGE64_FLOATS;
                f32x16 a0, a1;
                mfma_stage64(buf + sgn * (64 * LDS_ROW), buf + 2 * 64 * LDS_ROW + 64 * sgn, xB, lane_fresh(), a0, a1);
                const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
                const int qa = tile_q(2 * j), qb = tile_q(2 * j + 1), ua = (2 * j) / 5, ub = (2 * j + 1) / 5;
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(scr_r, lo_, P_SLOT(16 * (5 * ua + qa) + r), a0[r]);
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(scr_r, lo_, P_SLOT(16 * (5 * ub + qb) + r), a1[r]);
                stage64_store(lds + ((j + 1) & 1) * STAGE64_FLOATS, 0, 64, sigma, wave * 64 + lane_fresh(), cr);
                __syncthreads();
            }
            PROF_STAMP(3);
            // ---- pass 2
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = (t == 0) ? 0.f : ld1(scr_r, lo, H_SLOT(i));
            cell_load((uint32_t)p.off_h2h_w, (uint32_t)p.off_h2h_b, 0, cr);
            stage64_store(lds, 0, 64, sigma, wave * 64 + lane_fresh(), cr);
            __syncthreads();
            f32x16 hold;
            auto fold = [&](int m, const f32x16& acc, uint32_t lo_) {
                const int U = m / 5, j5 = m % 5;
                if (j5 == 0) {                                   // g1
                    hold = acc;
                } else if (j5 == 1) {                            // g = max(g1, g2)
#pragma unroll
                    for (int r = 0; r < 16; ++r) hold[r] = hold[r] > acc[r] ? hold[r] : acc[r];
                } else if (j5 == 2) {                            // ig * g
#pragma unroll
                    for (int r = 0; r < 16; ++r) hold[r] = nn_sigmoidf(acc[r]) * hold[r];
                } else if (j5 == 3) {                            // c' = f * c + ig * g
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float cold = (t == 0) ? 0.f : ld1(scr_r, lo_, C_SLOT(16 * U + r));
                        const float fcv = nn_sigmoidf(acc[r]) * cold;
                        const float cn = fcv + hold[r];
                        st1(scr_r, lo_, C_SLOT(16 * U + r), cn);
                        hold[r] = cn;
                    }
                } else {                                         // h' = o * tanh(c')
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        st1(scr_r, lo_, H_SLOT(16 * U + r), nn_sigmoidf(acc[r]) * nn_tanhf(hold[r]));
                }
            };
            for (int j = 0; j < 10; ++j) {
                const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
                const int ma = 2 * j, mb = 2 * j + 1;
                f32x16 a0, a1;
#pragma unroll
                for (int r = 0; r < 16; ++r) a0[r] = ld1(scr_r, lo_, P_SLOT(16 * (5 * (ma / 5) + tile_q(ma)) + r));
#pragma unroll
                for (int r = 0; r < 16; ++r) a1[r] = ld1(scr_r, lo_, P_SLOT(16 * (5 * (mb / 5) + tile_q(mb)) + r));
                __builtin_amdgcn_sched_barrier(0);
                cell_load((uint32_t)p.off_h2h_w, (uint32_t)p.off_h2h_b, min(j + 1, 9), cr);
                const float* buf = lds + (j & 1) * STAGE64_FLOATS;
                const float* bsg = buf + 2 * 64 * LDS_ROW + 64 * sgn;
                const int hh_ = lane_fresh() >> 5;
                a0 = a0 + bias_init(bsg, hh_);
                a1 = a1 + bias_init(bsg + 32, hh_);
                if (t > 0) mfma_stage64_acc(buf + sgn * (64 * LDS_ROW), hB, lane_fresh(), a0, a1);   // h = 0 at t = 0
                fold(ma, a0, lo_);
                fold(mb, a1, lo_);
                stage64_store(lds + ((j + 1) & 1) * STAGE64_FLOATS, 0, 64, sigma, wave * 64 + lane_fresh(), cr);
                __syncthreads();
            }
            PROF_STAMP(4);
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = ld1(scr_r, lo, H_SLOT(i));
        }
#elif !(DECODE_ABLATE & 4)
        {
            PROF_STAMP(2);
            const int ntile = 40;
            auto desc = [&](int n) {
                const int which = n >= 20, m = n - 20 * which, U = m / 5, q = m % 5;
                TileDesc d;
                d.w_off = (uint32_t)(which ? p.off_h2h_w : p.off_i2h_w); d.ld = 128; d.row0 = q * 128 + 32 * U;
                d.nvalid = 32; d.k0 = 0; d.b_off = (uint32_t)(which ? p.off_h2h_b : p.off_i2h_b); d.pad_bias = 0.f;
                return d;
            };
            stage_load(theta_r, noise_r, desc(0), tid, sr);
            stage_store(lds, desc(0), sigma, tid, sr);
            __syncthreads();
            // pass 1: i2h partials (h not live)
            for (int n = 0; n < 20; ++n) {
                stage_load(theta_r, noise_r, desc(n + 1), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_FLOATS;
                const f32x16 acc = mfma_tile(bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh), buf + sgn * SIGN_FLOATS, xB, lane);
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(scr_r, lo, P_SLOT(16 * n + r), acc[r]);
                stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), sigma, tid, sr);
                __syncthreads();
            }
            // pass 2: + b_h2h + Wh.h (x not live)
            PROF_STAMP(3);
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = (t == 0) ? 0.f : ld1(scr_r, lo, H_SLOT(i));
            for (int n = 20; n < ntile; ++n) {
                const int nn = min(n + 1, ntile - 1);
                const int m = n - 20;
                // partials first: vmcnt is in-order, so loads issued after the staging loads
                // would wait for them
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = ld1(scr_r, lo, P_SLOT(16 * m + r));
                __builtin_amdgcn_sched_barrier(0);
                stage_load(theta_r, noise_r, desc(nn), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_FLOATS;
                acc = acc + bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh);
                if (t > 0) acc = mfma_tile(acc, buf + sgn * SIGN_FLOATS, hB, lane);   // h = 0 at t = 0
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(scr_r, lo, P_SLOT(16 * m + r), acc[r]);
                stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(nn), sigma, tid, sr);
                __syncthreads();
            }
            // elementwise cell: c' = f*c + i*max(g1,g2), h' = o*tanh(c')
            PROF_STAMP(4);
            for (int U = 0; U < 4; ++U) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float s0 = ld1(scr_r, lo, P_SLOT(16 * (5 * U + 0) + r));
                    const float s1 = ld1(scr_r, lo, P_SLOT(16 * (5 * U + 1) + r));
                    const float s2 = ld1(scr_r, lo, P_SLOT(16 * (5 * U + 2) + r));
                    const float s3 = ld1(scr_r, lo, P_SLOT(16 * (5 * U + 3) + r));
                    const float s4 = ld1(scr_r, lo, P_SLOT(16 * (5 * U + 4) + r));
                    const float cold = (t == 0) ? 0.f : ld1(scr_r, lo, C_SLOT(16 * U + r));
                    float cn, hn;
                    nn_lstm_cell(s0, s1, s2, s3, s4, cold, &cn, &hn);
                    st1(scr_r, lo, C_SLOT(16 * U + r), cn);
                    st1(scr_r, lo, H_SLOT(16 * U + r), hn);
                }
            }
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = ld1(scr_r, lo, H_SLOT(i));
        }
#else
        if (t == 0) {
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = xB[i];
        }
#endif
        if (t == 0) continue;            // t=0 logits are discarded (nets.py:205-206)

        // ========== logits + log_softmax + greedy argmax (nets.py:202,208-209) ==============
        // 64 vocab rows per LDS stage (two independent 32-row MFMA chains per wave). The two
        // waves sharing a SIMD (w and w+4: opposite signs) run the MFMA chains and the VALU
        // epilogue of the previous stage in opposite orders, so VALU of one wave overlaps the
        // MFMAs of the other. Rows >= V1 read as zero through the bounded buffer resources.
        const int nvt = (p.V1 + 31) >> 5;            // 32-row tiles (exact fallback pass)
        auto desc = [&](int n) {
            TileDesc d;
            d.w_off = (uint32_t)p.off_log_w; d.ld = 128; d.row0 = 32 * n; d.nvalid = min(32, p.V1 - 32 * n); d.k0 = 0;
            d.b_off = (uint32_t)p.off_log_b; d.pad_bias = NEG_INF;
            return d;
        };
        const int nst = (p.V1 + 63) >> 6;
        PROF_STAMP(5);
        RowState st;
        row_state_init(st);
#if DECODE_GLDS
        glds_issue(lw_r, lz_r, lbw_r, lbz_r, lds, 0, wave);
        glds_form(lds, 0, p.V1, sigma, wave);
        __syncthreads();
        f32x16 prev0, prev1;
#pragma unroll
        for (int r = 0; r < 16; ++r) { prev0[r] = NEG_INF; prev1[r] = NEG_INF; }
        for (int s = 0; s < nst; ++s) {
            const bool more = s + 1 < nst;
            float* nbuf = lds + ((s + 1) & 1) * GST_FLOATS;
#if DECODE_PROF >= 2
            PROF_STAMP(8);
#endif
            if (more) glds_issue(lw_r, lz_r, lbw_r, lbz_r, nbuf, s + 1, wave);
#if DECODE_PROF >= 2
            PROF_STAMP(9);
#endif
            const float* buf = lds + (s & 1) * GST_FLOATS;
            const float* wsg = buf + sgn * (64 * 128);
            const float* bsg = buf + 2 * 64 * 128 + 64 * sgn;
            f32x16 acc0, acc1;
            if (sgn == 0) {
                mfma_stage64_g(wsg, bsg, hB, lane_fresh(), acc0, acc1);
                epilogue64(st, prev0, prev1, 64 * (s - 1) + 4 * (lane_fresh() >> 5));
            } else {
                epilogue64(st, prev0, prev1, 64 * (s - 1) + 4 * (lane_fresh() >> 5));
                mfma_stage64_g(wsg, bsg, hB, lane_fresh(), acc0, acc1);
            }
#if DECODE_PROF >= 2
            PROF_STAMP(10);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            PROF_STAMP(12);
#endif
            if (more) glds_form(nbuf, s + 1, p.V1, sigma, wave);
#if DECODE_PROF >= 2
            PROF_STAMP(11);
#endif
            __syncthreads();
#if DECODE_PROF >= 2
            PROF_STAMP(5);
#endif
            prev0 = acc0;
            prev1 = acc1;
        }
#else
#ifdef LOGIT_PRIO_SGN
        if (sgn == LOGIT_PRIO_SGN) __builtin_amdgcn_s_setprio(1);   // static priority for one half
#endif
        Stage64Regs s64;
        stage64_load(lw_r, lz_r, lbw_r, lbz_r, 0, tid, s64);
        stage64_store(lds, 0, p.V1, sigma, tid, s64);
        __syncthreads();
        f32x16 prev0, prev1;
#pragma unroll
        for (int r = 0; r < 16; ++r) { prev0[r] = NEG_INF; prev1[r] = NEG_INF; }
        for (int s = 0; s < nst; ++s) {
#if DECODE_PROF >= 2
            PROF_STAMP(8);
#endif
#if !(DECODE_ABLATE & 2)
            stage64_load(lw_r, lz_r, lbw_r, lbz_r, min(s + 1, nst - 1), wave * 64 + lane_fresh(), s64);
#endif
#if DECODE_PROF >= 2
            PROF_STAMP(9);
#endif
            const float* buf = lds + (s & 1) * STAGE64_FLOATS;
            const float* wsg = buf + sgn * (64 * LDS_ROW);
            const float* bsg = buf + 2 * 64 * LDS_ROW + 64 * sgn;
            f32x16 acc0, acc1;
#if DECODE_IEPI
            mfma_stage64_iepi(wsg, bsg, hB, lane_fresh(), acc0, acc1, st, prev0, prev1, 64 * (s - 1) + 4 * (lane_fresh() >> 5));
            if (false) {
#else
            if (sgn == 0) {
#endif
                mfma_stage64(wsg, bsg, hB, lane_fresh(), acc0, acc1);
#if !(DECODE_ABLATE & 1)
                epilogue64(st, prev0, prev1, 64 * (s - 1) + 4 * (lane_fresh() >> 5));
#endif
            } else {
#if !(DECODE_ABLATE & 1)
                epilogue64(st, prev0, prev1, 64 * (s - 1) + 4 * (lane_fresh() >> 5));
#endif
                mfma_stage64(wsg, bsg, hB, lane_fresh(), acc0, acc1);
            }
#if DECODE_PROF >= 2
            PROF_STAMP(10);
#endif
#if !(DECODE_ABLATE & 2)
            stage64_store(lds + ((s + 1) & 1) * STAGE64_FLOATS, min(s + 1, nst - 1), p.V1, sigma, wave * 64 + lane_fresh(), s64);
#endif
#if DECODE_PROF >= 2
            PROF_STAMP(11);
#endif
#if !(DECODE_ABLATE & 8)
            __syncthreads();
#endif
#if DECODE_PROF >= 2
            PROF_STAMP(5);
#endif
            prev0 = acc0;
            prev1 = acc1;
        }
#endif
        epilogue64(st, prev0, prev1, 64 * (nst - 1) + 4 * hh);
#ifdef LOGIT_PRIO_SGN
        __builtin_amdgcn_s_setprio(0);
#endif
        PROF_STAMP(6);
        // merge the two lane halves that share this batch row
        const float m_o = __shfl_xor(st.m, 32);
        const float s_o = __shfl_xor(st.s, 32);
        const float m = fmaxf(st.m, m_o);
        const float stot = st.s * __builtin_amdgcn_exp2f((st.m - m) * LOG2E) + s_o * __builtin_amdgcn_exp2f((m_o - m) * LOG2E);
        const float lse = logf(stot);
        int tok = 0x7fffffff;
#if DECODE_REC == 2
        {
            const int own = (int)((uint32_t)st.r1i + 4u * (uint32_t)hh);   // key -> vocab index of this lane half
            const float cv[2] = {st.r1v, __shfl_xor(st.r1v, 32)};
            const int ci[2] = {own, __shfl_xor(own, 32)};
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (in_window(cv[k], m, lse) && ci[k] < tok) tok = ci[k];
        }
        const bool ovf = p.force_exact || in_window(st.r0v, m, lse) || in_window(__shfl_xor(st.r0v, 32), m, lse);
#else
        {
            const float cv[4] = {st.r0v, st.r1v, __shfl_xor(st.r0v, 32), __shfl_xor(st.r1v, 32)};
            const int ci[4] = {st.r0i, st.r1i, __shfl_xor(st.r0i, 32), __shfl_xor(st.r1i, 32)};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (in_window(cv[k], m, lse) && ci[k] < tok) tok = ci[k];
        }
        const bool ovf = p.force_exact || in_window(st.ev, m, lse) || in_window(__shfl_xor(st.ev, 32), m, lse);
#endif
        if (__syncthreads_or(ovf ? 1 : 0)) {
            // rare: more records than tracked fall in the tie window -> exact second pass
            int best = 0x7fffffff;
            stage_load(theta_r, noise_r, desc(0), tid, sr);
            stage_store(lds, desc(0), sigma, tid, sr);
            __syncthreads();
            for (int n = 0; n < nvt; ++n) {
                if (n + 1 < nvt) stage_load(theta_r, noise_r, desc(n + 1), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_FLOATS;
                const f32x16 acc = mfma_tile(bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh), buf + sgn * SIGN_FLOATS, hB, lane);
                if (n + 1 < nvt) stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), sigma, tid, sr);
                logit_epilogue_exact(best, acc, 32 * n + 4 * hh, m, lse);
                __syncthreads();
            }
            tok = min(best, __shfl_xor(best, 32));
            if (tid == 0) atomicAdd(p.stats + 0, 1);
        }
        // no candidate only when every logit is NaN (torch.max would return a NaN's index):
        // end the caption instead of emitting an out-of-vocabulary id
        if (tok >= p.V1) tok = 0;
        // finished mask (nets.py:236-243)
        unfinished = unfinished && (tok > 0);
        it = unfinished ? tok : 0;
#if !DECODE_PROF
        if (hh == 0 && row_valid) p.seq[(((size_t)member * 2 + sgn) * p.B + b) * p.T + (t - 1)] = it;
#endif
        if (t == p.T) break;
        if (!__syncthreads_or((unfinished && row_valid) ? 1 : 0)) break;
    }
#if DECODE_PROF
    PROF_STAMP(7);
    if (lane == 0 && p.seq && slab == 0)
        for (int k = 0; k < 16; ++k) p.seq[(size_t)member * 2 * p.B * p.T + wave * 16 + k] = (int32_t)prof_acc[k];
#endif
#undef C_SLOT
#undef H_SLOT
#undef P_SLOT
}

extern "C" hipError_t nicnes_launch_decode(const DecodeParams* p, int member_count, int nslabs, hipStream_t stream) {
    const size_t lds_bytes = (size_t)(2 * STAGE64_FLOATS) * sizeof(float);   // >= 2 * STAGE_FLOATS
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)nicnes_decode_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(nicnes_decode_kernel, dim3(member_count, nslabs), dim3(NTHREADS), lds_bytes, stream, *p);
    return hipGetLastError();
}

extern "C" size_t nicnes_decode_scratch_floats(int member_count, int nslabs) {
    return (size_t)member_count * nslabs * 8 * SCR_SLOTS * 64;
}
