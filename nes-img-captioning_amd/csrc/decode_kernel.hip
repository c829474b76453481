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
// Perturbed weights are never materialised in HBM: each weight stage is formed in LDS as
// fp32(W0 +/- fp32(sigma * z[idx + offset])) from the base theta and the member's noise slice,
// once for both signs.
//
// Step structure (step_body; every step t = -1..T of a workgroup in one launch, nicnes_decode_steps_kernel):
// the logit GEMM of step t over h_t, the greedy token, then the LSTM cell of step t+1, whose gate sums
// i2h(x) + h2h(h) (nets.py:109-111) use h_t while it is still the live B operand. The cell runs as 20
// stages, one per 32-unit gate tile (i2h rows | h2h rows), folded per unit block as the gates complete
// (order g1, g2, i, f, o); only c' and h' cross to the next step, in lane scratch. Other paths: the coop
// kernel (S workgroups per member slab in one launch), the 64-row-slab steps2 kernel, the split path.
//
// Addressing: every global access goes through a buffer resource (wave-uniform 128-bit
// descriptor + 32-bit lane offset) so no 64-bit VGPR address pairs are kept live. Lane-derived
// offsets inside the stage loops are recomputed at use (lane_fresh) rather than held: the
// compiler would otherwise spill them and reload them behind in-flight staging loads.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nicnes_math.h"
#include "decode_kernel.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

#define NTHREADS 512
#define LDS_ROW 132                                   // 128 k + 4 pad: conflict-free b128 reads
#define SIGN_FLOATS (32 * LDS_ROW)
#define STAGE_FLOATS (2 * SIGN_FLOATS + 64)           // 32-row stage: W+ | W- | bias+ (32) | bias- (32)
#define STAGE64_FLOATS (2 * 64 * LDS_ROW + 128)       // 64-row stage: W+ | W- | bias+ (64) | bias- (64)
#define LOG2E 1.44269504088896340736f
#define NEG_INF (-__builtin_inff())

#ifndef DECODE_ABLATE
#define DECODE_ABLATE 0    // timing-only builds (scripts/ablate.py): 1 no logit epilogue, 4 no exp-sum, 2 no stage
#endif                     // staging, 8 no stage-loop barrier, 16 no cell activations, 64 no early
                           // exit, 128 no coop hand-off waits, 256 no sampled logit stores, 512 no sampled
                           // pick -- wrong results
#if DECODE_ABLATE & 16
#define CELL_SIG(x) ((x) * 0.5f)
#define CELL_TANH(x) ((x) * 0.25f)
#else
#define CELL_SIG(x) nn_sigmoidf(x)
#define CELL_TANH(x) nn_tanhf(x)
#endif
#ifndef NICNES_STORE_WAITS
#define NICNES_STORE_WAITS 1  // the product: wait states after the sampled pick's 16-byte record stores (gfx950
#endif                        // store-data hazard); 0 only in the scan's scratch build (tests/test_isa_hazards.py)
// The product's structural choices are fixed in the code below; each alternative was measured and dropped (DESIGN.md
// sections 5 and 10 and the git history up to round 5): the other sign's waves first in the logit stages, one launch
// per step, the 32-row-stage image projection on the fused path, no cross-phase prefetch / h read-back, the W+- store
// at the end of a stage, other mid-stage store positions, the unpeeled stage loop in the greedy steps kernels, sc1 loads
// of the coop hand-offs, s_setprio for half the waves, other cache policies of the sampled logit stores.
#define LOGIT_MID_AT 6     // logit stages: the next stage's W+- tile is stored before half-chunk 6 of 8
#ifndef DECODE_PROF
#define DECODE_PROF 0      // timing-only build: per-workgroup start/end s_memrealtime (100 MHz) of every
#endif                     // launch written over seq[wg * 4096 + slot] (wrong tokens; scripts/ablate.py)
#if DECODE_PROF
// (wgi, stride): the fused path keeps 4096 ints per workgroup (one per member: seq holds 2*B*T ints per
// member); the split path 1024 per workgroup (S * slabs <= 4 workgroups per member, slots < 256)
#define PROF_AT(wgi, stride, slot)                                                               \
    do {                                                                                         \
        if (threadIdx.x == 0) {                                                                  \
            unsigned long long t_, k_;                                                           \
            asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_), "=s"(k_)::"memory"); \
            unsigned hw_, xcc_;                                                                  \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                     \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                   \
            int32_t* q_ = p.seq + (size_t)(wgi) * (stride);                                      \
            q_[(slot)] = (int32_t)(uint32_t)t_;                                                  \
            q_[(stride) / 2 + (slot)] = (int32_t)(((xcc_ & 15u) << 16) | ((hw_ >> 8) & 0xffffu)); \
            q_[(stride) / 4 + (slot)] = (int32_t)(uint32_t)k_;                                   \
        }                                                                                        \
    } while (0)
#define PROF_MARK(slot) PROF_AT(blockIdx.x * gridDim.y + blockIdx.y, 4096, slot)
#define PROF_SPLIT(slot) PROF_AT((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, 1024, slot)
#else
#define PROF_AT(wgi, stride, slot) do { } while (0)
#define PROF_MARK(slot) do { } while (0)
#define PROF_SPLIT(slot) do { } while (0)
#endif

// lane id recomputed at the point of use (volatile: never hoisted or kept live across a loop)
__device__ __forceinline__ int lane_fresh() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// pins a loaded value in its register: without it the compiler may re-issue the (provably
// invariant) scratch load at every use inside a stage loop, behind the in-flight staging loads
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }

// ---- buffer helpers ------------------------------------------------------------------------
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 ld4(rsrc_t r, uint32_t byte_off, uint32_t soff = 0) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, (int)soff, 0));
}
__device__ __forceinline__ float ld1(rsrc_t r, uint32_t byte_off, uint32_t soff = 0) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, (int)soff, 0));
}
__device__ __forceinline__ void st1(rsrc_t r, uint32_t byte_off, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)byte_off, (int)soff, 0);
}

// ---- 32-row tiles (image projection, exact tie pass) ---------------------------------------
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

__device__ __forceinline__ void stage_store(float* buf, const TileDesc& d, int tid, const StageRegs& s) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = tid + NTHREADS * u, row = f >> 5, q = f & 31;
        const int T = q >> 3, hh = q & 1, a = (q & 7) >> 1;
        const int o = row * LDS_ROW + T * 32 + hh * 16 + 4 * a;
        const f32x4 delta = s.z[u];                   // fp32(sigma * z) from the sigma-scaled table, nets.py:102
        *reinterpret_cast<f32x4*>(buf + o) = s.w[u] + delta;            // nets.py:113
        *reinterpret_cast<f32x4*>(buf + SIGN_FLOATS + o) = s.w[u] - delta;   // nic_nes_worker.py:151
    }
    {   // slot (tid & 63): bias+ rows 0..31, bias- rows 32..63 (every wave writes the same values)
        const int r = tid & 31;
        const float delta = s.bz;
        const float v = (tid & 32) ? s.bw - delta : s.bw + delta;
        buf[2 * SIGN_FLOATS + (tid & 63)] = r < d.nvalid ? v : d.pad_bias;
    }
}

// ---- a mutated member's delta' formed in the decode (MutHead, decode_kernel.h) -----------------------
// fp32(sigma z) / s or fp32(sigma z) * s: the arithmetic of nicnes_mutate_kernel (update_kernels.hip, mutate1)
__device__ __forceinline__ f32x4 mut_delta(const f32x4& z, const f32x4& v, int mode) {
    f32x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = mode == 1 ? z[e] / v[e] : z[e] * v[e];
    return r;
}

// the member's sigma-scaled table slice and the mutation vector over the parameters below off_log_w
struct MutRes {
    rsrc_t head_r, vec_r;
    int mode;
};
__device__ __forceinline__ MutRes mut_res(const DecodeParams& p, const MutHead& mh, int member) {
    MutRes m;
    m.head_r = make_rsrc(mh.head_noise + mh.head_idx[member], 4u * (uint32_t)p.off_log_w);
    m.vec_r = make_rsrc(mh.mut_vec, 4u * (uint32_t)p.off_log_w);
    m.mode = mh.mode;
    return m;
}

// stage_load / stage_store of a mutated member's image projection: z from the table slice, s from the vector,
// delta' formed at the store (the loads' latency stays hidden behind the tile's MFMAs)
struct StageRegsM {
    StageRegs r;
    f32x4 v[2];
    float bv;
};
__device__ __forceinline__ void stage_load_m(rsrc_t theta_r, const MutRes& m, const TileDesc& d, int tid, StageRegsM& s) {
    stage_load(theta_r, m.head_r, d, tid, s.r);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int f = tid + NTHREADS * u, row = f >> 5, q = f & 31;
        const int rc = row < d.nvalid ? row : max(d.nvalid - 1, 0);
        s.v[u] = ld4(m.vec_r, 4u * (d.w_off + (uint32_t)((d.row0 + rc) * d.ld + d.k0 + 4 * q)));
    }
    const int r = tid & 31;
    s.bv = ld1(m.vec_r, 4u * (d.b_off + (uint32_t)(d.row0 + (r < d.nvalid ? r : 0))));
}
__device__ __forceinline__ void stage_store_m(float* buf, const TileDesc& d, int tid, const StageRegsM& s, int mode) {
    StageRegs t = s.r;
#pragma unroll
    for (int u = 0; u < 2; ++u) t.z[u] = mut_delta(s.r.z[u], s.v[u], mode);
    t.bz = mode == 1 ? s.r.bz / s.bv : s.r.bz * s.bv;
    stage_store(buf, d, tid, t);
}

// ---- MFMA tiles: acc += W_tile(32 x 128, LDS) . B(128 x 32, registers) -----------------------
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

// ---- 64-row stages: two 32-row tiles (a: stage rows 0-31, b: 32-63) -------------------------
struct Stage64Regs {
    f32x4 w[4], z[4];
    float bw, bz;
};

// Where a stage's rows come from: weight rows via w_r / z_r at byte offsets so_a / so_b (tile a /
// tile b), bias via b_r / bz_r at byte offset bso plus a lane offset bda (lanes 0-31) / bdb
// (lanes 32-63); bias rows at or past `valid` (stage row index) are padding.
struct StageSrc {
    rsrc_t w_r, z_r, b_r, bz_r;
    uint32_t so_a, so_b, bso, bda, bdb;
    int valid;
};

// thread tid loads row (tid>>5) + 16u, k 4*(tid&31): one lane offset for every load, the tile and
// chunk offsets ride in the scalar offset
__device__ __forceinline__ void stage64_load(const StageSrc& S, int tid, Stage64Regs& r) {
    const uint32_t vo = 16u * (uint32_t)(tid & 511);
    const int l = tid & 63;
    const uint32_t vb = 4u * (uint32_t)(l & 31) + ((l & 32) ? S.bdb : S.bda);
    r.bw = ld1(S.b_r, vb, S.bso);
    r.bz = ld1(S.bz_r, vb, S.bso);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        // row (tid>>5) + 16(u&1) of tile a (u < 2) or b: byte 16 tid + 8192 (u&1) of that tile
        const uint32_t so = (u < 2 ? S.so_a : S.so_b) + 8192u * (uint32_t)(u & 1);
        r.w[u] = ld4(S.w_r, vo, so);
        r.z[u] = ld4(S.z_r, vo, so);
    }
}

__device__ __forceinline__ void stage64_store(float* buf, int valid, int tid, const Stage64Regs& r) {
    // thread tid writes rows (tid >> 5) + 16u: one base offset, the row step rides in the ds offset
    const int q = tid & 31;
    float* b = buf + (tid >> 5) * LDS_ROW + (q >> 3) * 32 + (q & 1) * 16 + 4 * ((q & 7) >> 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const f32x4 delta = r.z[u];                   // fp32(sigma * z) from the sigma-scaled table, nets.py:102
        *reinterpret_cast<f32x4*>(b + 16 * u * LDS_ROW) = r.w[u] + delta;                  // nets.py:113
        *reinterpret_cast<f32x4*>(b + (64 + 16 * u) * LDS_ROW) = r.w[u] - delta;           // nic_nes_worker.py:151
    }
    const int row = tid & 63, sg = (tid >> 6) & 1;     // every pair of waves writes all 128 slots
    const float delta = r.bz;
    const float v = sg ? r.bw - delta : r.bw + delta;
    buf[2 * 64 * LDS_ROW + 64 * sg + row] = row < valid ? v : NEG_INF;
}

// Per-lane offsets of the logit stage loop, computed once per kernel (the loop would otherwise
// recompute them from the lane id at every stage): global load byte offset, LDS store float offset,
// MFMA A-operand row float offset, bias slot.
struct LaneOffs {
    uint32_t vo;      // 16 * tid: row (tid >> 5) + 16u, k 4 * (tid & 31) of a 32-row tile
    uint32_t vb;      // bias: 4 * (lane & 31) + tile-b byte offset for lanes 32..63
    int so;           // LDS float offset of this thread's first staged f32x4
    int arow;         // A-operand row of this lane: (lane & 31) * LDS_ROW + 16 * (lane >> 5)
    int bslot;        // bias slot: 64 * sign + row
};

__device__ __forceinline__ LaneOffs lane_offs(int wave, uint32_t bdb) {
    LaneOffs o;
    const int lane = lane_fresh(), tid = wave * 64 + lane, q = tid & 31;
    o.vo = 16u * (uint32_t)tid;
    o.vb = 4u * (uint32_t)(lane & 31) + ((lane & 32) ? bdb : 0u);
    o.so = (tid >> 5) * LDS_ROW + (q >> 3) * 32 + (q & 1) * 16 + 4 * ((q & 7) >> 1);
    o.arow = (lane & 31) * LDS_ROW + 16 * (lane >> 5);
    o.bslot = 64 * ((tid >> 6) & 1) + (tid & 63);
    return o;
}

__device__ __forceinline__ void stage64_load_o(const StageSrc& S, const LaneOffs& o, bool bias, Stage64Regs& r) {
    if (bias) {                                       // waves 0 and 1 stage the 2 x 64 bias slots
        r.bw = ld1(S.b_r, o.vb, S.bso);
        r.bz = ld1(S.bz_r, o.vb, S.bso);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t so = (u < 2 ? S.so_a : S.so_b) + 8192u * (uint32_t)(u & 1);
        r.w[u] = ld4(S.w_r, o.vo, so);
        r.z[u] = ld4(S.z_r, o.vo, so);
    }
}

__device__ __forceinline__ void stage64_store_o(float* buf, int valid, const LaneOffs& o, bool bias,
                                                const Stage64Regs& r) {
    float* b = buf + o.so;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const f32x4 delta = r.z[u];                   // fp32(sigma * z) from the sigma-scaled table, nets.py:102
        *reinterpret_cast<f32x4*>(b + 16 * u * LDS_ROW) = r.w[u] + delta;                  // nets.py:113
        *reinterpret_cast<f32x4*>(b + (64 + 16 * u) * LDS_ROW) = r.w[u] - delta;           // nic_nes_worker.py:151
    }
    if (bias) {
        const float delta = r.bz;
        const float v = o.bslot >= 64 ? r.bw - delta : r.bw + delta;
        buf[2 * 64 * LDS_ROW + o.bslot] = (o.bslot & 63) < valid ? v : NEG_INF;
    }
}

// two independent accumulator chains (stage rows 0-31 and 32-63) over the same B
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

struct NoMid {
    __device__ __forceinline__ void operator()() const {}
};

// mid() runs before half-chunk MID of the 8 (8: after the last MFMA; 9: never): the logit loop's W+- store
// of the next stage and the loads of the one after
template <int MID = 8, class Mid = NoMid>
__device__ __forceinline__ void mfma_stage64_o(const float* w, const float* bias, const float (&Bop)[64], int arow,
                                               int hh, f32x16& acc0, f32x16& acc1, Mid&& mid = Mid()) {
    const float* row0 = w + arow;
    const float* row1 = row0 + 32 * LDS_ROW;
    acc0 = bias_init(bias, hh);
    acc1 = bias_init(bias + 32, hh);
    auto at = [&](int h) __attribute__((always_inline)) {   // mid() before half-chunk h (8 halves of 8 k pairs)
        if (h == MID) {
            __builtin_amdgcn_sched_barrier(0);
            mid();
            __builtin_amdgcn_sched_barrier(0);
        }
    };
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        at(2 * T);
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a0[c] = *reinterpret_cast<const f32x4*>(row0 + T * 32 + 4 * c);
            a1[c] = *reinterpret_cast<const f32x4*>(row1 + T * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            if (jj == 8) at(2 * T + 1);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], acc1, 0, 0, 0);
        }
    }
    at(8);
}

template <int MID = 8, class Mid = NoMid>
__device__ __forceinline__ f32x16 mfma_tile_o(f32x16 acc, const float* w, const float (&Bop)[64], int arow,
                                              Mid&& mid = Mid()) {
    const float* row = w + arow;
    auto at = [&](int h) __attribute__((always_inline)) {
        if (h == MID) {
            __builtin_amdgcn_sched_barrier(0);
            mid();
            __builtin_amdgcn_sched_barrier(0);
        }
    };
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        at(2 * T);
        f32x4 a[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) a[c] = *reinterpret_cast<const f32x4*>(row + T * 32 + 4 * c);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            if (jj == 8) at(2 * T + 1);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[jj >> 2][jj & 3], Bop[16 * T + jj], acc, 0, 0, 0);
        }
    }
    at(8);
    return acc;
}

// cell stage: chain a = i2h tile (stage rows 0-31) over B = x, chain b = h2h tile (rows 32-63)
// over B = h; k chunks [T0, T1) of 32 (init: start from the bias)
template <int T0, int T1, bool H = true, bool X = true>
__device__ __forceinline__ void mfma_xh_part(const float* w, const float* bias, const float (&Bx)[64],
                                             const float (&Bh)[64], int lane, f32x16& acc0, f32x16& acc1) {
    const int hh = lane >> 5;
    const float* row0 = w + (lane & 31) * LDS_ROW + hh * 16;
    const float* row1 = row0 + 32 * LDS_ROW;
    if (T0 == 0) {
        if (X) acc0 = bias_init(bias, hh);
        acc1 = bias_init(bias + 32, hh);                 // H = false (h = 0): h2h(h) is its bias
    }
#pragma unroll
    for (int T = T0; T < T1; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (X) a0[c] = *reinterpret_cast<const f32x4*>(row0 + T * 32 + 4 * c);
            if (H) a1[c] = *reinterpret_cast<const f32x4*>(row1 + T * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            if (X) acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bx[16 * T + jj], acc0, 0, 0, 0);
            if (H) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bh[16 * T + jj], acc1, 0, 0, 0);
        }
    }
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

// Lane holds logits for vocab vbase + (r&3) + 8(r>>2), increasing in r. The greedy token is the
// earliest record (left-to-right maximum) inside the log_softmax tie window of the final max;
// each lane half keeps its last two records and the largest record it evicted, so an
// overflowing row is detected and decoded by the exact pass.
// records4: the record update over P[4k .. 4k+3] (vocab vbase + 8k + 0..3, in index order)
template <int K>
__device__ __forceinline__ void records4(RowState& st, const f32x16& P, int vbase) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float L = P[4 * K + e];
        const int v = vbase + 8 * K + e;
        const bool c = L > st.r1v;
        st.ev = c ? st.r0v : st.ev;
        st.r0v = c ? st.r1v : st.r0v;
        st.r0i = c ? st.r1i : st.r0i;
        st.r1v = c ? L : st.r1v;
        st.r1i = c ? v : st.r1i;
    }
}

__device__ __forceinline__ float max4(const f32x16& P, int k) {
    return fmaxf(fmaxf(fmaxf(P[4 * k], P[4 * k + 1]), P[4 * k + 2]), P[4 * k + 3]);
}

// v_max3 / v_max without the quieting copies LLVM puts in front of fmaxf on values it cannot prove
// canonical (every MFMA result): logits are NaN-free except in the all-NaN edge case, where the
// greedy rule ends the caption anyway (tok >= V1 -> 0)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// maximum of 15 + 1 values: 5 + 2 v_max3
__device__ __forceinline__ float vmax16(const f32x16& A) {
    const float a0 = vmax3(A[0], A[1], A[2]), a1 = vmax3(A[3], A[4], A[5]), a2 = vmax3(A[6], A[7], A[8]);
    const float a3 = vmax3(A[9], A[10], A[11]), a4 = vmax3(A[12], A[13], A[14]);
    return vmax3(vmax3(a0, a1, a2), a3, vmax2(a4, A[15]));
}

// record scans of one stage, run only in the (wave-uniform) case that some lane sees a new running
// max in it: per group of 4 consecutive vocab ids, again only where a lane's group max is a record
__device__ __forceinline__ void records_scan(RowState& st, const f32x16& P, int vbase) {
    const float g0 = max4(P, 0), g1 = max4(P, 1), g2 = max4(P, 2), g3 = max4(P, 3);
    if (__any(g0 > st.r1v)) records4<0>(st, P, vbase);
    if (__any(g1 > st.r1v)) records4<1>(st, P, vbase);
    if (__any(g2 > st.r1v)) records4<2>(st, P, vbase);
    if (__any(g3 > st.r1v)) records4<3>(st, P, vbase);
}

// online exp-sum: s = s * e^(m - mnew) + sum_r e^(P[r] - mnew), in vocab order
__device__ __forceinline__ void expsum16(float& s, const f32x16& P, float ml) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(P[r], LOG2E, -ml));
}

// epilogue of one logit stage: P0 holds vocab vbase + (r&3) + 8(r>>2), P1 the same + 32.
// Per stage and lane: 15 v_max3/v_max for the stage max, then 3 VALU per logit for the exp-sum; the
// record scans run only in stages that raise some lane's running max (few once it settles).
// PAIRS (greedy-only decodes, no log-prob output): the exp-sum runs over the maxima of adjacent
// pairs, a lower bound s of the row's sum with the true sum in [s, 2s]; that fixes lse to within
// ln 2, which is all the tie window needs except near a binade edge (tie_window / win_state).
template <bool PAIRS>
__device__ __forceinline__ void epilogue64(RowState& st, const f32x16& P0, const f32x16& P1, int vbase) {
    if constexpr (PAIRS) {
        float q[16];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            q[r] = vmax2(P0[2 * r], P0[2 * r + 1]);
            q[8 + r] = vmax2(P1[2 * r], P1[2 * r + 1]);
        }
        const float a0 = vmax3(q[0], q[1], q[2]), a1 = vmax3(q[3], q[4], q[5]), a2 = vmax3(q[6], q[7], q[8]);
        const float a3 = vmax3(q[9], q[10], q[11]), a4 = vmax3(q[12], q[13], q[14]);
        const float tmax = vmax3(vmax3(a0, a1, a2), a3, vmax2(a4, q[15]));
        if (__any(tmax > st.r1v)) {
            records_scan(st, P0, vbase);
            records_scan(st, P1, vbase + 32);
        }
        const float mnew = vmax2(st.m, tmax);
        const float ml = mnew * LOG2E;
        float s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
#pragma unroll
        for (int r = 0; r < 16; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(q[r], LOG2E, -ml));
        st.s = s;
        st.m = mnew;
        return;
    }
    const float tmax = vmax2(vmax16(P0), vmax16(P1));
    if (__any(tmax > st.r1v)) {
        records_scan(st, P0, vbase);
        records_scan(st, P1, vbase + 32);
    }
    const float mnew = vmax2(st.m, tmax);
    const float ml = mnew * LOG2E;
    float s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
#if !(DECODE_ABLATE & 4)
    expsum16(s, P0, ml);
    expsum16(s, P1, ml);
#else
    s += 64.0f;
#endif
    st.s = s;
    st.m = mnew;
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

// Tie window from a merged row state (m, s). Exact mode: lse = log(s) and in_window. PAIRS mode: s
// bounds the sum within a factor 2, so lse lies in [log s, log s + ln 2] (widened by p.lse_margin,
// 2e-3, for the fp32 sums and v_exp_f32). The window test fp32(d - lse) == -lse (d = x - m <= 0, lse >= 0) holds
// iff e = -d < ulp(lse) / 2, fails iff e > ulp(lse) / 2, and at e == ulp / 2 depends on lse's last
// bit, which no fp32 sum order pins (the reference's own lse bits are torch's): that tie is taken as
// in the window, as a candidate at exactly half an ulp is by round-half-even for an even lse. With
// hu_in / hu_out the half-ulps of the lowest / highest binade lse can be in, e <= hu_in is in,
// e > hu_out is out; between them (lse's binade is not fixed by the bounds) the row goes to the exact pass.
struct TieWindow {
    float lse, hu_in, hu_out;
    bool pairs;
};

__device__ __forceinline__ float binade_half_ulp(float a) {       // a > 0: 2^(E - 24) for a in [2^E, 2^(E+1))
    const uint32_t ex = __builtin_bit_cast(uint32_t, a) >> 23;
    return ex > 24u ? __builtin_bit_cast(float, (ex - 24u) << 23) : 0.f;
}

__device__ __forceinline__ TieWindow tie_window(float s, bool pairs, float margin) {
    TieWindow w;
    w.pairs = pairs;
    w.lse = logf(s);
    w.hu_in = w.hu_out = 0.f;
    if (pairs) {
        const float lo = w.lse - margin, hi = w.lse + (0.69314718f + margin);
        w.hu_in = lo > 0.f ? binade_half_ulp(lo) : 0.f;
        w.hu_out = binade_half_ulp(hi);
    }
    return w;
}

// 1 in the window, 0 out, 2 undecided (PAIRS mode only)
__device__ __forceinline__ int win_state(float v, float m, const TieWindow& w) {
    if (!w.pairs) return in_window(v, m, w.lse) ? 1 : 0;
    const float e = m - v;
    if (e == 0.f || e <= w.hu_in) return 1;
    if (!(e <= w.hu_out)) return 0;                 // also NaN and unset (-inf) records
    return 2;
}

// One sweep of the exact fallback over the whole vocabulary in 32-row tiles: sum mode accumulates the
// row's exp-sum relative to m (PAIRS mode has no usable lse), otherwise the first id in the window
__device__ __forceinline__ void exact_sweep(float* lds, const DecodeParams& p, rsrc_t theta_r, rsrc_t noise_r,
                                            int tid, int sgn, int hh, int lane, const float (&hB)[64],
                                            bool active, bool sum_mode, float m, float lse, float& s, int& best) {
    const int nvt = (p.V1 + 31) >> 5;
    auto desc = [&](int n) {
        TileDesc d;
        d.w_off = (uint32_t)p.off_log_w; d.ld = 128; d.row0 = 32 * n; d.nvalid = min(32, p.V1 - 32 * n); d.k0 = 0;
        d.b_off = (uint32_t)p.off_log_b; d.pad_bias = NEG_INF;
        return d;
    };
    const float ml = m * LOG2E;
    StageRegs sr;
    stage_load(theta_r, noise_r, desc(0), tid, sr);
    stage_store(lds, desc(0), tid, sr);
    __syncthreads();
    for (int n = 0; n < nvt; ++n) {
        if (n + 1 < nvt) stage_load(theta_r, noise_r, desc(n + 1), tid, sr);
        const float* buf = lds + (n & 1) * STAGE_FLOATS;
        if (active) {
            const f32x16 acc = mfma_tile(bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh), buf + sgn * SIGN_FLOATS, hB, lane);
            if (sum_mode) {
#pragma unroll
                for (int r = 0; r < 16; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[r], LOG2E, -ml));
            } else {
                logit_epilogue_exact(best, acc, 32 * n + 4 * hh, m, lse);
            }
        }
        if (n + 1 < nvt) stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), tid, sr);
        __syncthreads();
    }
}


// epilogue of one 32-row logit tile (G = 2: one tile per wave); P0 holds vocab vbase + (r&3) + 8(r>>2)
template <bool PAIRS>
__device__ __forceinline__ void epilogue32(RowState& st, const f32x16& P0, int vbase) {
    if constexpr (PAIRS) {
        float q[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) q[r] = vmax2(P0[2 * r], P0[2 * r + 1]);
        const float tmax = vmax3(vmax3(q[0], q[1], q[2]), vmax3(q[3], q[4], q[5]), vmax2(q[6], q[7]));
        if (__any(tmax > st.r1v)) records_scan(st, P0, vbase);
        const float mnew = vmax2(st.m, tmax);
        const float ml = mnew * LOG2E;
        float s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
#pragma unroll
        for (int r = 0; r < 8; ++r) s += __builtin_amdgcn_exp2f(__builtin_fmaf(q[r], LOG2E, -ml));
        st.s = s;
        st.m = mnew;
        return;
    }
    const float tmax = vmax16(P0);
    if (__any(tmax > st.r1v)) records_scan(st, P0, vbase);
    const float mnew = vmax2(st.m, tmax);
    const float ml = mnew * LOG2E;
    float s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
    expsum16(s, P0, ml);
    st.s = s;
    st.m = mnew;
}

// The logit GEMM of one step over 64-row stages [s0, s1) of the vocabulary, double-buffered in LDS
// from `lds` (stage s0 in buffer 0); the greedy state of this lane's rows accumulates in st.
// G = 4: each wave runs both 32-row tiles of a stage (two MFMA chains); G = 2: tile hf only.
// Stages alternate between two accumulator sets, so no stage copies its result for the next one's
// epilogue; the two waves of a SIMD (w, w + 4: opposite signs) run MFMA and epilogue in opposite
// orders. On return the last stage_store went to buffer (s1 - s0) & 1 (a redundant copy).
struct NoTail {
    __device__ __forceinline__ void operator()() const {}
};

// s64 carries staging registers in and out: with `preloaded` it already holds stage s0's loads (issued by
// the caller, e.g. during the previous cell's last stage); tail() runs at the last stage's mid-point in place
// of a store/load (the caller loads its next tile into s64 there)
// where logit rows 64s .. 64s+63 of the member (noise slice at nidx) come from
__device__ __forceinline__ StageSrc logit_src(const DecodeParams& p, uint64_t nidx, int s) {
    StageSrc Sx;
    Sx.w_r = make_rsrc(p.theta + p.off_log_w, 4u * 128u * (uint32_t)p.V1);
    Sx.z_r = make_rsrc(p.noise + nidx + p.off_log_w, 4u * 128u * (uint32_t)p.V1);
    Sx.b_r = make_rsrc(p.theta + p.off_log_b, 4u * (uint32_t)p.V1);
    Sx.bz_r = make_rsrc(p.noise + nidx + p.off_log_b, 4u * (uint32_t)p.V1);
    Sx.so_a = 32768u * (uint32_t)s; Sx.so_b = Sx.so_a + 16384u;
    Sx.bso = 256u * (uint32_t)s; Sx.bda = 0u; Sx.bdb = 128u;
    Sx.valid = p.V1 - 64 * s;
    return Sx;
}

// ---- sampled pick (FCModel._sample with greedy=False, nets.py:210-231) ------------------------------
// RandomState.choice takes the first id whose cumulative probability exceeds the draw u. Here the terms are
// p = exp2(fma(x, log2e, -r)) of logit x relative to an integer reference r >= max x * log2e (each lane's own,
// raised as its running max grows), scaled to a common reference R by exact powers of two: 2^(r - R) p. In
// proportion they are e^x (the normalisation cancels in u * sum(p)); against the oracle's exp((x - m) - lse)
// each differs by the argument's rounding (~3e-7 relative, as the oracle's own) and a tilt x 1.9e-8 from
// log2e's fp32 rounding. Four ids are summed in fp32 (a group), groups and stages in fp64.
//
// The logit loop writes every stage's logits to the workgroup's HBM slot (SampleStage) together with each
// lane's stage partial sum P (its 8 groups) and its r; its running total T (fp64, exact rescales) gives
// the row's sum(p) when the loop ends. The pick then scans the 149 stage sums (16 bytes per lane and stage)
// for the stage where the cumulative crosses u * T, and walks that stage's 64 logits id by id.
//
// Slot layout per stage: [wave][word 0..8][lane] x 16 bytes; words 0-3 / 4-7 the lane's logits of chain a /
// b (16 each), word 8 = {P (fp64), r, 0}.
#define SLOG_WAVE_BYTES 9216u                  // 9 words x 64 lanes x 16 bytes
#define SLOG_STAGE_BYTES (8u * SLOG_WAVE_BYTES)  // one 64-row stage of a workgroup (72 KiB)
// after the nst stages: one record per block of SLOG_BLOCK stages, {B (fp64), r, 0} per lane (8 waves x 1 KiB):
// the lane's sum of the block's terms relative to 2^r, so the pick finds the crossing block in two rounds of
// loads and then the crossing stage in one
#define SLOG_BLOCK 8
#define SLOG_BLK_BYTES 8192u
#define SAMP_L1_ROUND 20         // block records per round of the pick's level 1 (V1 <= 10240: one round)
#define SLOT_SPIN_TICKS 50000000ull   // 0.5 s of s_memrealtime (100 MHz) to find a free logit slot
#define SLOG_STORE_POLICY 2      // cache policy of the slot stores: nt (streaming; -2 % sampled kernel time vs the default, measured)

__device__ __forceinline__ float samp_p(float x, float ref) {
    return __builtin_amdgcn_exp2f(__builtin_fmaf(x, LOG2E, -ref));
}

// A group's sum: its four terms added in id order in fp32; the walk inside a group compares the cumulative
// plus each prefix of the same sum, so the group that crosses the threshold holds the pick.
__device__ __forceinline__ float samp_group(const float (&q)[4]) {
    return ((q[0] + q[1]) + q[2]) + q[3];
}

// 2^e x for fp64 x, exact (e clamped: a term 2^-2000 below the reference is 0 anyway)
__device__ __forceinline__ double samp_scale(double x, float e) {
    return x == 0.0 ? 0.0 : __builtin_ldexp(x, (int)fmaxf(e, -2000.f));
}

// logit_stages hook run after each stage (G = 4) with the stage's two tiles and its index; `replaces`: in
// place of the greedy epilogue
struct NoHook {
    static constexpr bool replaces = false;
    __device__ __forceinline__ void operator()(const f32x16&, const f32x16&, int) const {}
};

// the sampled decode's logit loop epilogue: running max m, reference r = ceil(m log2e), the lane's running sum T
// of its terms relative to 2^r; stores the stage's logits and {P, r} to the slot (one wave instruction per
// 1 KiB word; non-temporal). Measured and not kept (git history, r04): the late sign's stores after its MFMAs
// (+2.5 %), the early sign's logit stores before them (+0.7 %), sc1 / sc0 sc1 / sc1 nt logit stores (+1-2 %).
struct SampleStage {
    static constexpr bool replaces = true;
    rsrc_t slot;
    uint32_t vo;      // 16 * lane + SLOG_WAVE_BYTES * wave
    uint32_t vb;      // 16 * lane + 1024 * wave (block records)
    int nst;          // stages per step
    float& m;
    float& ref;
    double& T;
    double& Bk;       // the current block's sum of terms relative to 2^ref
    __device__ __forceinline__ void operator()(const f32x16& q0, const f32x16& q1, int s) const {
        if (s < 0) return;                               // the pipeline's first epilogue: no stage yet
        const uint32_t so = SLOG_STAGE_BYTES * (uint32_t)s;
#if !(DECODE_ABLATE & 256)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x4 a = {q0[4 * k], q0[4 * k + 1], q0[4 * k + 2], q0[4 * k + 3]};
            const f32x4 b = {q1[4 * k], q1[4 * k + 1], q1[4 * k + 2], q1[4 * k + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), slot, (int)vo, (int)(so + 1024u * k), SLOG_STORE_POLICY);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, b), slot, (int)vo, (int)(so + 1024u * (4 + k)), SLOG_STORE_POLICY);
        }
#endif
        const float mnew = vmax2(m, vmax2(vmax16(q0), vmax16(q1)));
        const float rnew = ceilf(mnew * LOG2E);
        if (rnew > ref) {
            T = samp_scale(T, ref - rnew);
            Bk = samp_scale(Bk, ref - rnew);
            ref = rnew;
        }
        m = mnew;
        double P = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float qa[4], qb[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                qa[e] = samp_p(q0[4 * k + e], ref);
                qb[e] = samp_p(q1[4 * k + e], ref);
            }
            P += (double)samp_group(qa);
            P += (double)samp_group(qb);
        }
        T += P;
        Bk += P;
        {
            const uint64_t pb = __builtin_bit_cast(uint64_t, P);
            const u32x4 w = {(uint32_t)pb, (uint32_t)(pb >> 32), __builtin_bit_cast(uint32_t, ref), 0u};
            __builtin_amdgcn_raw_buffer_store_b128(w, slot, (int)vo, (int)(so + 8u * 1024u), SLOG_STORE_POLICY);
#if NICNES_STORE_WAITS
            asm volatile("s_nop 1" ::"v"(w));                // (the wait states of the block record below)
#endif
            if ((s % SLOG_BLOCK) == SLOG_BLOCK - 1 || s == nst - 1) {      // the block's record (wave-uniform branch)
                const uint64_t bb = __builtin_bit_cast(uint64_t, Bk);
                const u32x4 wb = {(uint32_t)bb, (uint32_t)(bb >> 32), __builtin_bit_cast(uint32_t, ref), 0u};
                __builtin_amdgcn_raw_buffer_store_b128(wb, slot, (int)vb,
                                                       (int)(SLOG_STAGE_BYTES * (uint32_t)nst + SLOG_BLK_BYTES * (uint32_t)(s / SLOG_BLOCK)),
                                                       SLOG_STORE_POLICY);
                // the 16-byte store reads its data registers after issue: the compiler put the zeroing of Bk
                // right behind it with no wait state and lanes 12-15 of each 16 stored 0 (gfx950, measured); the
                // asm keeps Bk's registers unwritten for two wait states
#if NICNES_STORE_WAITS
                asm volatile("s_nop 1" : "+v"(Bk));
#endif
                Bk = 0.0;
            }
        }
    }
};

// The walk over one stage's logits (x0 / x1: the lane's chains a / b; ids 64s + 32c + 8k + 4hh + e) from the
// cumulative cb, the lane's terms scaled by sc = 2^(r - R): the first group in id order (the two lanes of a row
// alternate) whose cumulative exceeds thr, then its first id. mine / mlp: the pick and its log-prob
// (logprobs.gather, nets.py:225) on the lane holding it; found stays false if the stage's sums stop short.
__device__ __forceinline__ void sample_stage_walk(const f32x16& x0, const f32x16& x1, int s, int hh, float ref,
                                                  double sc, float m, float lse, double thr, double& cb, bool& found,
                                                  int& mine, float& mlp) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float x[4], q[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                x[e] = c ? x1[4 * k + e] : x0[4 * k + e];
                q[e] = samp_p(x[e], ref);
            }
            const float c1 = q[0] + q[1], c2 = c1 + q[2], g = c2 + q[3];
            const double gs = (double)g * sc;
            const double go = __shfl_xor(gs, 32);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const bool own = half == hh;
                const double gv = own ? gs : go;
                if (!found && cb + gv > thr) {
                    found = true;
                    if (own) {
                        const int e = cb + (double)q[0] * sc > thr ? 0 : cb + (double)c1 * sc > thr ? 1
                                    : cb + (double)c2 * sc > thr ? 2 : 3;
                        mine = 64 * s + 32 * c + 8 * k + 4 * hh + e;
                        mlp = (x[e] - m) - lse;
                    }
                }
                if (!found) cb += gv;
            }
        }
    }
}

__device__ __forceinline__ void samp_load_stage(rsrc_t lr, uint32_t vo, uint32_t so, f32x16& x0, f32x16& x1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(lr, (int)(vo + so), (int)(1024u * k), 16));
        const f32x4 b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(lr, (int)(vo + so), (int)(1024u * (4 + k)), 16));
#pragma unroll
        for (int e = 0; e < 4; ++e) { x0[4 * k + e] = a[e]; x1[4 * k + e] = b[e]; }
    }
}

// The pick of each row from its stored step (lr: the workgroup's slot, vo: the lane's offset in it), R: the row's
// common reference, thr = u * T. FULL (test hook NICNES_FORCE_EXACT): the walk runs through every stage's
// logits instead of scanning the stage sums first (the same terms; the sums associate differently, ~1e-16).
// If the crossing stage's own sums stop short of thr (rounding) or no stage crosses, the pick is the last id of
// that stage / V1 - 1 (stats[1] counts those rows).
template <bool FULL>
__device__ __forceinline__ void sample_pick(const DecodeParams& p, rsrc_t lr, uint32_t vo, int hh, float m, float lse,
                                            float R, double thr, int& tok, float& lpv, int pm = 0) {
    (void)pm;                                            // DECODE_PROF: the step's mark base
    const int nst = (p.V1 + 63) >> 6;
    double cum = 0.0, cb = 0.0;
    bool found = false;
    int mine = 0x7fffffff;
    float mlp = 0.f;
    int sf = nst - 1;                                    // the stage whose sums cross thr (default: the last)
    float rf = 0.f;
    if constexpr (FULL) {
        for (int s = 0; s < nst; ++s) {
            const f32x4 w = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(lr, (int)vo, (int)(SLOG_STAGE_BYTES * s + 8u * 1024u), 16));
            f32x16 x0, x1;
            samp_load_stage(lr, vo, SLOG_STAGE_BYTES * (uint32_t)s, x0, x1);
            const double c0 = cum;
            sample_stage_walk(x0, x1, s, hh, w[2], __builtin_ldexp(1.0, (int)fmaxf(w[2] - R, -2000.f)), m, lse, thr, cum,
                              found, mine, mlp);
            if (!found) { sf = s; cb = c0; rf = w[2]; }  // (kept for the no-crossing case: the last stage)
        }
        if (found) sf = -1;
    } else {
        // level 1: the block records (both lanes of a row sum the same values in the same order)
        const int nblk = (nst + SLOG_BLOCK - 1) / SLOG_BLOCK;
        const uint32_t vb = 16u * (uint32_t)(threadIdx.x & 63) + 1024u * (uint32_t)(threadIdx.x >> 6);
        int qf = -1;
        double cq = 0.0, cl = 0.0;
        for (int q0 = 0; q0 < nblk; q0 += SAMP_L1_ROUND) {
            // B and r as their own loads (a 16-byte load narrowed by the compiler returned B's low word as r)
            double Bw[SAMP_L1_ROUND];
            float rw[SAMP_L1_ROUND];
#pragma unroll
            for (int j = 0; j < SAMP_L1_ROUND; ++j) {
                const int so = (int)(SLOG_STAGE_BYTES * (uint32_t)nst + SLOG_BLK_BYTES * (uint32_t)min(q0 + j, nblk - 1));
                Bw[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(lr, (int)vb, so, 16));
                rw[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lr, (int)vb + 8, so, 16));
            }
#pragma unroll
            for (int j = 0; j < SAMP_L1_ROUND; ++j) {
                if (q0 + j < nblk) {
                    const double a = samp_scale(Bw[j], rw[j] - R);
                    const double ao = __shfl_xor(a, 32);
                    const double S = hh == 0 ? a + ao : ao + a;
                    if (qf < 0) {
                        if (cum + S > thr) { qf = q0 + j; cq = cum; }
                        else { cl = cum; cum += S; }
                    }
                }
            }
            if (__all(qf >= 0 ? 1 : 0)) break;
        }
        if (qf < 0) { qf = nblk - 1; cq = cl; }                 // thr at the very end (rounding): the last block
        PROF_MARK(pm + 22);
        // level 2: the stage records of block qf (a per-lane block: the stage offset goes in the vector offset)
        const int sa = SLOG_BLOCK * qf, sn = min(SLOG_BLOCK, nst - sa);
        double Pw[SLOG_BLOCK];
        float rw[SLOG_BLOCK];
#pragma unroll
        for (int j = 0; j < SLOG_BLOCK; ++j) {
            const uint32_t o = vo + SLOG_STAGE_BYTES * (uint32_t)(sa + min(j, sn - 1)) + 8u * 1024u;
            Pw[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(lr, (int)o, 0, 16));
            rw[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lr, (int)o + 8, 0, 16));
        }
        bool have = false;
        double cs = cq, csl = cq;
        float rl = rw[0];
#pragma unroll
        for (int j = 0; j < SLOG_BLOCK; ++j) {
            const double a = samp_scale(Pw[j], rw[j] - R);
            const double ao = __shfl_xor(a, 32);
            const double S = hh == 0 ? a + ao : ao + a;
            if (!have && j < sn) {
                if (cs + S > thr) { have = true; sf = sa + j; cb = cs; rf = rw[j]; }
                else { csl = cs; rl = rw[j]; cs += S; }
            }
        }
        if (!have) { sf = sa + sn - 1; cb = csl; rf = rl; }     // the block's stage sums stop short: its last stage
        PROF_MARK(pm + 23);
        f32x16 x0, x1;
        samp_load_stage(lr, vo, SLOG_STAGE_BYTES * (uint32_t)sf, x0, x1);
        sample_stage_walk(x0, x1, sf, hh, rf, __builtin_ldexp(1.0, (int)fmaxf(rf - R, -2000.f)), m, lse, thr, cb, found,
                          mine, mlp);
        if (found) sf = -1;
        else {                                           // the stage's sums stop short: its last id
            const int id = min(64 * sf + 63, p.V1 - 1), j = id - 64 * sf, jj = j & 31;
            if (((jj >> 2) & 1) == hh) {
                float xv = 0.f;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (4 * (jj >> 3) + (jj & 3) == i) xv = (j >> 5) ? x1[i] : x0[i];
                }
                mine = id;
                mlp = (xv - m) - lse;
            }
        }
    }
    if constexpr (FULL) {
        if (sf >= 0) {                                   // no stage crossed: V1 - 1, from the last stage
            f32x16 x0, x1;
            samp_load_stage(lr, vo, SLOG_STAGE_BYTES * (uint32_t)(nst - 1), x0, x1);
            const int id = p.V1 - 1, j = id - 64 * (nst - 1), jj = j & 31;
            if (((jj >> 2) & 1) == hh) {
                float xv = 0.f;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (4 * (jj >> 3) + (jj & 3) == i) xv = (j >> 5) ? x1[i] : x0[i];
                }
                mine = id;
                mlp = (xv - m) - lse;
            }
        }
    }
    if (sf >= 0 && hh == 0) atomicAdd(p.stats + 1, 1);
    const int other = __shfl_xor(mine, 32);
    const float olp = __shfl_xor(mlp, 32);
    if (mine != 0x7fffffff) { tok = mine; lpv = mlp; }
    else { tok = other; lpv = olp; }
}

// Measured and not kept (git history, r04): per-wave LDS progress words in place of the per-stage barrier (+0.4 %),
// a chain-a-only last stage for the coop ranges (+1.3 % / +2.2 % at P = 64 / 128, or spills inside the loop).
template <int G, bool PAIRS, bool PEEL = true, class Tail = NoTail, class Hook = NoHook>
__device__ __forceinline__ void logit_stages(float* lds, const DecodeParams& p, uint64_t nidx, int wave, int sgn,
                                             int hf, const float (&hB)[64], int s0, int s1, RowState& st,
                                             Stage64Regs& s64, bool preloaded = false, Tail&& tail = Tail(),
                                             const Hook& hook = Hook()) {
    const rsrc_t lw_r = make_rsrc(p.theta + p.off_log_w, 4u * 128u * (uint32_t)p.V1);
    const rsrc_t lz_r = make_rsrc(p.noise + nidx + p.off_log_w, 4u * 128u * (uint32_t)p.V1);
    const rsrc_t lbw_r = make_rsrc(p.theta + p.off_log_b, 4u * (uint32_t)p.V1);
    const rsrc_t lbz_r = make_rsrc(p.noise + nidx + p.off_log_b, 4u * (uint32_t)p.V1);
    auto lsrc = [&](int s) {                                 // logit rows 64s .. 64s+63
        StageSrc Sx;
        Sx.w_r = lw_r; Sx.z_r = lz_r; Sx.b_r = lbw_r; Sx.bz_r = lbz_r;
        Sx.so_a = 32768u * (uint32_t)s; Sx.so_b = Sx.so_a + 16384u;
        Sx.bso = 256u * (uint32_t)s; Sx.bda = 0u; Sx.bdb = 128u;
        Sx.valid = p.V1 - 64 * s;
        return Sx;
    };
    const LaneOffs lo = lane_offs(wave, 128u);
    const int hh = lane_fresh() >> 5, vl = 4 * hh + (G == 4 ? 0 : 32 * hf);
    const bool bias = wave < 2;
    if (!preloaded) stage64_load_o(lsrc(s0), lo, bias, s64);
    stage64_store_o(lds, lsrc(s0).valid, lo, bias, s64);
    // the registers carry stage s + 1 into stage s: its W+- tile is written before the last quarter of the
    // MFMAs of stage s (its buffer was last read in stage s - 1), then the loads of stage s + 2 are issued,
    // so the end of a stage has no staging wait and no LDS-write tail in front of the barrier
    if (PEEL) stage64_load_o(lsrc(min(s0 + 1, s1 - 1)), lo, bias, s64);   // (unconditional: one definition of s64)
    else if (s0 + 1 < s1) stage64_load_o(lsrc(s0 + 1), lo, bias, s64);
    __syncthreads();
    f32x16 a0, a1, b0, b1;
#pragma unroll
    for (int r = 0; r < 16; ++r) { b0[r] = NEG_INF; b1[r] = NEG_INF; }
    // MODE (PEEL): 0 a stage with two more after it (store s + 1, load s + 2), 1 the last but one (store
    // s + 1), 2 the last (the tail's loads); -1: decided at run time (the loop without the peel)
    auto stage = [&](auto mode_t, int s, f32x16& o0, f32x16& o1, const f32x16& q0, const f32x16& q1) {
        constexpr int MODE = decltype(mode_t)::value;
        const int sn = min(s + 1, s1 - 1);
        const float* buf = lds + ((s - s0) & 1) * STAGE64_FLOATS;
        const float* wsg = buf + sgn * (64 * LDS_ROW);
        const float* bsg = buf + 2 * 64 * LDS_ROW + 64 * sgn;
        auto mid = [&]() __attribute__((always_inline)) {
#if !(DECODE_ABLATE & 2)
            // s64 is loaded on every non-last path (at s1 - 2 the load repeats tile s1 - 1): a conditional load
            // here would make the compiler copy the 32 staging registers at every stage to merge the paths
            if constexpr (MODE == 0) {
                stage64_store_o(lds + ((s - s0 + 1) & 1) * STAGE64_FLOATS, lsrc(sn).valid, lo, bias, s64);
                stage64_load_o(lsrc(min(s + 2, s1 - 1)), lo, bias, s64);
            } else if constexpr (MODE == 1) {
                stage64_store_o(lds + ((s - s0 + 1) & 1) * STAGE64_FLOATS, lsrc(sn).valid, lo, bias, s64);
            } else if constexpr (MODE == 2) {
                tail();
            } else if (s + 1 < s1) {
                stage64_store_o(lds + ((s - s0 + 1) & 1) * STAGE64_FLOATS, lsrc(sn).valid, lo, bias, s64);
                stage64_load_o(lsrc(min(s + 2, s1 - 1)), lo, bias, s64);
            } else {
                tail();
            }
#endif
        };
        constexpr int MID = LOGIT_MID_AT;
        if constexpr (G == 4) {
            if (sgn == 0) {
                mfma_stage64_o<MID>(wsg, bsg, hB, lo.arow, hh, o0, o1, mid);
#if !(DECODE_ABLATE & 1)
                if constexpr (Hook::replaces) hook(q0, q1, s - 1);
                else epilogue64<PAIRS>(st, q0, q1, 64 * (s - 1) + vl);
#endif
            } else {
#if !(DECODE_ABLATE & 1)
                if constexpr (Hook::replaces) hook(q0, q1, s - 1);
                else epilogue64<PAIRS>(st, q0, q1, 64 * (s - 1) + vl);
#endif
                mfma_stage64_o<MID>(wsg, bsg, hB, lo.arow, hh, o0, o1, mid);
            }
        } else {
            const float* w1 = wsg + 32 * hf * LDS_ROW;         // this wave's 32-row tile of the stage
            const float* bb = bsg + 32 * hf;
            if (sgn == 0) {
                o0 = mfma_tile_o<MID>(bias_init(bb, hh), w1, hB, lo.arow, mid);
                epilogue32<PAIRS>(st, q0, 64 * (s - 1) + vl);
            } else {
                epilogue32<PAIRS>(st, q0, 64 * (s - 1) + vl);
                o0 = mfma_tile_o<MID>(bias_init(bb, hh), w1, hB, lo.arow, mid);
            }
        }
#if !(DECODE_ABLATE & 8)
        __syncthreads();
#endif
    };
    auto last = [&](const f32x16& q0, const f32x16& q1, int s) {
        if constexpr (G == 4) {
            if constexpr (Hook::replaces) hook(q0, q1, s);
            else epilogue64<PAIRS>(st, q0, q1, 64 * s + vl);
        } else {
            epilogue32<PAIRS>(st, q0, 64 * s + vl);
        }
    };
    if constexpr (PEEL) {
    // the last two stages peeled off the loop: inside it every stage stores and loads unconditionally, so the
    // staging registers have one definition and no copy (with a wait for their loads) at a merge point
    using M0 = std::integral_constant<int, 0>;
    using M1 = std::integral_constant<int, 1>;
    using M2 = std::integral_constant<int, 2>;
    int s = s0;
    for (; s + 2 < s1; s += 2) {
        stage(M0{}, s, a0, a1, b0, b1);
        stage(M0{}, s + 1, b0, b1, a0, a1);
    }
    if (s + 1 == s1) {
        stage(M2{}, s, a0, a1, b0, b1);
        last(a0, a1, s);
    } else {
        stage(M1{}, s, a0, a1, b0, b1);
        stage(M2{}, s + 1, b0, b1, a0, a1);
        last(b0, b1, s + 1);
    }
    } else {
    using MR = std::integral_constant<int, -1>;
    for (int s = s0; s < s1; s += 2) {
        stage(MR{}, s, a0, a1, b0, b1);
        if (s + 1 == s1) {
            last(a0, a1, s);
            return;
        }
        stage(MR{}, s + 1, b0, b1, a0, a1);
    }
    last(b0, b1, s1 - 1);
    }
}

// gate tiles of the cell: tile m = 0..19 is gate chunk tile_q(m) (order g1, g2, i, f, o) of the
// 32-unit block U = m / 5; its 32 rows of the 640-row i2h / h2h matrices start at gate_row(m)
__device__ __forceinline__ int tile_q(int m) { const int j = m % 5; return j < 2 ? j + 3 : j - 2; }
__device__ __forceinline__ uint32_t gate_row(int m) { return (uint32_t)(tile_q(m) * 128 + 32 * (m / 5)); }

// ---- the kernels ------------------------------------------------------------------------------
// One evaluate = img, then step(t) for t = -1..T. State between launches is lane-private scratch
// plus a per-workgroup `alive` flag (nets.py:242-243 early exit).
#define C_SLOT(s) (4u * 64u * (uint32_t)(s))            // c
#define H_SLOT(s) (4u * 64u * (uint32_t)(64 + (s)))     // h'
#define X_SLOT(s) (4u * 64u * (uint32_t)(128 + (s)))    // x of t = 0 (img_embed)
#define U_SLOT (4u * 64u * 192u)                        // row unfinished (1.0 / 0.0)

struct Ctx {
    int tid, lane, wave, sgn, grp, hh, member, slab, b, bc, wg;
    bool row_valid;
    rsrc_t theta_r, noise_r, scr_r;
    rsrc_t slog_r;    // sampled steps kernel: the workgroup's logit slot (else unused)
};

// a row is decoded when it lies in the slab range and in the batch's B_img * rpi rows (sign_off > 0: sign 1 takes
// the second half of the rows, DecodeParams::sign_off)
__device__ __forceinline__ bool row_ok(const DecodeParams& p, int b, int sgn) {
    return b < p.B && b + sgn * p.sign_off < p.B_img * p.rpi;
}

// XCD_GROUP (the sampled decode, whose rollouts span several 128-row slabs): the member slabs are taken in groups of
// 8 members, slab-major inside a group, so the slabs of one member are dispatched next to each other and, with the
// dispatcher's round-robin over the 8 XCDs (linear block id mod 8), on the same XCD: the member's noise rows are then
// read from HBM by one slab and from that XCD's L2 by the others, instead of once per slab a whole grid apart.
template <bool XCD_GROUP = false>
__device__ __forceinline__ Ctx make_ctx(const DecodeParams& p) {
    Ctx c;
    c.tid = threadIdx.x;
    c.lane = c.tid & 63;
    c.wave = __builtin_amdgcn_readfirstlane(c.tid >> 6);
    c.sgn = c.wave >> 2;
    c.grp = c.wave & 3;
    c.hh = c.lane >> 5;
    c.member = blockIdx.x;
    c.slab = blockIdx.y;
    if constexpr (XCD_GROUP) {
        const int M = (int)gridDim.x, NS = (int)gridDim.y;
        const int L = (int)(blockIdx.x + gridDim.x * blockIdx.y), gs = 8 * NS, g = L / gs;
        const int w = min(8, M - 8 * g), r = L - g * gs;       // members in this group (the last may hold fewer)
        c.member = 8 * g + r % w;
        c.slab = r / w;
    }
    c.wg = c.member * gridDim.y + c.slab;
    c.b = c.slab * 128 + c.grp * 32 + (c.lane & 31);
    c.row_valid = row_ok(p, c.b, c.sgn);
    c.bc = c.row_valid ? c.b : 0;
    const uint64_t nidx = p.noise_idx[c.member];
    const uint32_t Dbytes = 4u * (uint32_t)p.D;
    c.theta_r = make_rsrc(p.theta, Dbytes);
    c.noise_r = make_rsrc(p.noise + nidx, Dbytes);
    float* wscr = p.scratch + ((size_t)c.wg * 8 + c.wave) * (SCR_SLOTS * 64);
    c.scr_r = make_rsrc(wscr, SCR_SLOTS * 64 * 4);
    return c;
}

// ---- workgroup roles of the img kernel and the split path -----------------------------------
// grid (q, member, slab). G = 4: wave w = sign (w >> 2) x 32-row group (w & 3) of a 128-row slab.
// G = 2 (64-row slabs, B <= 64): wave w = sign (w >> 2) x group ((w >> 1) & 1) x tile half (w & 1);
// the two halves of a (sign, group) pair share rows and run one 32-row MFMA tile each.
// w and w + 4 (opposite signs, same rows / tile half) share a SIMD in both layouts.
template <int G>
struct SCtx {
    int tid, lane, wave, sgn, grp, hf, hh, member, slab, q, wg, b, bc;
    bool row_valid;
    rsrc_t theta_r, noise_r, scr_r;
};

template <int G>
__device__ __forceinline__ SCtx<G> make_sctx(const DecodeParams& p) {
    SCtx<G> c;
    c.tid = threadIdx.x;
    c.lane = c.tid & 63;
    c.wave = __builtin_amdgcn_readfirstlane(c.tid >> 6);
    c.sgn = c.wave >> 2;
    c.grp = G == 4 ? (c.wave & 3) : ((c.wave >> 1) & 1);
    c.hf = G == 4 ? 0 : (c.wave & 1);
    c.hh = c.lane >> 5;
    c.q = blockIdx.x;
    c.member = blockIdx.y;
    c.slab = blockIdx.z;
    c.wg = c.member * gridDim.z + c.slab;
    c.b = c.slab * (32 * G) + c.grp * 32 + (c.lane & 31);
    c.row_valid = row_ok(p, c.b, c.sgn);
    c.bc = c.row_valid ? c.b : 0;
    const uint64_t nidx = p.noise_idx[c.member];
    const uint32_t Dbytes = 4u * (uint32_t)p.D;
    c.theta_r = make_rsrc(p.theta, Dbytes);
    c.noise_r = make_rsrc(p.noise + nidx, Dbytes);
    // lane scratch per (slab, sign, row group); G = 4 gives the fused kernel's (wg * 8 + wave)
    float* wscr = p.scratch + ((size_t)c.wg * (2 * G) + c.sgn * G + c.grp) * (SCR_SLOTS * 64);
    c.scr_r = make_rsrc(wscr, SCR_SLOTS * 64 * 4);
    return c;
}

// ========== t = 0 input: x = img_embed(fc) (nets.py:194-195) ====================================
// grid (Sc, members, slabs): workgroup q computes the 32-unit blocks [q * 4/Sc, (q+1) * 4/Sc) of x
// (Sc = 1: all four, the fused path). With G = 2 the tile-half-1 waves only help stage.
template <int G>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_img_kernel(DecodeParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SCtx<G> c = make_sctx<G>(p);
    const bool fused_path = G == 4 && p.S == 1;
    if (fused_path) PROF_MARK(80); else PROF_SPLIT(250);
    const float* fcm = p.fc + (p.member_batch ? (size_t)p.member_batch[c.member] * p.B_img * p.F : 0);
    const rsrc_t fc_r = make_rsrc(fcm, 4u * (uint32_t)p.B_img * (uint32_t)p.F);
    const int fr = c.row_valid ? (c.b + c.sgn * p.sign_off) / p.rpi : 0;      // the lane's fc row (its image)
    const uint32_t lo = 4u * c.lane;
    const bool mm = G == 4 || c.hf == 0;
    StageRegs sr;
    f32x16 accU[4];
    const int nK = p.F >> 7;
    const int nb = 4 / (int)gridDim.x, U0 = nb * c.q;
    const int ntile = nK * nb;
    auto desc = [&](int n) {
        TileDesc d;
        d.w_off = (uint32_t)p.off_img_w; d.ld = p.F; d.row0 = 32 * (U0 + n % nb); d.nvalid = 32; d.k0 = 128 * (n / nb);
        d.b_off = (uint32_t)p.off_img_b; d.pad_bias = 0.f;
        return d;
    };
    stage_load(c.theta_r, c.noise_r, desc(0), c.tid, sr);
    stage_store(lds, desc(0), c.tid, sr);
    __syncthreads();
    for (int kc = 0; kc < nK; ++kc) {
        const uint32_t frow = 4u * (uint32_t)(fr * p.F + 128 * kc + 4 * c.hh);
#pragma unroll
        for (int U = 0; U < 4; ++U) {
            if (U < nb) {
                const int n = kc * nb + U;
                if (n + 1 < ntile) stage_load(c.theta_r, c.noise_r, desc(n + 1), c.tid, sr);
                const float* buf = lds + (n & 1) * STAGE_FLOATS;
                if (mm) {
                    if (kc == 0) accU[U] = bias_init(buf + 2 * SIGN_FLOATS + 32 * c.sgn, c.hh);
                    accU[U] = mfma_tile_fc(accU[U], buf + c.sgn * SIGN_FLOATS, fc_r, frow, c.lane);
                }
                if (n + 1 < ntile) stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), c.tid, sr);
                __syncthreads();
            }
        }
    }
    if (mm) {
#pragma unroll
        for (int U = 0; U < 4; ++U)
            if (U < nb) {
#pragma unroll
                for (int r = 0; r < 16; ++r) st1(c.scr_r, lo, X_SLOT(16 * (U0 + U) + r), accU[U][r]);
            }
        st1(c.scr_r, lo, U_SLOT, 1.0f);
    }
    if (c.q == 0 && c.tid == 0) p.alive[c.wg] = 1;
    if (fused_path) PROF_MARK(81); else PROF_SPLIT(251);
}

// The same for a mutated member on the fused path (MutHead): delta' of img_embed formed at the stage store. The
// 32-row kernel: its staging registers leave room for the vector's; the x it writes is nicnes_decode_img_kernel<4>'s.
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_img_mut_kernel(DecodeParams p, MutHead mh) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SCtx<4> c = make_sctx<4>(p);
    const MutRes mr = mut_res(p, mh, c.member);
    PROF_MARK(80);
    const float* fcm = p.fc + (p.member_batch ? (size_t)p.member_batch[c.member] * p.B_img * p.F : 0);
    const rsrc_t fc_r = make_rsrc(fcm, 4u * (uint32_t)p.B_img * (uint32_t)p.F);
    const int fr = c.row_valid ? (c.b + c.sgn * p.sign_off) / p.rpi : 0;      // the lane's fc row (its image)
    const uint32_t lo = 4u * c.lane;
    StageRegsM sr;
    f32x16 accU[4];
    const int nK = p.F >> 7;
    const int ntile = nK * 4;
    auto desc = [&](int n) {
        TileDesc d;
        d.w_off = (uint32_t)p.off_img_w; d.ld = p.F; d.row0 = 32 * (n % 4); d.nvalid = 32; d.k0 = 128 * (n / 4);
        d.b_off = (uint32_t)p.off_img_b; d.pad_bias = 0.f;
        return d;
    };
    stage_load_m(c.theta_r, mr, desc(0), c.tid, sr);
    stage_store_m(lds, desc(0), c.tid, sr, mr.mode);
    __syncthreads();
    for (int kc = 0; kc < nK; ++kc) {
        const uint32_t frow = 4u * (uint32_t)(fr * p.F + 128 * kc + 4 * c.hh);
#pragma unroll
        for (int U = 0; U < 4; ++U) {
            const int n = kc * 4 + U;
            if (n + 1 < ntile) stage_load_m(c.theta_r, mr, desc(n + 1), c.tid, sr);
            const float* buf = lds + (n & 1) * STAGE_FLOATS;
            if (kc == 0) accU[U] = bias_init(buf + 2 * SIGN_FLOATS + 32 * c.sgn, c.hh);
            accU[U] = mfma_tile_fc(accU[U], buf + c.sgn * SIGN_FLOATS, fc_r, frow, c.lane);
            if (n + 1 < ntile) stage_store_m(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), c.tid, sr, mr.mode);
            __syncthreads();
        }
    }
#pragma unroll
    for (int U = 0; U < 4; ++U)
#pragma unroll
        for (int r = 0; r < 16; ++r) st1(c.scr_r, lo, X_SLOT(16 * U + r), accU[U][r]);
    st1(c.scr_r, lo, U_SLOT, 1.0f);
    if (c.tid == 0) p.alive[c.wg] = 1;
    PROF_MARK(81);
}

// ========== t = 0 input on the fused path: 64-row stages, fc chunk as a register B operand ==========
// x = img_embed(fc) of both signs for the workgroup's 128 rows (nets.py:194-195): 2 nK stages of 64 img_w rows
// (unit blocks 0-1 for even stages, 2-3 for odd) x 128 k (chunk j >> 1), staged and double-buffered as the logit
// stages; the fc chunk of the lane's row (64 values) is the B operand of both stages of a chunk, the next chunk's
// loaded during the current one. Every unit-block chain starts from the bias and takes k in the same order as
// nicnes_decode_img_kernel: identical x, written to X_SLOT.
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_img64_kernel(DecodeParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const Ctx c = make_ctx(p);
    PROF_MARK(80);
    const float* fcm = p.fc + (p.member_batch ? (size_t)p.member_batch[c.member] * p.B_img * p.F : 0);
    const rsrc_t fc_r = make_rsrc(fcm, 4u * (uint32_t)p.B_img * (uint32_t)p.F);
    const int fr = c.row_valid ? (c.b + c.sgn * p.sign_off) / p.rpi : 0;      // the lane's fc row (its image)
    const int nK = p.F >> 7;
    const uint32_t F = (uint32_t)p.F;
    auto load = [&](int j, Stage64Regs& r) __attribute__((always_inline)) {
        const int tid = c.wave * 64 + lane_fresh();
        // thread tid: img_w row 64 (j & 1) + (tid >> 5) + 16 u, k 128 (j >> 1) + 4 (tid & 31) (stage64_store's rows)
        const uint32_t vo = 4u * ((uint32_t)(tid >> 5) * F + 4u * (uint32_t)(tid & 31));
        const uint32_t base = 4u * ((uint32_t)p.off_img_w + (uint32_t)(64 * (j & 1)) * F + 128u * (uint32_t)(j >> 1));
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            r.w[u] = ld4(c.theta_r, vo, base + 64u * F * (uint32_t)u);
            r.z[u] = ld4(c.noise_r, vo, base + 64u * F * (uint32_t)u);
        }
        const uint32_t bo = 4u * ((uint32_t)p.off_img_b + (uint32_t)(64 * (j & 1) + (tid & 63)));
        r.bw = ld1(c.theta_r, bo);
        r.bz = ld1(c.noise_r, bo);
    };
    auto load_fc = [&](int kc, float (&dst)[64]) __attribute__((always_inline)) {
        const uint32_t frow = 4u * ((uint32_t)fr * F + 128u * (uint32_t)kc + 4u * (uint32_t)c.hh);
#pragma unroll
        for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 v = ld4(fc_r, frow + 4u * (uint32_t)(32 * T + 8 * a));
#pragma unroll
                for (int e = 0; e < 4; ++e) dst[16 * T + 4 * a + e] = v[e];
            }
    };
    // two chains (unit blocks u0, u0 + 1) over one stage, accumulating (bias first at chunk 0)
    auto mm = [&](const float* buf, bool first, const float (&Bop)[64], f32x16& A0, f32x16& A1)
        __attribute__((always_inline)) {
        const int lane = lane_fresh(), hh = lane >> 5;
        const float* wsg = buf + c.sgn * (64 * LDS_ROW);
        const float* bsg = buf + 2 * 64 * LDS_ROW + 64 * c.sgn;
        if (first) {
            A0 = bias_init(bsg, hh);
            A1 = bias_init(bsg + 32, hh);
        }
        const float* row0 = wsg + (lane & 31) * LDS_ROW + 16 * hh;
        const float* row1 = row0 + 32 * LDS_ROW;
#pragma unroll
        for (int T = 0; T < 4; ++T) {
            f32x4 a0[4], a1[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a0[q] = *reinterpret_cast<const f32x4*>(row0 + T * 32 + 4 * q);
                a1[q] = *reinterpret_cast<const f32x4*>(row1 + T * 32 + 4 * q);
            }
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                A0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], Bop[16 * T + jj], A0, 0, 0, 0);
                A1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], Bop[16 * T + jj], A1, 0, 0, 0);
            }
        }
    };
    const int tid0 = c.wave * 64;
    Stage64Regs s64;
    f32x16 acc[4];
    float fcB[64], fcN[64];
    load(0, s64);
    load_fc(0, fcB);
    stage64_store(lds, 64, tid0 + lane_fresh(), s64);
    __syncthreads();
#pragma unroll 1
    for (int kc = 0; kc < nK; ++kc) {
        load(2 * kc + 1, s64);                                   // stage 2 kc + 1: unit blocks 2-3
        if (kc + 1 < nK) load_fc(kc + 1, fcN);
        mm(lds, kc == 0, fcB, acc[0], acc[1]);
        stage64_store(lds + STAGE64_FLOATS, 64, tid0 + lane_fresh(), s64);
        __syncthreads();
        if (kc + 1 < nK) load(2 * kc + 2, s64);                  // stage 2 kc + 2: unit blocks 0-1
        mm(lds + STAGE64_FLOATS, kc == 0, fcB, acc[2], acc[3]);
        if (kc + 1 < nK) stage64_store(lds, 64, tid0 + lane_fresh(), s64);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 64; ++i) fcB[i] = fcN[i];
    }
    const uint32_t lo = 4u * (uint32_t)lane_fresh();
#pragma unroll
    for (int U = 0; U < 4; ++U)
#pragma unroll
        for (int r = 0; r < 16; ++r) st1(c.scr_r, lo, X_SLOT(16 * U + r), acc[U][r]);
    st1(c.scr_r, lo, U_SLOT, 1.0f);
    if (c.tid == 0) p.alive[c.wg] = 1;
    PROF_MARK(81);
}

// ========== step kernel: logits + greedy token of step t, then the LSTM cell of step t+1 ========
// One launch per step t = -1 .. T. Logits (nets.py:202,208-209) run for t >= 1 over h = h_t (t = 0
// is the image step, whose output the reference discards). The cell of step t+1 (nets.py:98-134)
// follows in the same launch while h_t is still the live B operand: its gate sums
// s = (b_i2h + Wi.x) + (b_h2h + Wh.h) run as 20 stages, one per 32-unit gate tile, each staging
// the tile's i2h rows (chain a, B = x = embed(token), nets.py:196-199, or img_embed(fc) at t = -1)
// and its h2h rows (chain b, B = h). The tiles come in nn_lstm_cell's fold order per unit block
// (g1, g2, i, f, o), so c' and h' are folded in registers as the gates complete; only c' and h'
// go to lane scratch. In the logit loop the two waves sharing a SIMD (w and w+4: opposite signs)
// run the MFMA chains and the VALU epilogue of the previous stage in opposite orders, so VALU of
// one wave overlaps the MFMAs of the other.
// one step of one workgroup; false when the workgroup is done (every row finished, or t = T).
// s64 / pre (the steps kernel): staging registers kept across steps; pre says they hold this step's first
// logit tile, loaded during the previous step's last cell stage (PREFETCH: that load is issued)
// SAMPLE: the sampled decode (nets.py:210-231): the logit loop stores its logits and stage sums (SampleStage), then
// sample_pick draws each row's token with its uniform p.sample_u (fused path only)
template <bool PAIRS, bool PREFETCH, bool SAMPLE = false, bool MUT = false>
__device__ __forceinline__ bool step_body(const DecodeParams& p, const Ctx& c, float* lds, int t, Stage64Regs& s64,
                                          bool& pre, float (&hB)[64], bool& hpre, const MutRes* mr = nullptr) {
    PROF_MARK(2 * (t + 1));
    const uint32_t lo = 4u * c.lane;
    const int nst = (p.V1 + 63) >> 6;
    const int nl = t > 0 ? nst : 0;
    const uint64_t nidx = p.noise_idx[c.member];
    // the row's unfinished flag, read now: the token phase needs it right after the logit loop
    const float unf_prev = nl > 0 ? ld1(c.scr_r, lo, U_SLOT) : 0.f;
    // SAMPLE: the row's uniform for this step, loaded now (the pick's first dependent load otherwise)
    double u_pre = 0.5;
    if constexpr (SAMPLE) {
        if (nl > 0 && c.row_valid)
            u_pre = p.sample_u[(((size_t)c.member * 2 + c.sgn) * p.B + c.bc) * p.T + (t - 1)];
    }
    if (t < 0) {
#pragma unroll
        for (int i = 0; i < 64; ++i) hB[i] = 0.f;               // h = 0 before the first cell
    } else if (!hpre) {                                          // (hpre: loaded at the end of the last step)
#pragma unroll
        for (int i = 0; i < 64; ++i) hB[i] = ld1(c.scr_r, lo, H_SLOT(i));
    }
    hpre = false;
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(hB[i]);
    const uint32_t ib = (uint32_t)p.off_i2h_b, hb = (uint32_t)p.off_h2h_b, bmin = min(ib, hb);
    auto csrc = [&](int m) {                                     // gate tile m: i2h rows | h2h rows
        const uint32_t r = gate_row(m);
        StageSrc S;
        S.w_r = c.theta_r; S.z_r = c.noise_r; S.b_r = c.theta_r; S.bz_r = c.noise_r;
        S.so_a = 4u * ((uint32_t)p.off_i2h_w + 128u * r);
        S.so_b = 4u * ((uint32_t)p.off_h2h_w + 128u * r);
        S.bso = 4u * (bmin + r);
        S.bda = 4u * (ib - bmin); S.bdb = 4u * (hb - bmin);
        S.valid = 64;
        return S;
    };
    int it = 0;                                   // token fed to the next cell (0 = BOS at t = 0)
    bool cell_pre = false;                        // s64 holds the cell's first gate tile
    if (nl > 0) {
        RowState st;
        row_state_init(st);
        // the cell's first gate tile does not depend on the token: its loads are issued at the last logit
        // stage's mid-point (tail) and land while the token is picked
        const bool xpre = t < p.T;
        auto tail = [&]() __attribute__((always_inline)) {
            if (xpre) stage64_load(csrc(0), c.wave * 64 + lane_fresh(), s64);
        };
        // SAMPLE: the lane's running max, reference and sum of terms (SampleStage), the logits to the slot
        float sm = -1.0e30f, sref = -1.0e30f;
        double sT = 0.0, sB = 0.0;
        if constexpr (SAMPLE) {
            const SampleStage ss{c.slog_r, 16u * (uint32_t)lane_fresh() + SLOG_WAVE_BYTES * (uint32_t)c.wave,
                                 16u * (uint32_t)lane_fresh() + 1024u * (uint32_t)c.wave, (p.V1 + 63) >> 6, sm, sref, sT,
                                 sB};
            // (no peel for the sampled decode: +2.2 %, measured)
            logit_stages<4, PAIRS, false>(lds, p, nidx, c.wave, c.sgn, 0, hB, 0, nl, st, s64, pre, tail, ss);
        } else {
            logit_stages<4, PAIRS>(lds, p, nidx, c.wave, c.sgn, 0, hB, 0, nl, st, s64, pre, tail);
        }
        cell_pre = xpre;
        PROF_MARK(120 + 24 * (t + 1));

        // ---- greedy token (nets.py:208-209) ------------------------------------------------
        const float m_o = __shfl_xor(st.m, 32);
        const float s_o = __shfl_xor(st.s, 32);
        const float m = fmaxf(st.m, m_o);
        const float stot = st.s * __builtin_amdgcn_exp2f((st.m - m) * LOG2E) + s_o * __builtin_amdgcn_exp2f((m_o - m) * LOG2E);
        const TieWindow w = tie_window(stot, PAIRS, p.lse_margin);
        float lse = w.lse;
        int tok = 0x7fffffff;
        float lp_tok = 0.f;                      // seq_logprobs: -lse (the max, greedy) or the draw's log-prob
        bool amb = false;
        if constexpr (SAMPLE) {
            const double u = u_pre;
            // the row: max, common reference R, sum T of its terms relative to 2^R (lane 0's part first), lse
            const float mo = __shfl_xor(sm, 32), ro = __shfl_xor(sref, 32);
            const double To = __shfl_xor(sT, 32);
            const float mr = fmaxf(sm, mo), R = fmaxf(sref, ro);
            const double ta = samp_scale(sT, sref - R), tb = samp_scale(To, ro - R);
            const double T = c.hh == 0 ? ta + tb : tb + ta;
            const float lse_s = (float)(log(T) + (double)R * 0.69314718055994531 - (double)mr);
            const uint32_t vo = 16u * (uint32_t)c.lane + SLOG_WAVE_BYTES * (uint32_t)c.wave;
#if DECODE_ABLATE & 512
            tok = 1 + (int)(u * 9000.0);                 // timing only: no pick
            lp_tok = -lse_s;
#else
            if (p.force_exact)
                sample_pick<true>(p, c.slog_r, vo, c.hh, mr, lse_s, R, u * T, tok, lp_tok);
            else
                sample_pick<false>(p, c.slog_r, vo, c.hh, mr, lse_s, R, u * T, tok, lp_tok, 120 + 24 * (t + 1));
#endif
        } else {
            const float cv[4] = {st.r0v, st.r1v, __shfl_xor(st.r0v, 32), __shfl_xor(st.r1v, 32)};
            const int ci[4] = {st.r0i, st.r1i, __shfl_xor(st.r0i, 32), __shfl_xor(st.r1i, 32)};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int ws = win_state(cv[k], m, w);
                if (ws == 1 && ci[k] < tok) tok = ci[k];
                amb = amb || ws == 2;
            }
        const bool ovf = p.force_exact || amb || win_state(st.ev, m, w) != 0 ||
                         win_state(__shfl_xor(st.ev, 32), m, w) != 0;
        if (__syncthreads_or(ovf ? 1 : 0)) {
            // rare: more records than tracked fall in the tie window (or, PAIRS mode, the bounds on
            // lse leave a record undecided) -> exact pass. PAIRS: the exp-sum sweep first, then the
            // records decide as in the exact mode, and only an evicted record in the window needs the
            // sweep for the first id in the window
            int best = 0x7fffffff;
            float ssum = 0.f;
            bool find = true;
            if (PAIRS) {
                exact_sweep(lds, p, c.theta_r, c.noise_r, c.tid, c.sgn, c.hh, c.lane, hB, true, true, m, 0.f,
                            ssum, best);
                lse = logf(ssum + __shfl_xor(ssum, 32));
                const float cv[4] = {st.r0v, st.r1v, __shfl_xor(st.r0v, 32), __shfl_xor(st.r1v, 32)};
                const int ci[4] = {st.r0i, st.r1i, __shfl_xor(st.r0i, 32), __shfl_xor(st.r1i, 32)};
                int t2 = 0x7fffffff;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (in_window(cv[k], m, lse) && ci[k] < t2) t2 = ci[k];
                const bool ev2 = p.force_exact || in_window(st.ev, m, lse) || in_window(__shfl_xor(st.ev, 32), m, lse);
                find = __syncthreads_or(ev2 ? 1 : 0) != 0;
                if (!find) tok = t2;
            }
            if (find) {
                exact_sweep(lds, p, c.theta_r, c.noise_r, c.tid, c.sgn, c.hh, c.lane, hB, true, false, m, lse,
                            ssum, best);
                tok = min(best, __shfl_xor(best, 32));
            }
            if (c.tid == 0) atomicAdd(p.stats + 0, 1);
        }
        lp_tok = -lse;                           // seq_logprobs[:, t-1] = max lp = fp32((m - m) - lse) (nets.py:208,241)
        }
        // no candidate only when every logit is NaN (torch.max would return a NaN's index):
        // end the caption instead of emitting an out-of-vocabulary id
        if (tok >= p.V1) tok = 0;
        // finished mask (nets.py:236-243); forward_for_sensitivity feeds every argmax back (nets.py:62-63)
        const bool unfinished = unf_prev != 0.f && tok > 0;
        it = (unfinished || p.no_mask) ? tok : 0;
        st1(c.scr_r, lo, U_SLOT, unfinished ? 1.f : 0.f);
#if !DECODE_PROF
        if (c.hh == 0 && c.row_valid) {
            const size_t o = (((size_t)c.member * 2 + c.sgn) * p.B + c.b) * p.T + (t - 1);
            p.seq[o] = it;
            if (p.lp) p.lp[o] = lp_tok;
        }
#endif
        const int any = __syncthreads_or(((unfinished && c.row_valid) || p.no_exit || (DECODE_ABLATE & 64)) ? 1 : 0);
        if (c.tid == 0) p.alive[c.wg] = any;
        if (!any) { PROF_MARK(2 * (t + 1) + 1); return false; } // the reference stops here (nets.py:242-243)
    }
    if (t >= p.T) { PROF_MARK(2 * (t + 1) + 1); return false; }

    // ---- LSTM cell of step t+1 ---------------------------------------------------------------
    float xB[64];
    if (t < 0) {                                                 // x = img_embed(fc) (nets.py:194-195)
#pragma unroll
        for (int i = 0; i < 64; ++i) xB[i] = ld1(c.scr_r, lo, X_SLOT(i));
    } else {                                                     // x = embed(it) (nets.py:196-199)
        const uint32_t eo = 4u * ((uint32_t)p.off_emb_w + (uint32_t)it * 128u + 4u * c.hh);
#pragma unroll
        for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 w = ld4(c.theta_r, eo + 4u * (32 * T + 8 * a));
                f32x4 delta;                                // fp32(sigma * z): the table is sigma-scaled
                if constexpr (MUT)                          // a mutated member: the row's delta' formed here
                    delta = mut_delta(ld4(mr->head_r, eo + 4u * (32 * T + 8 * a)),
                                      ld4(mr->vec_r, eo + 4u * (32 * T + 8 * a)), mr->mode);
                else
                    delta = ld4(c.noise_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 x = c.sgn ? (w - delta) : (w + delta);
#pragma unroll
                for (int e = 0; e < 4; ++e) xB[16 * T + 4 * a + e] = x[e];
            }
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(xB[i]);
    const int b0 = nl & 1;                                       // next free stage buffer
    PROF_MARK(120 + 24 * (t + 1) + 1);
    if (!cell_pre) stage64_load(csrc(0), c.wave * 64 + lane_fresh(), s64);
    stage64_store(lds + b0 * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
    constexpr bool CMID = !SAMPLE;                               // (the sampled decode: +0.9 %, measured)
    if constexpr (CMID) stage64_load(csrc(1), c.wave * 64 + lane_fresh(), s64);   // tile 1: stored at tile 0's mid-point
    __syncthreads();
    f32x16 hold;
    // fold of gate tile m (s_ = its gate sums) into the unit block's c' / h'
    auto fold = [&](int m, const f32x16& s_, const f32x16& cpre) __attribute__((always_inline)) {
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
        const int U = m / 5, j5 = m % 5;
        if (j5 == 0) {                                           // g1
            hold = s_;
        } else if (j5 == 1) {                                    // g = max(g1, g2)
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = hold[r] > s_[r] ? hold[r] : s_[r];
        } else if (j5 == 2) {                                    // ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = CELL_SIG(s_[r]) * hold[r];
        } else if (j5 == 3) {                                    // c' = f * c + ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float fcv = CELL_SIG(s_[r]) * cpre[r];
                const float cn = fcv + hold[r];
                st1(c.scr_r, lo_, C_SLOT(16 * U + r), cn);
                hold[r] = cn;
            }
        } else {                                                 // h' = o * tanh(c')
#pragma unroll
            for (int r = 0; r < 16; ++r)
                st1(c.scr_r, lo_, H_SLOT(16 * U + r), CELL_SIG(s_[r]) * CELL_TANH(hold[r]));
        }
    };
    auto load_c = [&](int m) __attribute__((always_inline)) {                                   // c of the f tile's unit block
        f32x16 cp;
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
#pragma unroll
        for (int r = 0; r < 16; ++r) cp[r] = (m % 5 == 3 && t >= 0) ? ld1(c.scr_r, lo_, C_SLOT(16 * (m / 5) + r)) : 0.f;
        return cp;
    };
#pragma unroll 1
    for (int m = 0; m < 20; ++m) {
        const f32x16 cpre = load_c(m);                           // before the staging loads (in-order vmcnt)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!CMID) {
            if (m < 19) {
                stage64_load(csrc(m + 1), c.wave * 64 + lane_fresh(), s64);
            } else if (PREFETCH && t >= 0) {                     // the next step's first logit tile
                const LaneOffs lo_ = lane_offs(c.wave, 128u);
                stage64_load_o(logit_src(p, nidx, 0), lo_, c.wave < 2, s64);
            }
        }
        const float* buf = lds + ((m + b0) & 1) * STAGE64_FLOATS;
        const float* wsg = buf + c.sgn * (64 * LDS_ROW);
        const float* bsg = buf + 2 * 64 * LDS_ROW + 64 * c.sgn;
        f32x16 a0, a1;
        if constexpr (CMID) {
        // tile m + 1 goes to the other buffer before the last quarter of tile m's MFMAs (that buffer was last read
        // in tile m - 1, before the barrier); tile m + 2's loads follow the fold, so the staging registers are
        // free while it runs
        auto midst = [&]() __attribute__((always_inline)) {
            __builtin_amdgcn_sched_barrier(0);
            if (m < 19) stage64_store(lds + ((m + 1 + b0) & 1) * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
            __builtin_amdgcn_sched_barrier(0);
        };
        if (t < 0) {    // h = 0 before the first cell: h2h(h) is its bias (fma(w, 0, acc) == acc)
            mfma_xh_part<0, 3, false>(wsg, bsg, xB, hB, lane_fresh(), a0, a1);
            midst();
            mfma_xh_part<3, 4, false>(wsg, bsg, xB, hB, lane_fresh(), a0, a1);
        } else {
            mfma_xh_part<0, 3>(wsg, bsg, xB, hB, lane_fresh(), a0, a1);
            midst();
            mfma_xh_part<3, 4>(wsg, bsg, xB, hB, lane_fresh(), a0, a1);
        }
        fold(m, a0 + a1, cpre);                            // i2h(x) + h2h(h), nets.py:109-111
        if (m < 18) {
            stage64_load(csrc(m + 2), c.wave * 64 + lane_fresh(), s64);
        } else if (m == 18 && PREFETCH && t >= 0) {             // the next step's first logit tile
            const LaneOffs lo_ = lane_offs(c.wave, 128u);
            stage64_load_o(logit_src(p, nidx, 0), lo_, c.wave < 2, s64);
        }
        } else {
        if (t < 0)      // h = 0 before the first cell: h2h(h) is its bias (fma(w, 0, acc) == acc)
            mfma_xh_part<0, 4, false>(wsg, bsg, xB, hB, lane_fresh(), a0, a1);
        else
            mfma_xh_part<0, 4>(wsg, bsg, xB, hB, lane_fresh(), a0, a1);
        fold(m, a0 + a1, cpre);                            // i2h(x) + h2h(h), nets.py:109-111
        if (m < 19) stage64_store(lds + ((m + 1 + b0) & 1) * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
        }
        __syncthreads();
        PROF_MARK(120 + 24 * (t + 1) + 2 + m);
    }
    pre = PREFETCH && t >= 0;
    if (PREFETCH && t + 1 <= p.T) {                // h_{t+1}: this lane's own h' stores, read back
#pragma unroll                                                  // while the next step's prologue runs
        for (int i = 0; i < 64; ++i) hB[i] = ld1(c.scr_r, lo, H_SLOT(i));
        hpre = true;
    }
    PROF_MARK(2 * (t + 1) + 1);
    return true;
}

#if DECODE_PROF
// timing build only: one launch per step t, so the marks of every workgroup and step land in its own seq slots
template <bool PAIRS>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_step_kernel(DecodeParams p, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const Ctx c = make_ctx(p);
    if (t > 0 && p.alive[c.wg] == 0) return;
    Stage64Regs s64;
    bool pre = false, hpre = false;
    float hB[64];
    step_body<PAIRS, false>(p, c, lds, t, s64, pre, hB, hpre);
}
#endif

// The whole decode of a workgroup (steps t = -1 .. T) in one launch: a member's steps depend only on
// that member, so nothing needs a grid-wide step boundary. Saves the per-launch ramp and tail (every
// CU waits for the slowest at each of the T + 2 step boundaries), the launch gaps and the per-launch
// workgroup setup; the state between steps stays in the same lane scratch, and a lane re-reads only
// slots it wrote itself (a same-address store -> load of one lane: ordered like any C++ store/load pair).
// The LDS stage buffers are free at a step boundary: every step ends on a barrier after its last read.
// SAMPLE: the workgroup holds one of p.slog_ns logit slots for its lifetime, claimed from the slot flags at its
// start (the first free one from its block index mod ns; fewer workgroups are resident than there are slots, one
// per CU) and released at its end, after every wave's last read of it
template <bool PAIRS, bool SAMPLE = false>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_steps_kernel(DecodeParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    Ctx c = make_ctx<SAMPLE>(p);
    int slot = -1;
    if constexpr (SAMPLE) {
        __shared__ int slot_sh;
        if (c.tid == 0) {
            int q = (int)((blockIdx.x + blockIdx.y * gridDim.x) % (unsigned)p.slog_ns);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (atomicCAS(p.slog_slots + q, 0, 1) != 0) {
                q = q + 1 == p.slog_ns ? 0 : q + 1;
                if (__builtin_amdgcn_s_memrealtime() - t0 > SLOT_SPIN_TICKS) {   // no free slot: report, leave
                    atomicAdd(p.stats + 3, 1);
                    q = -1;
                    break;
                }
            }
            // the previous owner's stores were released before its flag store: acquire them, so this XCD's L2 holds
            // no stale line of the slot (the slot is larger than an L2)
            if (q >= 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            slot_sh = q;
        }
        __syncthreads();
        slot = slot_sh;
        if (slot < 0) return;
        const int nst = (p.V1 + 63) >> 6;
        const uint32_t sbytes = SLOG_STAGE_BYTES * (uint32_t)nst + SLOG_BLK_BYTES * (uint32_t)((nst + SLOG_BLOCK - 1) / SLOG_BLOCK);
        c.slog_r = make_rsrc(p.slog + (size_t)slot * (sbytes / 4), sbytes);
        static_assert(SLOG_STAGE_BYTES % 4 == 0, "slot stage size");
    }
    Stage64Regs s64;
    bool pre = false, hpre = false;
    float hB[64];
    for (int t = -1; t <= p.T; ++t)
        if (!step_body<PAIRS, true, SAMPLE>(p, c, lds, t, s64, pre, hB, hpre)) break;
    if constexpr (SAMPLE) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // this wave's accesses of the slot are done
        __syncthreads();
        if (c.tid == 0) {
            // release: this XCD's dirty lines of the slot reach HBM before another workgroup (maybe on another XCD)
            // can claim it; the explicit vmcnt keeps the flag store behind the L2 write-back (MI355X_MICROARCH.md)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(p.slog_slots + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// a mutated greedy decode on the fused path (MutHead: the embedding rows' delta' formed in step_body)
template <bool PAIRS>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_steps_mut_kernel(DecodeParams p, MutHead mh) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const Ctx c = make_ctx(p);
    const MutRes mr = mut_res(p, mh, c.member);
    Stage64Regs s64;
    bool pre = false, hpre = false;
    float hB[64];
    for (int t = -1; t <= p.T; ++t)
        if (!step_body<PAIRS, true, false, true>(p, c, lds, t, s64, pre, hB, hpre, &mr)) break;
}

// ========== split path: one member step over several workgroups =================================
// When members x slabs workgroups cannot fill the chip (64 members per GPU: configs[1] pop=64 and
// the per-GPU slice of configs[4]), each step t is split in two launches:
//   nicnes_decode_logit_kernel  grid (S, members, slabs): the logit GEMM of step t over vocabulary
//       stage range q; each lane leaves its rows' partial greedy state (online max and exp-sum, the
//       last two left-to-right records, the largest evicted record) in HBM;
//   nicnes_decode_cell_kernel   grid (Sc, members, slabs), Sc = min(S, 4): every workgroup of the
//       member merges the S partials into the same token (the fused kernel's candidate rule holds on
//       any partition of the vocabulary scanned in index order: the first in-window id of a range is
//       one of that range's last two records unless an evicted record is in the window too, which
//       sends the row to the exact pass), then runs the gate tiles of its 4/Sc unit blocks.
// h crosses launches in two parity slots: cell(t) reads h_t and writes its blocks of h_{t+1}. The
// unfinished flag of a row is seq[t-2] != 0 (it = tok * unfinished, nets.py:236-241). The q index
// is blockIdx.x, so consecutive workgroups (round-robin over the 8 XCDs) take different vocabulary
// ranges and each XCD's L2 holds a quarter of the logit matrix at S = 4.
#define HP_SLOT(par, s) (4u * 64u * (uint32_t)((par) ? 193 + (s) : 64 + (s)))   // h' by step parity

__device__ __forceinline__ float* part_ptr(const DecodeParams& p, int wg, int q, int wave) {
    return p.part + (((size_t)wg * p.S + q) * 8 + wave) * (7 * 64);
}

template <int G, bool PAIRS>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_logit_kernel(DecodeParams p, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SCtx<G> c = make_sctx<G>(p);
    PROF_SPLIT(2 * t - 2);
    if (t > 1 && p.alive2[((t - 1) & 1) * p.alive_stride + c.wg] == 0) return;
    const uint32_t lo = 4u * c.lane;
    const int nst = (p.V1 + 63) >> 6, S = (int)gridDim.x;
    // the coop kernel's range split (coop_step), so that both paths merge the same partials (bit-identical tokens
    // and log-probs); ±0 on this path's own timing (P = 64, B = 64)
    const int sh = nst >= 2 * S ? 1 : 0;
    const int s0 = c.q * nst / S + (c.q > 0 ? sh : 0), s1 = (c.q + 1) * nst / S + (c.q + 1 < S ? sh : 0);
    const uint64_t nidx = p.noise_idx[c.member];
    float hB[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) hB[i] = ld1(c.scr_r, lo, HP_SLOT(t & 1, i));
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(hB[i]);
    RowState st;
    row_state_init(st);
    Stage64Regs s64;
    if (s1 > s0) logit_stages<G, PAIRS>(lds, p, nidx, c.wave, c.sgn, c.hf, hB, s0, s1, st, s64);
    float* pb = part_ptr(p, c.wg, c.q, c.wave) + lane_fresh();
    pb[0] = st.m;
    pb[64] = st.s;
    pb[128] = st.r0v;
    pb[192] = __builtin_bit_cast(float, st.r0i);
    pb[256] = st.r1v;
    pb[320] = __builtin_bit_cast(float, st.r1i);
    pb[384] = st.ev;
    PROF_SPLIT(2 * t - 1);
}

// partials k0 .. k0+7 of a row (those < nk: the merge skips the others)
struct Part8 {
    float m[8], s[8], r0v[8], r1v[8], ev[8];
    int r0i[8], r1i[8];
};
__device__ __forceinline__ void load_part8(const DecodeParams& p, int wg, int wave, int lane, int nh, int nk, int k0,
                                           Part8& o) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
        if (k0 + u < nk) {                        // uniform: no load for the absent partials
            const int k = k0 + u;
            const float* pb = part_ptr(p, wg, k / nh, wave + k % nh) + lane;
            o.m[u] = pb[0]; o.s[u] = pb[64];
            o.r0v[u] = pb[128]; o.r1v[u] = pb[256]; o.ev[u] = pb[384];
            o.r0i[u] = __builtin_bit_cast(int, pb[192]); o.r1i[u] = __builtin_bit_cast(int, pb[320]);
        }
}

// Merge of a row's nk = S * nh partial greedy states (split and coop paths): the merged (m, s) give the
// tie window; the token is the first in-window record; ovf when a record is undecided (PAIRS) or an
// evicted record is in the window (-> merge_exact). pre holds partials 0..7 (loaded by the caller).
__device__ __forceinline__ void merge_partials(const DecodeParams& p, int wg, int wave, int lane, int nh, int nk,
                                               const Part8& pre, bool pairs, float& m, float& lse, int& tok,
                                               bool& ovf) {
    float mh = -1.0e30f, sh = 0.f;
    for (int k0 = 0; k0 < nk; k0 += 8) {              // every load of 8 partials issued before use
        Part8 cur;
        if (k0 == 0) cur = pre; else load_part8(p, wg, wave, lane, nh, nk, k0, cur);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k0 + u < nk) {
                const float mn = fmaxf(mh, cur.m[u]);
                sh = sh * __builtin_amdgcn_exp2f((mh - mn) * LOG2E) + cur.s[u] * __builtin_amdgcn_exp2f((cur.m[u] - mn) * LOG2E);
                mh = mn;
            }
    }
    const float m_o = __shfl_xor(mh, 32);
    const float s_o = __shfl_xor(sh, 32);
    m = fmaxf(mh, m_o);
    const float stot = sh * __builtin_amdgcn_exp2f((mh - m) * LOG2E) + s_o * __builtin_amdgcn_exp2f((m_o - m) * LOG2E);
    const TieWindow w = tie_window(stot, pairs, p.lse_margin);
    lse = w.lse;
    for (int k0 = 0; k0 < nk; k0 += 8) {
        Part8 cur;
        if (k0 == 0) cur = pre; else load_part8(p, wg, wave, lane, nh, nk, k0, cur);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (k0 + u < nk) {
                const int w0 = win_state(cur.r0v[u], m, w), w1 = win_state(cur.r1v[u], m, w);
                if (w0 == 1 && cur.r0i[u] < tok) tok = cur.r0i[u];
                if (w1 == 1 && cur.r1i[u] < tok) tok = cur.r1i[u];
                ovf = ovf || w0 == 2 || w1 == 2 || win_state(cur.ev[u], m, w) != 0;
            }
    }
    tok = min(tok, __shfl_xor(tok, 32));
    ovf = ovf || (__shfl_xor(ovf ? 1 : 0, 32) != 0);
}

// rare: more records than tracked fall in the tie window, or (PAIRS mode) the bounds on lse leave a
// record undecided -> exact pass over the whole vocabulary (every workgroup of the member does it: it
// needs the token); PAIRS mode sums the exp first and re-decides from the records, sweeping for the
// first id only when an evicted record is in the window. Workgroup-uniform call (barriers inside).
__device__ __forceinline__ void merge_exact(const DecodeParams& p, float* lds, int wg, rsrc_t theta_r, rsrc_t noise_r,
                                            int tid, int sgn, int hh, int wave, int lane, int nh, int nk,
                                            const float (&hB)[64], bool folder, bool pairs, float m, float& lse,
                                            int& tok) {
    int best = 0x7fffffff;
    float ssum = 0.f;
    bool find = true;
    if (pairs) {
        exact_sweep(lds, p, theta_r, noise_r, tid, sgn, hh, lane, hB, folder, true, m, 0.f, ssum, best);
        lse = logf(ssum + __shfl_xor(ssum, 32));
        int t2 = 0x7fffffff;
        bool ev2 = p.force_exact;
        if (folder) {
            for (int k = 0; k < nk; ++k) {
                const float* pb = part_ptr(p, wg, k / nh, wave + k % nh) + lane;
                const float r0v = pb[128], r1v = pb[256];
                const int r0i = __builtin_bit_cast(int, pb[192]), r1i = __builtin_bit_cast(int, pb[320]);
                if (in_window(r0v, m, lse) && r0i < t2) t2 = r0i;
                if (in_window(r1v, m, lse) && r1i < t2) t2 = r1i;
                ev2 = ev2 || in_window(pb[384], m, lse);
            }
            t2 = min(t2, __shfl_xor(t2, 32));
            ev2 = ev2 || (__shfl_xor(ev2 ? 1 : 0, 32) != 0);
        }
        find = __syncthreads_or(ev2 ? 1 : 0) != 0;
        if (!find) tok = t2;
    }
    if (find) {
        exact_sweep(lds, p, theta_r, noise_r, tid, sgn, hh, lane, hB, folder, false, m, lse, ssum, best);
        tok = min(best, __shfl_xor(best, 32));
    }
}

template <int G>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_cell_kernel(DecodeParams p, int t) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SCtx<G> c = make_sctx<G>(p);
    const bool lead = c.q == 0 && c.tid == 0;
    [[maybe_unused]] const int pb0 = 32 + 12 * (t + 1);   // DECODE_PROF slots: start, merged, staged, 5 tiles, end
    PROF_SPLIT(pb0);
    if (t > 1 && p.alive2[((t - 1) & 1) * p.alive_stride + c.wg] == 0) {
        if (lead) p.alive2[(t & 1) * p.alive_stride + c.wg] = 0;   // keep the parity chain current
        return;
    }
    const uint32_t lo = 4u * c.lane;
    const bool folder = G == 4 || c.hf == 0;       // waves that own the rows' token and the cell fold
    const uint32_t ib = (uint32_t)p.off_i2h_b, hb = (uint32_t)p.off_h2h_b, bmin = min(ib, hb);
    auto csrc = [&](int m) {                                     // gate tile m: i2h rows | h2h rows
        const uint32_t r = gate_row(m);
        StageSrc Sx;
        Sx.w_r = c.theta_r; Sx.z_r = c.noise_r; Sx.b_r = c.theta_r; Sx.bz_r = c.noise_r;
        Sx.so_a = 4u * ((uint32_t)p.off_i2h_w + 128u * r);
        Sx.so_b = 4u * ((uint32_t)p.off_h2h_w + 128u * r);
        Sx.bso = 4u * (bmin + r);
        Sx.bda = 4u * (ib - bmin); Sx.bdb = 4u * (hb - bmin);
        Sx.valid = 64;
        return Sx;
    };
    const int nb = 4 / (int)gridDim.x, m0 = 5 * nb * c.q, m1 = m0 + 5 * nb;
    const int nh = G == 4 ? 1 : 2, nk = p.S * nh;             // partial k = q * nh + f, in (q, f) order
    // load order = order of need: the first 8 partials of the rows, the first gate tile, then h (after
    // the merge). vmcnt retires in issue order and counts at most 63 loads: a load issued ahead of the
    // partials, or more than 63 behind them, would make the merge wait for the 64 KB tile
    PROF_SPLIT(pb0 + 8);
    Part8 pre;
    if (t >= 1 && folder) load_part8(p, c.wg, c.wave, c.lane, nh, nk, 0, pre);
#if DECODE_PROF
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PROF_SPLIT(pb0 + 9);
#endif
    Stage64Regs s64;
    // the first gate tile's rows do not depend on the token: their loads fly during the merge
    if (t < p.T) stage64_load(csrc(m0), c.wave * 64 + lane_fresh(), s64);
    float hB[64];
    auto load_h = [&]() {
        if (t < 0) {
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = 0.f;           // h = 0 before the first cell
        } else {
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = ld1(c.scr_r, lo, HP_SLOT(t & 1, i));
        }
#pragma unroll
        for (int i = 0; i < 64; ++i) pin(hB[i]);
    };
    int it = 0;                                   // token fed to the next cell (0 = BOS at t = 0)
    if (t >= 1) {
        // ---- merge the S partial states of each row (lane halves combined last, as the fused kernel)
        float m = 0.f, lse = 0.f;
        int tok = 0x7fffffff;
        bool ovf = false;
        const bool pairs = p.bounded_lse && p.lp == nullptr;   // the logit kernel ran its PAIRS variant
        if (folder) merge_partials(p, c.wg, c.wave, c.lane, nh, nk, pre, pairs, m, lse, tok, ovf);
        PROF_SPLIT(pb0 + 10);
        load_h();
        if (__syncthreads_or((p.force_exact || ovf) ? 1 : 0)) {
            merge_exact(p, lds, c.wg, c.theta_r, c.noise_r, c.tid, c.sgn, c.hh, c.wave, c.lane, nh, nk, hB, folder,
                        pairs, m, lse, tok);
            if (lead) atomicAdd(p.stats + 0, 1);
        }
        if (tok >= p.V1) tok = 0;               // every logit NaN: end the caption (fused kernel rule)
        const size_t o = (((size_t)c.member * 2 + c.sgn) * p.B + c.bc) * p.T + (t - 1);
#if DECODE_PROF
        const bool prev_unf = true;             // timing build: seq holds the marks
#else
        const bool prev_unf = t == 1 || p.seq[o - 1] != 0;
#endif
        const bool unfinished = prev_unf && tok > 0;
        it = (unfinished || p.no_mask) ? tok : 0;
#if !DECODE_PROF
        if (c.q == 0 && folder && c.hh == 0 && c.row_valid) {
            p.seq[o] = it;
            if (p.lp) p.lp[o] = -lse;           // seq_logprobs[:, t-1] (nets.py:208,241)
        }
#endif
        const int any = __syncthreads_or(((folder && unfinished && c.row_valid) || p.no_exit) ? 1 : 0);
        if (lead) p.alive2[(t & 1) * p.alive_stride + c.wg] = any;
        if (!any) return;                       // the reference stops here (nets.py:242-243)
        PROF_SPLIT(pb0 + 1);
    } else {
        load_h();
        if (t == 0 && lead) p.alive2[c.wg] = 1;   // parity slot 0 read by step 1
    }
    if (t >= p.T) return;

    // ---- LSTM cell of step t+1, gate tiles of this workgroup's unit blocks -------------------
    float xB[64];
    if (!folder) {
#pragma unroll
        for (int i = 0; i < 64; ++i) xB[i] = 0.f;
    } else if (t < 0) {                                          // x = img_embed(fc) (nets.py:194-195)
#pragma unroll
        for (int i = 0; i < 64; ++i) xB[i] = ld1(c.scr_r, lo, X_SLOT(i));
    } else {                                                     // x = embed(it) (nets.py:196-199)
        const uint32_t eo = 4u * ((uint32_t)p.off_emb_w + (uint32_t)it * 128u + 4u * c.hh);
#pragma unroll
        for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 w = ld4(c.theta_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 z = ld4(c.noise_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 delta = z;                      // fp32(sigma * z): the table is sigma-scaled
                const f32x4 x = c.sgn ? (w - delta) : (w + delta);
#pragma unroll
                for (int e = 0; e < 4; ++e) xB[16 * T + 4 * a + e] = x[e];
            }
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(xB[i]);
    const int hpar = (t + 1) & 1;
    stage64_store(lds, 64, c.wave * 64 + lane_fresh(), s64);
    __syncthreads();
    PROF_SPLIT(pb0 + 2);
    f32x16 hold;
    auto fold = [&](int m, const f32x16& s_, const f32x16& cpre) __attribute__((always_inline)) {
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
        const int U = m / 5, j5 = m % 5;
        if (j5 == 0) {                                           // g1
            hold = s_;
        } else if (j5 == 1) {                                    // g = max(g1, g2)
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = hold[r] > s_[r] ? hold[r] : s_[r];
        } else if (j5 == 2) {                                    // ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = CELL_SIG(s_[r]) * hold[r];
        } else if (j5 == 3) {                                    // c' = f * c + ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float fcv = CELL_SIG(s_[r]) * cpre[r];
                const float cn = fcv + hold[r];
                st1(c.scr_r, lo_, C_SLOT(16 * U + r), cn);
                hold[r] = cn;
            }
        } else {                                                 // h' = o * tanh(c')
#pragma unroll
            for (int r = 0; r < 16; ++r)
                st1(c.scr_r, lo_, HP_SLOT(hpar, 16 * U + r), CELL_SIG(s_[r]) * CELL_TANH(hold[r]));
        }
    };
    auto load_c = [&](int m) __attribute__((always_inline)) {                                   // c of the f tile's unit block
        f32x16 cp;
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
#pragma unroll
        for (int r = 0; r < 16; ++r) cp[r] = (m % 5 == 3 && t >= 0) ? ld1(c.scr_r, lo_, C_SLOT(16 * (m / 5) + r)) : 0.f;
        return cp;
    };
    float* xch = lds + 2 * STAGE64_FLOATS + (c.sgn * 2 + c.grp) * 1024;   // G = 2: h2h half -> i2h half
#pragma unroll 1
    for (int m = m0; m < m1; ++m) {
        const f32x16 cpre = load_c(m);
        __builtin_amdgcn_sched_barrier(0);
        if (m + 1 < m1) stage64_load(csrc(m + 1), c.wave * 64 + lane_fresh(), s64);
        const float* buf = lds + ((m - m0) & 1) * STAGE64_FLOATS;
        if constexpr (G == 4) {
            f32x16 a0, a1;
            if (t < 0)      // h = 0 before the first cell: h2h(h) is its bias
                mfma_xh_part<0, 4, false>(buf + c.sgn * (64 * LDS_ROW), buf + 2 * 64 * LDS_ROW + 64 * c.sgn, xB, hB, lane_fresh(), a0, a1);
            else
                mfma_xh_part<0, 4>(buf + c.sgn * (64 * LDS_ROW), buf + 2 * 64 * LDS_ROW + 64 * c.sgn, xB, hB, lane_fresh(), a0, a1);
            fold(m, a0 + a1, cpre);                              // i2h(x) + h2h(h), nets.py:109-111
            if (m + 1 < m1) stage64_store(lds + ((m - m0 + 1) & 1) * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
            __syncthreads();
        } else {
            // half 0: i2h tile over x (chain a); half 1: h2h tile over h (chain b), handed over in LDS
            const float* w1 = buf + c.sgn * (64 * LDS_ROW) + 32 * c.hf * LDS_ROW;
            const float* b1 = buf + 2 * 64 * LDS_ROW + 64 * c.sgn + 32 * c.hf;
            f32x16 a = bias_init(b1, lane_fresh() >> 5);
            if (c.hf == 0) a = mfma_tile(a, w1, xB, lane_fresh());
            else if (t >= 0) a = mfma_tile(a, w1, hB, lane_fresh());
            if (c.hf == 1) {
                const int l = lane_fresh();
#pragma unroll
                for (int r = 0; r < 16; ++r) xch[r * 64 + l] = a[r];
            }
            __syncthreads();
            if (c.hf == 0) {
                const int l = lane_fresh();
                f32x16 a1;
#pragma unroll
                for (int r = 0; r < 16; ++r) a1[r] = xch[r * 64 + l];
                fold(m, a + a1, cpre);                           // i2h(x) + h2h(h), nets.py:109-111
            }
            if (m + 1 < m1) stage64_store(lds + ((m - m0 + 1) & 1) * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
            __syncthreads();
        }
        if (m - m0 < 5) PROF_SPLIT(pb0 + 3 + (m - m0));
    }
    PROF_SPLIT(pb0 + 11);
}

// ========== coop path: the split decode in ONE launch ==============================================
// For populations too small to fill the chip with one workgroup per member slab (64 members per GPU:
// configs[1], the per-GPU slice of configs[4] and of the metric at 8 GPUs; 128 at 4 GPUs), the S
// workgroups of a member slab split the vocabulary as the split path does, but run every step in one
// persistent launch and hand each other data inside it: per step t >= 1 the partial greedy states of
// the logit ranges (phase A), then per step the unit blocks of h' (phase B). Every workgroup merges the
// S partials into the same token (the tie rule holds on any partition of the vocabulary), runs the gate
// tiles of its 4 / S unit blocks, and after phase B reads the whole h_{t+1} back for its logit range.
// The logit W0 rows stay split over the XCDs as on the split path (workgroup L takes range q = L % S, and
// blocks L, L + 8, ... share an XCD), and a phase's first staging tile is loaded during the previous
// phase, as in the fused steps kernel.
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility; cdna_hip_programming.md Guideline 16, R1):
// payload stored write-through (sc1) -> every storing wave s_waitcnt vmcnt(0) -> barrier -> one lane's
// agent-scope atomic add on the group's counter; the consumer's wave 0 polls the counter relaxed, then
// one agent acquire + vmcnt(0) + barrier before the plain loads. Counters are zeroed before each launch
// (phase k complete = S * k arrivals). Residency: S * members * slabs <= CUs (checked on the host) and
// one workgroup per CU (LDS), so a group's workgroups are resident together; every spin is bounded.
#define COOP_SPIN_TICKS 50000000ull      // 0.5 s of s_memrealtime (100 MHz): a partner that never arrives

__device__ __forceinline__ void st1_wt(rsrc_t r, uint32_t byte_off, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)byte_off, (int)soff, 16);   // sc1
}

__device__ __forceinline__ void coop_arrive(uint32_t* ctr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // this wave's write-through stores have landed
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// false (for every thread) when the partners have not arrived within COOP_SPIN_TICKS: the launch then
// ends early and stats[2] counts it (the engine reports it as an error). ACQ: one agent acquire after the
// poll (plain loads of the handed-off bytes may follow); without it every such load must be an sc1 load
// (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 hand-off table)
template <bool ACQ = true>
__device__ __forceinline__ bool coop_wait(uint32_t* ctr, uint32_t target, int32_t* stats) {
    int bad = 0;
    if (threadIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > COOP_SPIN_TICKS) {
                bad = 1;
                atomicAdd(stats + 2, 1);
                break;
            }
        }
    }
    if (ACQ && threadIdx.x < 64) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!ACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: the loads stay below the poll
    return __syncthreads_or(bad) == 0;
}

// one step of one coop workgroup (range q of its member slab); false when the group is done (every
// row finished, t = T, or a partner timed out). Mirrors step_body: s64 / pre carry a prefetched logit
// tile across steps; hB holds h_t on entry (read back after the previous step's phase B).
template <bool PAIRS, int S>
__device__ __forceinline__ bool coop_step(const DecodeParams& p, const Ctx& c, int q, float* lds, int t,
                                          Stage64Regs& s64, bool& pre, float (&hB)[64], uint32_t* ctr,
                                          uint32_t& phase) {
    [[maybe_unused]] const int pm = 8 * (t + 1);         // DECODE_PROF slots: start, logits, A, token, cell, B
    PROF_AT(blockIdx.x, 1024, pm);
    const uint32_t lo = 4u * c.lane;
    const int nst = (p.V1 + 63) >> 6;
    // the inner range boundaries one stage later than an even split: the last range, which holds the partial last
    // stage (it costs as much as a full one), gets one full stage less (P = 64 / 128: -0.7 / -0.6 %, round 6)
    const int sh = nst >= 2 * S ? 1 : 0;
    const int s0 = q * nst / S + (q > 0 ? sh : 0), s1 = (q + 1) * nst / S + (q + 1 < S ? sh : 0);
    // a range is never empty (nst >= S): without this the logit loop's zero-trip path changes the register
    // allocation of the whole step (the cell loop spills its B operand)
    __builtin_assume(s1 > s0);
    const int nb = 4 / S, m0 = 5 * nb * q, m1 = m0 + 5 * nb;
    const bool nl = t > 0;
    const uint64_t nidx = p.noise_idx[c.member];
    // the row's unfinished flag (every workgroup of the group writes the same value to the same slot)
    const float unf_prev = nl ? ld1(c.scr_r, lo, U_SLOT) : 0.f;
    if (t < 0) {
#pragma unroll
        for (int i = 0; i < 64; ++i) hB[i] = 0.f;               // h = 0 before the first cell
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(hB[i]);
    const uint32_t ib = (uint32_t)p.off_i2h_b, hb = (uint32_t)p.off_h2h_b, bmin = min(ib, hb);
    auto csrc = [&](int m) {                                     // gate tile m: i2h rows | h2h rows
        const uint32_t r = gate_row(m);
        StageSrc Sx;
        Sx.w_r = c.theta_r; Sx.z_r = c.noise_r; Sx.b_r = c.theta_r; Sx.bz_r = c.noise_r;
        Sx.so_a = 4u * ((uint32_t)p.off_i2h_w + 128u * r);
        Sx.so_b = 4u * ((uint32_t)p.off_h2h_w + 128u * r);
        Sx.bso = 4u * (bmin + r);
        Sx.bda = 4u * (ib - bmin); Sx.bdb = 4u * (hb - bmin);
        Sx.valid = 64;
        return Sx;
    };
    int it = 0;                                   // token fed to the next cell (0 = BOS at t = 0)
    bool cell_pre = false;                        // s64 holds the cell's first gate tile
    if (nl) {
        RowState st;
        row_state_init(st);
        auto tail = [&]() __attribute__((always_inline)) {
            if (t < p.T) stage64_load(csrc(m0), c.wave * 64 + lane_fresh(), s64);
        };
        // (no peel here: +1.4 % at P = 64, the coop kernel's spills 28 -> 80)
        logit_stages<4, PAIRS, false>(lds, p, nidx, c.wave, c.sgn, 0, hB, s0, s1, st, s64, pre, tail);
        cell_pre = t < p.T;
        PROF_AT(blockIdx.x, 1024, pm + 1);
        // ---- phase A: this range's partial greedy state, write-through, then the group's merge
        {
            const rsrc_t part_r = make_rsrc(part_ptr(p, c.wg, q, 0), PART_FLOATS * 4);
            const uint32_t po = 4u * (uint32_t)(c.wave * (7 * 64) + lane_fresh());
            st1_wt(part_r, po, 0u, st.m);
            st1_wt(part_r, po, 256u, st.s);
            st1_wt(part_r, po, 512u, st.r0v);
            st1_wt(part_r, po, 768u, __builtin_bit_cast(float, st.r0i));
            st1_wt(part_r, po, 1024u, st.r1v);
            st1_wt(part_r, po, 1280u, __builtin_bit_cast(float, st.r1i));
            st1_wt(part_r, po, 1536u, st.ev);
        }
        coop_arrive(ctr);
        ++phase;
#if !(DECODE_ABLATE & 128)
        if (!coop_wait(ctr, (uint32_t)S * phase, p.stats)) return false;
#endif
        PROF_AT(blockIdx.x, 1024, pm + 2);
        float m = 0.f, lse = 0.f;
        int tok = 0x7fffffff;
        bool ovf = false;
        {
            Part8 pr;
            load_part8(p, c.wg, c.wave, lane_fresh(), 1, S, 0, pr);
            merge_partials(p, c.wg, c.wave, lane_fresh(), 1, S, pr, PAIRS, m, lse, tok, ovf);
        }
        if (__syncthreads_or((p.force_exact || ovf) ? 1 : 0)) {
            // the exact sweep stages through LDS with registers of its own: the prefetched cell tile is
            // given up (reloaded below)
            merge_exact(p, lds, c.wg, c.theta_r, c.noise_r, c.tid, c.sgn, c.hh, c.wave, c.lane, 1, S, hB, true,
                        PAIRS, m, lse, tok);
            if (q == 0 && c.tid == 0) atomicAdd(p.stats + 0, 1);
            cell_pre = false;
        }
        if (tok >= p.V1) tok = 0;               // every logit NaN: end the caption (fused kernel rule)
        const bool unfinished = unf_prev != 0.f && tok > 0;
        it = (unfinished || p.no_mask) ? tok : 0;
        st1(c.scr_r, lo, U_SLOT, unfinished ? 1.f : 0.f);
#if !DECODE_PROF
        if (q == 0 && c.hh == 0 && c.row_valid) {
            const size_t o = (((size_t)c.member * 2 + c.sgn) * p.B + c.b) * p.T + (t - 1);
            p.seq[o] = it;
            if (p.lp) p.lp[o] = -lse;           // seq_logprobs[:, t-1] (nets.py:208,241)
        }
#endif
        PROF_AT(blockIdx.x, 1024, pm + 3);
        // every workgroup of the group reaches the same decision (the reference stops here, nets.py:242-243)
        if (!__syncthreads_or(((unfinished && c.row_valid) || p.no_exit) ? 1 : 0)) return false;
    }
    if (t >= p.T) return false;

    // ---- LSTM cell of step t+1, gate tiles of this workgroup's unit blocks (nets.py:98-134) ---------
    float xB[64];
    if (t < 0) {                                                 // x = img_embed(fc) (nets.py:194-195)
#pragma unroll
        for (int i = 0; i < 64; ++i) xB[i] = ld1(c.scr_r, lo, X_SLOT(i));
    } else {                                                     // x = embed(it) (nets.py:196-199)
        const uint32_t eo = 4u * ((uint32_t)p.off_emb_w + (uint32_t)it * 128u + 4u * c.hh);
#pragma unroll
        for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 w = ld4(c.theta_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 z = ld4(c.noise_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 x = c.sgn ? (w - z) : (w + z);         // the table is sigma-scaled
#pragma unroll
                for (int e = 0; e < 4; ++e) xB[16 * T + 4 * a + e] = x[e];
            }
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(xB[i]);
    const int hpar = (t + 1) & 1;
    if (!cell_pre) stage64_load(csrc(m0), c.wave * 64 + lane_fresh(), s64);
    stage64_store(lds, 64, c.wave * 64 + lane_fresh(), s64);
    __syncthreads();
    f32x16 hold;
    auto fold = [&](int m, const f32x16& s_, const f32x16& cpre) __attribute__((always_inline)) {
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
        const int U = m / 5, j5 = m % 5;
        if (j5 == 0) {                                           // g1
            hold = s_;
        } else if (j5 == 1) {                                    // g = max(g1, g2)
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = hold[r] > s_[r] ? hold[r] : s_[r];
        } else if (j5 == 2) {                                    // ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = CELL_SIG(s_[r]) * hold[r];
        } else if (j5 == 3) {                                    // c' = f * c + ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float fcv = CELL_SIG(s_[r]) * cpre[r];
                const float cn = fcv + hold[r];
                st1(c.scr_r, lo_, C_SLOT(16 * U + r), cn);      // c: read back only by this workgroup
                hold[r] = cn;
            }
        } else {                                                 // h' = o * tanh(c'), handed to the group
#pragma unroll
            for (int r = 0; r < 16; ++r)
                st1_wt(c.scr_r, lo_, HP_SLOT(hpar, 16 * U + r), CELL_SIG(s_[r]) * CELL_TANH(hold[r]));
        }
    };
    auto load_c = [&](int m) __attribute__((always_inline)) {   // c of the f tile's unit block
        f32x16 cp;
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
#pragma unroll
        for (int r = 0; r < 16; ++r) cp[r] = (m % 5 == 3 && t >= 0) ? ld1(c.scr_r, lo_, C_SLOT(16 * (m / 5) + r)) : 0.f;
        return cp;
    };
    const bool lpf = t >= 0;                                       // the next step's first logit tile
#pragma unroll 1
    for (int m = m0; m < m1; ++m) {
        const f32x16 cpre = load_c(m);
        __builtin_amdgcn_sched_barrier(0);
        if (m + 1 < m1) {
            stage64_load(csrc(m + 1), c.wave * 64 + lane_fresh(), s64);
        } else if (lpf) {
            const LaneOffs lo_ = lane_offs(c.wave, 128u);
            stage64_load_o(logit_src(p, nidx, s0), lo_, c.wave < 2, s64);
        }
        const float* buf = lds + ((m - m0) & 1) * STAGE64_FLOATS;
        f32x16 a0, a1;
        if (t < 0)      // h = 0 before the first cell: h2h(h) is its bias (fma(w, 0, acc) == acc)
            mfma_xh_part<0, 4, false>(buf + c.sgn * (64 * LDS_ROW), buf + 2 * 64 * LDS_ROW + 64 * c.sgn, xB, hB, lane_fresh(), a0, a1);
        else
            mfma_xh_part<0, 4>(buf + c.sgn * (64 * LDS_ROW), buf + 2 * 64 * LDS_ROW + 64 * c.sgn, xB, hB, lane_fresh(), a0, a1);
        fold(m, a0 + a1, cpre);                                  // i2h(x) + h2h(h), nets.py:109-111
        if (m + 1 < m1) stage64_store(lds + ((m - m0 + 1) & 1) * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
        __syncthreads();
    }
    pre = lpf;
    PROF_AT(blockIdx.x, 1024, pm + 4);
    // ---- phase B: h_{t+1} complete in the group -> every workgroup reads all of it
    coop_arrive(ctr);
    ++phase;
#if !(DECODE_ABLATE & 128)
    if (!coop_wait(ctr, (uint32_t)S * phase, p.stats)) return false;
#endif
    PROF_AT(blockIdx.x, 1024, pm + 5);
#pragma unroll
    for (int i = 0; i < 64; ++i) hB[i] = ld1(c.scr_r, lo, HP_SLOT(hpar, i));
    return true;
}

// grid: S x member slabs workgroups, L = blockIdx.x -> range q = L % S of group L / S
template <bool PAIRS, int S>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_coop_kernel(DecodeParams p, int nslabs) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int L = blockIdx.x, q = L % S, gi = L / S;
    Ctx c;
    c.tid = threadIdx.x;
    c.lane = c.tid & 63;
    c.wave = __builtin_amdgcn_readfirstlane(c.tid >> 6);
    c.sgn = c.wave >> 2;
    c.grp = c.wave & 3;
    c.hh = c.lane >> 5;
    c.member = gi / nslabs;
    c.slab = gi % nslabs;
    c.wg = gi;
    c.b = c.slab * 128 + c.grp * 32 + (c.lane & 31);
    c.row_valid = row_ok(p, c.b, c.sgn);
    c.bc = c.row_valid ? c.b : 0;
    const uint64_t nidx = p.noise_idx[c.member];
    const uint32_t Dbytes = 4u * (uint32_t)p.D;
    c.theta_r = make_rsrc(p.theta, Dbytes);
    c.noise_r = make_rsrc(p.noise + nidx, Dbytes);
    float* wscr = p.scratch + ((size_t)c.wg * 8 + c.wave) * (SCR_SLOTS * 64);
    c.scr_r = make_rsrc(wscr, SCR_SLOTS * 64 * 4);
    uint32_t* ctr = p.coop_ctr + (size_t)gi * COOP_CTR_STRIDE;
    uint32_t phase = 0;
    if (p.test_stall_ms && L == 0) {               // test hook: a partner that arrives past the spin bound
        if (c.tid == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < 100000ull * p.test_stall_ms) __builtin_amdgcn_s_sleep(127);
        }
        __syncthreads();
    }
    Stage64Regs s64;
    bool pre = false;
    float hB[64];
    for (int t = -1; t <= p.T; ++t)
        if (!coop_step<PAIRS, S>(p, c, q, lds, t, s64, pre, hB, ctr, phase)) break;
}

// ========== fused path for 64-row slabs (G = 2): every step of a workgroup in one launch =========
// B <= 64 (mscoco_nes.json's own batch_size 64) with one workgroup per member slab (S = 1): wave w =
// sign (w >> 2) x 32-row group ((w >> 1) & 1) x tile half (w & 1), as on the split path. Per step the
// two tile halves of a row group scan opposite halves of each 64-row logit stage; their partial greedy
// states go through memory (the workgroup's own part_ptr slots) to the half-0 waves, which merge them
// exactly as the split cell kernel does (nh = 2), pick the token and fold the cell; in every gate tile
// the half-1 waves run the h2h chain over h and hand it over in LDS (nicnes_decode_cell_kernel<2>).
// h' crosses steps in the lane scratch of the row group (parity slots), read back by both halves.
template <bool PAIRS>
__device__ __forceinline__ bool step_body2(const DecodeParams& p, const SCtx<2>& c, float* lds, int t,
                                           Stage64Regs& s64, bool& pre, float (&hB)[64]) {
    PROF_AT(c.wg, 4096, 2 * (t + 1));
    const uint32_t lo = 4u * c.lane;
    const int nst = (p.V1 + 63) >> 6;
    __builtin_assume(nst > 0);                     // (as in coop_step: no zero-trip logit loop)
    const bool nl = t > 0;
    const bool folder = c.hf == 0;                 // waves that own the rows' token and the cell fold
    const uint64_t nidx = p.noise_idx[c.member];
    const float unf_prev = (nl && folder) ? ld1(c.scr_r, lo, U_SLOT) : 0.f;
    if (t < 0) {
#pragma unroll
        for (int i = 0; i < 64; ++i) hB[i] = 0.f;               // h = 0 before the first cell
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(hB[i]);
    const uint32_t ib = (uint32_t)p.off_i2h_b, hb = (uint32_t)p.off_h2h_b, bmin = min(ib, hb);
    auto csrc = [&](int m) {                                     // gate tile m: i2h rows | h2h rows
        const uint32_t r = gate_row(m);
        StageSrc Sx;
        Sx.w_r = c.theta_r; Sx.z_r = c.noise_r; Sx.b_r = c.theta_r; Sx.bz_r = c.noise_r;
        Sx.so_a = 4u * ((uint32_t)p.off_i2h_w + 128u * r);
        Sx.so_b = 4u * ((uint32_t)p.off_h2h_w + 128u * r);
        Sx.bso = 4u * (bmin + r);
        Sx.bda = 4u * (ib - bmin); Sx.bdb = 4u * (hb - bmin);
        Sx.valid = 64;
        return Sx;
    };
    int it = 0;                                   // token fed to the next cell (0 = BOS at t = 0)
    bool cell_pre = false;                        // s64 holds the cell's first gate tile
    if (nl) {
        RowState st;
        row_state_init(st);
        auto tail = [&]() __attribute__((always_inline)) {
            if (t < p.T) stage64_load(csrc(0), c.wave * 64 + lane_fresh(), s64);
        };
        logit_stages<2, PAIRS>(lds, p, nidx, c.wave, c.sgn, c.hf, hB, 0, nst, st, s64, pre, tail);
        cell_pre = t < p.T;
        {   // this tile half's partial greedy state (read back by the half-0 wave of the row group)
            float* pb = part_ptr(p, c.wg, 0, c.wave) + lane_fresh();
            pb[0] = st.m;
            pb[64] = st.s;
            pb[128] = st.r0v;
            pb[192] = __builtin_bit_cast(float, st.r0i);
            pb[256] = st.r1v;
            pb[320] = __builtin_bit_cast(float, st.r1i);
            pb[384] = st.ev;
        }
        __syncthreads();
        float m = 0.f, lse = 0.f;
        int tok = 0x7fffffff;
        bool ovf = false;
        if (folder) {
            Part8 pr;
            load_part8(p, c.wg, c.wave, lane_fresh(), 2, 2, 0, pr);
            merge_partials(p, c.wg, c.wave, lane_fresh(), 2, 2, pr, PAIRS, m, lse, tok, ovf);
        }
        if (__syncthreads_or((p.force_exact || ovf) ? 1 : 0)) {
            merge_exact(p, lds, c.wg, c.theta_r, c.noise_r, c.tid, c.sgn, c.hh, c.wave, c.lane, 2, 2, hB, folder,
                        PAIRS, m, lse, tok);
            if (c.tid == 0) atomicAdd(p.stats + 0, 1);
            cell_pre = false;                   // the exact sweep staged through LDS with its own registers
        }
        if (tok >= p.V1) tok = 0;               // every logit NaN: end the caption (fused kernel rule)
        const bool unfinished = unf_prev != 0.f && tok > 0;
        it = unfinished ? tok : 0;
        if (folder) {
            st1(c.scr_r, lo, U_SLOT, unfinished ? 1.f : 0.f);
#if !DECODE_PROF
            if (c.hh == 0 && c.row_valid) {
                const size_t o = (((size_t)c.member * 2 + c.sgn) * p.B + c.b) * p.T + (t - 1);
                p.seq[o] = it;
                if (p.lp) p.lp[o] = -lse;       // seq_logprobs[:, t-1] (nets.py:208,241)
            }
#endif
        }
        const int any = __syncthreads_or(((folder && unfinished && c.row_valid) || p.no_exit) ? 1 : 0);
        if (!any) return false;                 // the reference stops here (nets.py:242-243)
    }
    if (t >= p.T) return false;

    // ---- LSTM cell of step t+1 (nets.py:98-134): half 0 i2h over x, half 1 h2h over h -------------
    float xB[64];
    if (!folder) {
#pragma unroll
        for (int i = 0; i < 64; ++i) xB[i] = 0.f;
    } else if (t < 0) {                                          // x = img_embed(fc) (nets.py:194-195)
#pragma unroll
        for (int i = 0; i < 64; ++i) xB[i] = ld1(c.scr_r, lo, X_SLOT(i));
    } else {                                                     // x = embed(it) (nets.py:196-199)
        const uint32_t eo = 4u * ((uint32_t)p.off_emb_w + (uint32_t)it * 128u + 4u * c.hh);
#pragma unroll
        for (int T = 0; T < 4; ++T)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 w = ld4(c.theta_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 z = ld4(c.noise_r, eo + 4u * (32 * T + 8 * a));
                const f32x4 x = c.sgn ? (w - z) : (w + z);         // the table is sigma-scaled
#pragma unroll
                for (int e = 0; e < 4; ++e) xB[16 * T + 4 * a + e] = x[e];
            }
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) pin(xB[i]);
    const int hpar = (t + 1) & 1;
    if (!cell_pre) stage64_load(csrc(0), c.wave * 64 + lane_fresh(), s64);
    stage64_store(lds, 64, c.wave * 64 + lane_fresh(), s64);
    __syncthreads();
    f32x16 hold;
    auto fold = [&](int m, const f32x16& s_, const f32x16& cpre) __attribute__((always_inline)) {
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
        const int U = m / 5, j5 = m % 5;
        if (j5 == 0) {                                           // g1
            hold = s_;
        } else if (j5 == 1) {                                    // g = max(g1, g2)
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = hold[r] > s_[r] ? hold[r] : s_[r];
        } else if (j5 == 2) {                                    // ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) hold[r] = CELL_SIG(s_[r]) * hold[r];
        } else if (j5 == 3) {                                    // c' = f * c + ig * g
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float fcv = CELL_SIG(s_[r]) * cpre[r];
                const float cn = fcv + hold[r];
                st1(c.scr_r, lo_, C_SLOT(16 * U + r), cn);
                hold[r] = cn;
            }
        } else {                                                 // h' = o * tanh(c')
#pragma unroll
            for (int r = 0; r < 16; ++r)
                st1(c.scr_r, lo_, HP_SLOT(hpar, 16 * U + r), CELL_SIG(s_[r]) * CELL_TANH(hold[r]));
        }
    };
    auto load_c = [&](int m) __attribute__((always_inline)) {   // c of the f tile's unit block
        f32x16 cp;
        const uint32_t lo_ = 4u * (uint32_t)lane_fresh();
#pragma unroll
        for (int r = 0; r < 16; ++r) cp[r] = (m % 5 == 3 && t >= 0) ? ld1(c.scr_r, lo_, C_SLOT(16 * (m / 5) + r)) : 0.f;
        return cp;
    };
    float* xch = lds + 2 * STAGE64_FLOATS + (c.sgn * 2 + c.grp) * 1024;   // h2h half -> i2h half
    const bool lpf = t >= 0;                                              // the next step's first logit tile
#pragma unroll 1
    for (int m = 0; m < 20; ++m) {
        const f32x16 cpre = load_c(m);
        __builtin_amdgcn_sched_barrier(0);
        if (m + 1 < 20) {
            stage64_load(csrc(m + 1), c.wave * 64 + lane_fresh(), s64);
        } else if (lpf) {
            const LaneOffs lo_ = lane_offs(c.wave, 128u);
            stage64_load_o(logit_src(p, nidx, 0), lo_, c.wave < 2, s64);
        }
        const float* buf = lds + (m & 1) * STAGE64_FLOATS;
        const float* w1 = buf + c.sgn * (64 * LDS_ROW) + 32 * c.hf * LDS_ROW;
        const float* b1 = buf + 2 * 64 * LDS_ROW + 64 * c.sgn + 32 * c.hf;
        f32x16 a = bias_init(b1, lane_fresh() >> 5);
        if (folder) a = mfma_tile(a, w1, xB, lane_fresh());
        else if (t >= 0) a = mfma_tile(a, w1, hB, lane_fresh());   // h = 0 before the first cell: the bias
        if (!folder) {
            const int l = lane_fresh();
#pragma unroll
            for (int r = 0; r < 16; ++r) xch[r * 64 + l] = a[r];
        }
        __syncthreads();
        if (folder) {
            const int l = lane_fresh();
            f32x16 a1;
#pragma unroll
            for (int r = 0; r < 16; ++r) a1[r] = xch[r * 64 + l];
            fold(m, a + a1, cpre);                               // i2h(x) + h2h(h), nets.py:109-111
        }
        if (m + 1 < 20) stage64_store(lds + ((m + 1) & 1) * STAGE64_FLOATS, 64, c.wave * 64 + lane_fresh(), s64);
        __syncthreads();
    }
    pre = lpf;
    // h_{t+1}: the half-0 waves' h' stores of the row group, read back by both halves
#pragma unroll
    for (int i = 0; i < 64; ++i) hB[i] = ld1(c.scr_r, lo, HP_SLOT(hpar, i));
    PROF_AT(c.wg, 4096, 2 * (t + 1) + 1);
    return true;
}

template <bool PAIRS>
__global__ __launch_bounds__(NTHREADS) void nicnes_decode_steps2_kernel(DecodeParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const SCtx<2> c = make_sctx<2>(p);            // grid (1, members, slabs)
    Stage64Regs s64;
    bool pre = false;
    float hB[64];
    for (int t = -1; t <= p.T; ++t)
        if (!step_body2<PAIRS>(p, c, lds, t, s64, pre, hB)) break;
}

namespace {
const size_t LDS64 = (size_t)(2 * STAGE64_FLOATS) * sizeof(float);
const size_t LDS32 = (size_t)(2 * STAGE_FLOATS) * sizeof(float);
const size_t LDS_CELL2 = LDS64 + (size_t)4 * 1024 * sizeof(float);   // + the G = 2 hand-over buffer
}

// per device, once per handle (nicnes_create, after hipSetDevice): dynamic LDS above 64 KB
extern "C" hipError_t nicnes_decode_init() {
    const struct { const void* f; size_t b; } ks[] = {
#if DECODE_PROF
        {(const void*)nicnes_decode_step_kernel<true>, LDS64},
        {(const void*)nicnes_decode_step_kernel<false>, LDS64},
#endif
        {(const void*)nicnes_decode_img64_kernel, LDS64},
        {(const void*)nicnes_decode_steps_kernel<true>, LDS64},
        {(const void*)nicnes_decode_steps_kernel<false>, LDS64},
        {(const void*)nicnes_decode_steps_kernel<false, true>, LDS64},
        {(const void*)nicnes_decode_steps_mut_kernel<true>, LDS64},
        {(const void*)nicnes_decode_steps_mut_kernel<false>, LDS64},
        {(const void*)nicnes_decode_logit_kernel<4, true>, LDS64},
        {(const void*)nicnes_decode_logit_kernel<4, false>, LDS64},
        {(const void*)nicnes_decode_logit_kernel<2, true>, LDS64},
        {(const void*)nicnes_decode_logit_kernel<2, false>, LDS64},
        {(const void*)nicnes_decode_cell_kernel<4>, LDS64},
        {(const void*)nicnes_decode_coop_kernel<true, 2>, LDS64},
        {(const void*)nicnes_decode_coop_kernel<false, 2>, LDS64},
        {(const void*)nicnes_decode_coop_kernel<true, 4>, LDS64},
        {(const void*)nicnes_decode_coop_kernel<false, 4>, LDS64},
        {(const void*)nicnes_decode_cell_kernel<2>, LDS_CELL2},
        {(const void*)nicnes_decode_steps2_kernel<true>, LDS_CELL2},
        {(const void*)nicnes_decode_steps2_kernel<false>, LDS_CELL2},
        {(const void*)nicnes_decode_img_kernel<4>, LDS32},
        {(const void*)nicnes_decode_img_mut_kernel, LDS32},
        {(const void*)nicnes_decode_img_kernel<2>, LDS32},
    };
    for (const auto& k : ks) {
        hipError_t e = hipFuncSetAttribute(k.f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)k.b);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

extern "C" hipError_t nicnes_decode_occupancy(int* coop_per_cu, int* sample_per_cu) {
    const void* coop[] = {(const void*)nicnes_decode_coop_kernel<true, 2>, (const void*)nicnes_decode_coop_kernel<false, 2>,
                          (const void*)nicnes_decode_coop_kernel<true, 4>, (const void*)nicnes_decode_coop_kernel<false, 4>};
    int lo = 1 << 30;
    for (const void* f : coop) {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, NTHREADS, LDS64);
        if (e != hipSuccess) return e;
        lo = n < lo ? n : lo;
    }
    *coop_per_cu = lo;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(sample_per_cu, (const void*)nicnes_decode_steps_kernel<false, true>,
                                                        NTHREADS, LDS64);
}

extern "C" void nicnes_decode_shift(DecodeParams* p, int m0, int nslabs, MutHead* mh) {
    const size_t wg0 = (size_t)m0 * (size_t)nslabs;        // workgroup index wg = member * slabs + slab
    const size_t rows = (size_t)m0 * 2 * (size_t)p->B * (size_t)p->T;
    p->noise_idx += m0;
    if (mh && mh->head_idx) mh->head_idx += m0;
    if (p->member_batch) p->member_batch += m0;
    p->seq += rows;
    if (p->lp) p->lp += rows;
    p->scratch += wg0 * (size_t)(2 * p->G) * (SCR_SLOTS * 64);   // make_ctx / make_sctx lane scratch
    p->alive += wg0;
    p->alive2 += wg0;
    p->part += wg0 * (size_t)p->S * PART_FLOATS;                 // part_ptr
    if (p->coop_ctr) p->coop_ctr += wg0 * COOP_CTR_STRIDE;
}

extern "C" hipError_t nicnes_launch_decode(const DecodeParams* p, const MutHead* mh, int member_count, int nslabs,
                                           hipStream_t stream, hipEvent_t* evs, int* kinds, int* n_launch) {
    const bool fused = p->G == 4 && p->S == 1;
    if (p->G != 4 && p->G != 2) return hipErrorInvalidValue;
    if (p->S < 1 || p->S > 64) return hipErrorInvalidValue;
    if (p->coop && (p->G != 4 || (p->S != 2 && p->S != 4) || !p->coop_ctr)) return hipErrorInvalidValue;
    if (p->sample_u && (!fused || p->coop)) return hipErrorInvalidValue;     // the sampled pick: fused path only
    // delta' formed in the decode for the head parameters: the fused greedy kernels only
    const bool mut = mh && mh->mode;
    if (mut && (!fused || p->coop || p->sample_u || !mh->head_noise || !mh->head_idx || !mh->mut_vec))
        return hipErrorInvalidValue;
    const int nl = fused || p->coop ? p->T + 3 : 3 + 2 * p->T;
    if (evs && nl + 1 > DECODE_MAX_EVENTS) return hipErrorInvalidValue;
    int ne = 0;
    auto mark = [&](int kind) {
        if (evs) {
            if (ne > 0) kinds[ne] = kind;
            (void)hipEventRecord(evs[ne++], stream);
        }
    };
    const dim3 block(NTHREADS);
    // greedy-only decodes (no log-prob output) may bound lse by pair maxima (PAIRS, the engine decides:
    // nicnes_evaluate_batches); with p->lp the exact exp-sum gives seq_logprobs
    const bool pairs = p->bounded_lse && p->lp == nullptr;
    mark(0);
    if (p->coop) {
        // the group counters are zeroed before every launch (one 128-byte line per member slab)
        hipError_t e = hipMemsetAsync(p->coop_ctr, 0, (size_t)member_count * nslabs * COOP_CTR_STRIDE * sizeof(uint32_t),
                                      stream);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(nicnes_decode_img_kernel<4>, dim3(p->S, member_count, nslabs), block, LDS32, stream, *p);
        mark(DK_IMG);
        const dim3 grid(p->S * member_count * nslabs);
        const void* kf = p->S == 2 ? (pairs ? (const void*)nicnes_decode_coop_kernel<true, 2>
                                            : (const void*)nicnes_decode_coop_kernel<false, 2>)
                                   : (pairs ? (const void*)nicnes_decode_coop_kernel<true, 4>
                                            : (const void*)nicnes_decode_coop_kernel<false, 4>);
        DecodeParams pk = *p;
        int ns = nslabs;
        void* args[] = {&pk, &ns};
        // the group hand-offs need every workgroup resident at once: the engine bounds the grid by the occupancy query
        // (coop_fits); the cooperative launch (opt-in) has the runtime check it too and fail instead of queueing a
        // workgroup behind its partners
        e = p->coop_launch ? hipLaunchCooperativeKernel(kf, grid, block, args, LDS64, stream)
                           : hipLaunchKernel(kf, grid, block, args, LDS64, stream);
        if (e != hipSuccess) return e;
        mark(DK_COOP);
    } else if (fused) {
        if (mut)
            hipLaunchKernelGGL(nicnes_decode_img_mut_kernel, dim3(1, member_count, nslabs), block, LDS32, stream, *p, *mh);
        else
            hipLaunchKernelGGL(nicnes_decode_img64_kernel, dim3(member_count, nslabs), block, LDS64, stream, *p);
        mark(DK_IMG);
        const dim3 grid(member_count, nslabs);
        if (p->sample_u) {                                  // sampled decode: the exact lse, then the draw's pick
            hipLaunchKernelGGL((nicnes_decode_steps_kernel<false, true>), grid, block, LDS64, stream, *p);
            mark(DK_STEPS);
        } else {
#if !DECODE_PROF
            if (mut && pairs)
                hipLaunchKernelGGL(nicnes_decode_steps_mut_kernel<true>, grid, block, LDS64, stream, *p, *mh);
            else if (mut)
                hipLaunchKernelGGL(nicnes_decode_steps_mut_kernel<false>, grid, block, LDS64, stream, *p, *mh);
            else if (pairs)
                hipLaunchKernelGGL(nicnes_decode_steps_kernel<true>, grid, block, LDS64, stream, *p);
            else
                hipLaunchKernelGGL(nicnes_decode_steps_kernel<false>, grid, block, LDS64, stream, *p);
            mark(DK_STEPS);
#else
            for (int t = -1; t <= p->T; ++t) {
                if (pairs)
                    hipLaunchKernelGGL(nicnes_decode_step_kernel<true>, grid, block, LDS64, stream, *p, t);
                else
                    hipLaunchKernelGGL(nicnes_decode_step_kernel<false>, grid, block, LDS64, stream, *p, t);
                mark(DK_STEP);
            }
#endif
        }
    } else {
        const int Sc = p->S < 4 ? p->S : 4;
        const dim3 gl(p->S, member_count, nslabs), gc(Sc, member_count, nslabs);
        if (p->G == 4) {
            hipLaunchKernelGGL(nicnes_decode_img_kernel<4>, gc, block, LDS32, stream, *p);
            mark(DK_IMG);
            for (int t = -1; t <= p->T; ++t) {
                if (t >= 1) {
                    if (pairs)
                        hipLaunchKernelGGL((nicnes_decode_logit_kernel<4, true>), gl, block, LDS64, stream, *p, t);
                    else
                        hipLaunchKernelGGL((nicnes_decode_logit_kernel<4, false>), gl, block, LDS64, stream, *p, t);
                    mark(DK_LOGIT);
                }
                hipLaunchKernelGGL(nicnes_decode_cell_kernel<4>, gc, block, LDS64, stream, *p, t);
                mark(DK_CELL);
            }
        } else if (p->S == 1 && !DECODE_PROF) {
            // 64-row slabs, one workgroup per member slab: every step in one launch
            hipLaunchKernelGGL(nicnes_decode_img_kernel<2>, gc, block, LDS32, stream, *p);
            mark(DK_IMG);
            if (pairs)
                hipLaunchKernelGGL(nicnes_decode_steps2_kernel<true>, gc, block, LDS_CELL2, stream, *p);
            else
                hipLaunchKernelGGL(nicnes_decode_steps2_kernel<false>, gc, block, LDS_CELL2, stream, *p);
            mark(DK_STEPS2);
        } else {
            hipLaunchKernelGGL(nicnes_decode_img_kernel<2>, gc, block, LDS32, stream, *p);
            mark(DK_IMG);
            for (int t = -1; t <= p->T; ++t) {
                if (t >= 1) {
                    if (pairs)
                        hipLaunchKernelGGL((nicnes_decode_logit_kernel<2, true>), gl, block, LDS64, stream, *p, t);
                    else
                        hipLaunchKernelGGL((nicnes_decode_logit_kernel<2, false>), gl, block, LDS64, stream, *p, t);
                    mark(DK_LOGIT);
                }
                hipLaunchKernelGGL(nicnes_decode_cell_kernel<2>, gc, block, LDS_CELL2, stream, *p, t);
                mark(DK_CELL);
            }
        }
    }
    if (n_launch) *n_launch = ne;
    return hipGetLastError();
}

// seq_logprobs as FCModel._sample leaves them when a member's rows span several slabs: the reference
// writes the greedy log-prob of EVERY row at every step until the whole batch has finished
// (nets.py:240-243), so a decode with log-prob output runs every slab to step T (no_exit) and this pass
// zeroes the steps after the batch's last finishing step (the reference's seq_logprobs start as zeros,
// nets.py:191). One workgroup per (member, sign) rollout of B rows.
__global__ __launch_bounds__(256) void nicnes_lp_batch_exit_kernel(const int32_t* seq, float* lp, int B, int T) {
    __shared__ int last;
    const size_t base = (size_t)blockIdx.x * B * T;
    if (threadIdx.x == 0) last = 0;
    __syncthreads();
    int mine = 0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        int f = T - 1;                                   // a row that never emits the end token: all T steps
        for (int t = 0; t < T; ++t)
            if (seq[base + (size_t)b * T + t] == 0) { f = t; break; }
        mine = max(mine, f);
    }
    atomicMax(&last, mine);
    __syncthreads();
    const int t_last = last;
    for (int i = threadIdx.x; i < B * T; i += blockDim.x)
        if (i % T > t_last) lp[base + i] = 0.f;
}

extern "C" hipError_t nicnes_launch_lp_batch_exit(const int32_t* seq, float* lp, int rollouts, int B, int T,
                                                  hipStream_t stream) {
    hipLaunchKernelGGL(nicnes_lp_batch_exit_kernel, dim3(rollouts), dim3(256), 0, stream, seq, lp, B, T);
    return hipGetLastError();
}

extern "C" size_t nicnes_decode_scratch_floats(int member_count, int row_waves_per_member) {
    return (size_t)member_count * row_waves_per_member * SCR_SLOTS * 64;
}
