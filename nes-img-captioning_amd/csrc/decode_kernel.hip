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
        const int rc = row < d.nvalid ? row : d.nvalid - 1;          // clamp, zero after the load
        const uint32_t off = 4u * (d.w_off + (uint32_t)((d.row0 + rc) * d.ld + d.k0 + 4 * q));
        const f32x4 w = ld4(theta_r, off), z = ld4(noise_r, off);
        const bool ok = row < d.nvalid;
        s.w[u] = ok ? w : f32x4{0.f, 0.f, 0.f, 0.f};
        s.z[u] = ok ? z : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (tid < 32) {
        const int rc = tid < d.nvalid ? tid : 0;
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
    if (tid < 32) {
        const float delta = sigma * s.bz;
        const bool ok = tid < d.nvalid;
        buf[2 * SIGN_FLOATS + tid] = ok ? s.bw + delta : d.pad_bias;
        buf[2 * SIGN_FLOATS + 32 + tid] = ok ? s.bw - delta : d.pad_bias;
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
    st.m = NEG_INF; st.s = 0.f;
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
    if (tmax > st.m) {
        st.s = (st.m == NEG_INF) ? 0.f : st.s * __builtin_amdgcn_exp2f((st.m - tmax) * LOG2E);
        st.m = tmax;
    }
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
    const uint32_t lo = 4u * lane;
#define C_SLOT(s) (4u * 64u * (uint32_t)(s))
#define H_SLOT(s) (4u * 64u * (uint32_t)(64 + (s)))
#define P_SLOT(s) (4u * 64u * (uint32_t)(128 + (s)))

    float xB[64], hB[64];
    StageRegs sr;

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
        // i2h products and park the 20 partial gate tiles in lane-private scratch; tiles 20..39
        // finish them with h2h, so x and h are never live in registers together.
        {
            const int ntile = 40;
            auto desc = [&](int n) {
                const int which = n >= 20, m = n - 20 * which, U = m / 5, qi = m % 5;
                const int q = qi < 2 ? 3 + qi : qi - 2;        // (3,4,0,1,2): g1, g2, in, forget, out
                TileDesc d;
                d.w_off = (uint32_t)(which ? p.off_h2h_w : p.off_i2h_w); d.ld = 128; d.row0 = q * 128 + 32 * U;
                d.nvalid = 32; d.k0 = 0; d.b_off = (uint32_t)(which ? p.off_h2h_b : p.off_i2h_b); d.pad_bias = 0.f;
                return d;
            };
            float g[16];      // holds max(g1,g2), then i*g, then c'
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
            // pass 2: + b_h2h + Wh.h, then the cell elementwise (x not live)
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = (t == 0) ? 0.f : ld1(scr_r, lo, H_SLOT(i));
            for (int n = 20; n < ntile; ++n) {
                if (n + 1 < ntile) stage_load(theta_r, noise_r, desc(n + 1), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_FLOATS;
                const int m = n - 20, U = m / 5, qi = m % 5;
                const f32x16 bias = bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh);
                f32x16 acc;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = ld1(scr_r, lo, P_SLOT(16 * m + r));
                acc = acc + bias;
                if (t > 0) acc = mfma_tile(acc, buf + sgn * SIGN_FLOATS, hB, lane);   // h = 0 at t = 0
                if (qi == 0) {                                              // q = 3: g1
#pragma unroll
                    for (int r = 0; r < 16; ++r) g[r] = acc[r];
                } else if (qi == 1) {                                       // q = 4: max(g1, g2)
#pragma unroll
                    for (int r = 0; r < 16; ++r) g[r] = g[r] > acc[r] ? g[r] : acc[r];
                } else if (qi == 2) {                                       // q = 0: i*g
#pragma unroll
                    for (int r = 0; r < 16; ++r) g[r] = nn_sigmoidf(acc[r]) * g[r];
                } else if (qi == 3) {                                       // q = 1: c' = f*c + i*g
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float cold = (t == 0) ? 0.f : ld1(scr_r, lo, C_SLOT(16 * U + r));
                        const float fc_ = nn_sigmoidf(acc[r]) * cold;
                        g[r] = fc_ + g[r];
                        st1(scr_r, lo, C_SLOT(16 * U + r), g[r]);
                    }
                } else {                                                    // q = 2: h' = o*tanh(c')
#pragma unroll
                    for (int r = 0; r < 16; ++r) st1(scr_r, lo, H_SLOT(16 * U + r), nn_sigmoidf(acc[r]) * nn_tanhf(g[r]));
                }
                if (n + 1 < ntile) stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), sigma, tid, sr);
                __syncthreads();
            }
#pragma unroll
            for (int i = 0; i < 64; ++i) hB[i] = ld1(scr_r, lo, H_SLOT(i));
        }
        if (t == 0) continue;            // t=0 logits are discarded (nets.py:205-206)

        // ========== logits + log_softmax + greedy argmax (nets.py:202,208-209) ==============
        const int nvt = (p.V1 + 31) >> 5;
        auto desc = [&](int n) {
            TileDesc d;
            d.w_off = (uint32_t)p.off_log_w; d.ld = 128; d.row0 = 32 * n; d.nvalid = min(32, p.V1 - 32 * n); d.k0 = 0;
            d.b_off = (uint32_t)p.off_log_b; d.pad_bias = NEG_INF;
            return d;
        };
        RowState st;
        row_state_init(st);
        stage_load(theta_r, noise_r, desc(0), tid, sr);
        stage_store(lds, desc(0), sigma, tid, sr);
        __syncthreads();
        for (int n = 0; n < nvt; ++n) {
            if (n + 1 < nvt) stage_load(theta_r, noise_r, desc(n + 1), tid, sr);
            const float* buf = lds + (n & 1) * STAGE_FLOATS;
            const f32x16 acc = mfma_tile(bias_init(buf + 2 * SIGN_FLOATS + 32 * sgn, hh), buf + sgn * SIGN_FLOATS, hB, lane);
            if (n + 1 < nvt) stage_store(lds + ((n + 1) & 1) * STAGE_FLOATS, desc(n + 1), sigma, tid, sr);
            logit_epilogue(st, acc, 32 * n + 4 * hh);
            __syncthreads();
        }
        // merge the two lane halves that share this batch row
        const float m_o = __shfl_xor(st.m, 32);
        const float s_o = __shfl_xor(st.s, 32);
        const float m = fmaxf(st.m, m_o);
        const float stot = st.s * __builtin_amdgcn_exp2f((st.m - m) * LOG2E) + s_o * __builtin_amdgcn_exp2f((m_o - m) * LOG2E);
        const float lse = logf(stot);
        int tok = 0x7fffffff;
        {
            const float cv[4] = {st.r0v, st.r1v, __shfl_xor(st.r0v, 32), __shfl_xor(st.r1v, 32)};
            const int ci[4] = {st.r0i, st.r1i, __shfl_xor(st.r0i, 32), __shfl_xor(st.r1i, 32)};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (in_window(cv[k], m, lse) && ci[k] < tok) tok = ci[k];
        }
        const bool ovf = in_window(st.ev, m, lse) || in_window(__shfl_xor(st.ev, 32), m, lse);
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
        // finished mask (nets.py:236-243)
        unfinished = unfinished && (tok > 0);
        it = unfinished ? tok : 0;
        if (hh == 0 && row_valid) p.seq[(((size_t)member * 2 + sgn) * p.B + b) * p.T + (t - 1)] = it;
        if (t == p.T) break;
        if (!__syncthreads_or((unfinished && row_valid) ? 1 : 0)) break;
    }
#undef C_SLOT
#undef H_SLOT
#undef P_SLOT
}

extern "C" hipError_t nicnes_launch_decode(const DecodeParams* p, int member_count, int nslabs, hipStream_t stream) {
    const size_t lds_bytes = (size_t)(2 * STAGE_FLOATS) * sizeof(float);
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
