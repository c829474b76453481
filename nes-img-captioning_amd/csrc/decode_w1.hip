// decode_w1.hip -- population greedy decode of the fc_caption LSTM, one wave per SIMD.
//
// Same arithmetic contract as decode_kernel.hip (bit-identical tokens; the oracle defines it):
//   NESWorker.fitness -> PolicyNet.evolve -> CaptPolicy.rollout -> FCModel._sample
//   (/root/reference/src/algorithm/nic_nes/nic_nes_worker.py:142-154,
//    /root/reference/src/algorithm/nets.py:101-113, /root/reference/src/captioning/nets.py:98-134,183-245)
//
// Layout: one workgroup = one member x one slab of <=128 images, 4 waves (one per SIMD, up to
// 512 registers each). Wave g decodes batch rows 32g..32g+31 for BOTH antithetic signs, so every
// MFMA stream has two independent accumulator chains (theta+delta, theta-delta) that share the
// activation-free A tile staging. The logit loop is hand scheduled: between consecutive MFMAs the
// wave issues a slice of the previous tile's epilogue (log-sum-exp + greedy records) and of the
// LDS store of the next staged tile; sched_barrier(0) pins that order (in-order issue then hides
// the VALU under the running MFMA).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nicnes_math.h"
#include "decode_kernel.h"

namespace w1 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int NT = 256;                 // threads per workgroup
constexpr int LDS_ROW = 132;            // 128 k + 4 pad
constexpr int SIGN_F = 32 * LDS_ROW;    // one sign's 32-row tile
constexpr int STAGE_F = 2 * SIGN_F + 64;
constexpr float LOG2E = 1.44269504088896340736f;
constexpr int SLOTS = 128 + 128 + 640;  // per lane: c(2x64) | h(2x64) | partials(2 x 20 x 16)

#define NEG_INF (-__builtin_inff())

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 ld4(rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ float ld1(rsrc_t r, uint32_t off, uint32_t soff = 0) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, (int)soff, 0));
}
__device__ __forceinline__ void st1(rsrc_t r, uint32_t off, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)off, (int)soff, 0);
}

// A 32-row x 128-k weight tile of a matrix viewed through (wr, zr): rows row0.. (row length ld),
// k window k0..k0+127, bias rows through (br, bzr). Rows outside the views read as 0.
struct Tile {
    rsrc_t wr, zr, br, bzr;
    int32_t row0, ld, k0;
    int32_t nvalid;      // bias rows >= nvalid get pad
    float pad;
};

struct Stage {
    f32x4 w[4], z[4];
    float bw, bz;
};

__device__ __forceinline__ void stage_load(const Tile& d, int tid, Stage& s) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int f = tid + NT * u, row = f >> 5, q = f & 31;
        const uint32_t off = 4u * (uint32_t)((d.row0 + row) * d.ld + d.k0 + 4 * q);
        s.w[u] = ld4(d.wr, off);
        s.z[u] = ld4(d.zr, off);
    }
    const uint32_t boff = 4u * (uint32_t)(d.row0 + (tid & 31));
    s.bw = ld1(d.br, boff);
    s.bz = ld1(d.bzr, boff);
}

__device__ __forceinline__ void store_pair(float* buf, int u, float sigma, int tid, const Stage& s) {
    const int f = tid + NT * u, row = f >> 5, q = f & 31;
    const int o = row * LDS_ROW + (q >> 3) * 32 + (q & 1) * 16 + 4 * ((q & 7) >> 1);
    const f32x4 delta = sigma * s.z[u];                                  // fp32(sigma z), nets.py:102
    *reinterpret_cast<f32x4*>(buf + o) = s.w[u] + delta;                 // nets.py:113
    *reinterpret_cast<f32x4*>(buf + SIGN_F + o) = s.w[u] - delta;        // nic_nes_worker.py:151
}

__device__ __forceinline__ void store_bias(float* buf, const Tile& d, float sigma, int tid, const Stage& s) {
    const int r = tid & 31, sg = (tid >> 5) & 1;   // each wave writes all 64 slots (same values)
    const float delta = sigma * s.bz;
    const float v = sg ? s.bw - delta : s.bw + delta;
    buf[2 * SIGN_F + 32 * sg + r] = r < d.nvalid ? v : d.pad;
}

__device__ __forceinline__ void stage_store(float* buf, const Tile& d, float sigma, int tid, const Stage& s) {
#pragma unroll
    for (int u = 0; u < 4; ++u) store_pair(buf, u, sigma, tid, s);
    store_bias(buf, d, sigma, tid, s);
}

__device__ __forceinline__ f32x16 bias_init(const float* bias, int hh) {
    f32x16 acc;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const f32x4 bb = *reinterpret_cast<const f32x4*>(bias + 8 * a + 4 * hh);
        acc[4 * a + 0] = bb[0]; acc[4 * a + 1] = bb[1]; acc[4 * a + 2] = bb[2]; acc[4 * a + 3] = bb[3];
    }
    return acc;
}

// two chains (+, -) over one staged tile: accp += W+ . Bp, accm += W- . Bm
__device__ __forceinline__ void mfma2(f32x16& accp, f32x16& accm, const float* buf, const float (&Bp)[64],
                                      const float (&Bm)[64], int lane) {
    const float* rp = buf + (lane & 31) * LDS_ROW + (lane >> 5) * 16;
    const float* rm = rp + SIGN_F;
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 ap[4], am[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            ap[c] = *reinterpret_cast<const f32x4*>(rp + T * 32 + 4 * c);
            am[c] = *reinterpret_cast<const f32x4*>(rm + T * 32 + 4 * c);
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            accp = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[jj >> 2][jj & 3], Bp[16 * T + jj], accp, 0, 0, 0);
            accm = __builtin_amdgcn_mfma_f32_32x32x2f32(am[jj >> 2][jj & 3], Bm[16 * T + jj], accm, 0, 0, 0);
        }
    }
}

// ---- greedy state of one row (log_softmax + first argmax, nets.py:202,208-209) ---------------
struct Row {
    float m, s;            // running max, sum exp(L - m)
    float r1v; int r1i;    // newest left-to-right record (running max, first index)
    float r0v; int r0i;    // previous record
    float ev;              // largest evicted record
    float x0, x1, x2, x3, x4, ml;   // epilogue scratch (tile max partials, m*log2e)
};

__device__ __forceinline__ void row_init(Row& st) {
    st.m = -1.0e30f; st.s = 0.f;
    st.r1v = NEG_INF; st.r1i = 0x7fffffff; st.r0v = NEG_INF; st.r0i = 0x7fffffff; st.ev = NEG_INF;
    st.x0 = st.x1 = st.x2 = st.x3 = st.x4 = 0.f; st.ml = 0.f;
}

// epilogue micro-op k (0..38) of one 32x32 tile; P holds vocab vbase + (r&3) + 8(r>>2)
__device__ __forceinline__ void epi_op(int k, Row& st, const f32x16& P, int vbase) {
    if (k == 0) st.x0 = fmaxf(fmaxf(P[0], P[1]), P[2]);
    else if (k == 1) st.x1 = fmaxf(fmaxf(P[3], P[4]), P[5]);
    else if (k == 2) st.x2 = fmaxf(fmaxf(P[6], P[7]), P[8]);
    else if (k == 3) st.x3 = fmaxf(fmaxf(P[9], P[10]), P[11]);
    else if (k == 4) st.x4 = fmaxf(fmaxf(P[12], P[13]), P[14]);
    else if (k == 5) st.x0 = fmaxf(fmaxf(st.x0, st.x1), st.x2);
    else if (k == 6) {
        const float tmax = fmaxf(fmaxf(st.x0, st.x3), fmaxf(st.x4, P[15]));
        const float mnew = fmaxf(st.m, tmax);
        st.s = st.s * __builtin_amdgcn_exp2f((st.m - mnew) * LOG2E);
        st.m = mnew;
        st.ml = mnew * LOG2E;
    } else if (k < 23) {
        st.s += __builtin_amdgcn_exp2f(__builtin_fmaf(P[k - 7], LOG2E, -st.ml));
    } else if (k < 39) {
        const int r = k - 23;
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

__device__ __forceinline__ void epilogue(Row& st, const f32x16& P, int vbase) {
#pragma unroll
    for (int k = 0; k < 39; ++k) epi_op(k, st, P, vbase);
}

// One logit tile, hand scheduled. 64 slots; slot j issues MFMA step j of both chains, then
// micro-ops [j*K/64, (j+1)*K/64) of: epilogue(prev+) 0..38, epilogue(prev-) 39..77, LDS store of
// the next tile 78..82. A fragments of sub-chunk T+1 are read at the first slot of T.
__device__ __forceinline__ void logit_tile(f32x16& accp, f32x16& accm, const float* buf, const float (&Bp)[64],
                                           const float (&Bm)[64], int lane, Row& sp, Row& sm, const f32x16& Pp,
                                           const f32x16& Pm, int vbase_prev, float* nbuf, const Tile& nd,
                                           float sigma, int tid, const Stage& sr) {
    constexpr int K = 83;
    const int hh = lane >> 5;
    const float* rp = buf + (lane & 31) * LDS_ROW + hh * 16;
    const float* rm = rp + SIGN_F;
    accp = bias_init(buf + 2 * SIGN_F, hh);
    accm = bias_init(buf + 2 * SIGN_F + 32, hh);
    f32x4 ap[4], am[4], np_[4], nm[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        ap[c] = *reinterpret_cast<const f32x4*>(rp + 4 * c);
        am[c] = *reinterpret_cast<const f32x4*>(rm + 4 * c);
    }
#pragma unroll
    for (int T = 0; T < 4; ++T) {
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int j = 16 * T + jj;
            if (jj == 0 && T < 3) {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    np_[c] = *reinterpret_cast<const f32x4*>(rp + (T + 1) * 32 + 4 * c);
                    nm[c] = *reinterpret_cast<const f32x4*>(rm + (T + 1) * 32 + 4 * c);
                }
            }
            accp = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[jj >> 2][jj & 3], Bp[j], accp, 0, 0, 0);
            accm = __builtin_amdgcn_mfma_f32_32x32x2f32(am[jj >> 2][jj & 3], Bm[j], accm, 0, 0, 0);
            const int k0 = (j * K) / 64, k1 = ((j + 1) * K) / 64;
#pragma unroll
            for (int k = k0; k < k1; ++k) {
                if (k < 39) epi_op(k, sp, Pp, vbase_prev);
                else if (k < 78) epi_op(k - 39, sm, Pm, vbase_prev);
                else if (k < 82) store_pair(nbuf, k - 78, sigma, tid, sr);
                else store_bias(nbuf, nd, sigma, tid, sr);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (T < 3) {
#pragma unroll
            for (int c = 0; c < 4; ++c) { ap[c] = np_[c]; am[c] = nm[c]; }
        }
    }
}

__device__ __forceinline__ bool in_window(float v, float m, float lse) { return ((v - m) - lse) == -lse; }

// greedy token of this lane's row from its state and its partner half (lane ^ 32)
__device__ __forceinline__ int finish_row(const Row& st, float& m, float& lse, bool& ovf) {
    const float m_o = __shfl_xor(st.m, 32), s_o = __shfl_xor(st.s, 32);
    m = fmaxf(st.m, m_o);
    const float stot = st.s * __builtin_amdgcn_exp2f((st.m - m) * LOG2E) + s_o * __builtin_amdgcn_exp2f((m_o - m) * LOG2E);
    lse = logf(stot);
    const float cv[4] = {st.r0v, st.r1v, __shfl_xor(st.r0v, 32), __shfl_xor(st.r1v, 32)};
    const int ci[4] = {st.r0i, st.r1i, __shfl_xor(st.r0i, 32), __shfl_xor(st.r1i, 32)};
    int tok = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (in_window(cv[k], m, lse) && ci[k] < tok) tok = ci[k];
    ovf = in_window(st.ev, m, lse) || in_window(__shfl_xor(st.ev, 32), m, lse);
    return tok;
}

__device__ __forceinline__ void exact_op(int& best, const f32x16& P, int vbase, float m, float lse) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int v = vbase + (r & 3) + 8 * (r >> 2);
        if (((P[r] - m) - lse) == -lse && v < best) best = v;
    }
}

}  // namespace w1

using namespace w1;

__global__ __launch_bounds__(NT) void nicnes_decode_w1_kernel(DecodeParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hh = lane >> 5, li = lane & 31;
    const int member = blockIdx.x, slab = blockIdx.y;
    const int b = slab * 128 + wave * 32 + li;
    const bool row_valid = b < p.B;
    const int bc = row_valid ? b : 0;
    const uint64_t nidx = p.noise_idx[member];
    const float sigma = p.sigma;
    const uint32_t D4 = 4u * (uint32_t)p.D;
    const float* th = p.theta;
    const float* nz = p.noise + nidx;

    const rsrc_t theta_r = make_rsrc(th, D4), noise_r = make_rsrc(nz, D4);
    const rsrc_t fc_r = make_rsrc(p.fc, 4u * (uint32_t)p.B * (uint32_t)p.F);
    float* wscr = p.scratch + ((size_t)(member * gridDim.y + slab) * 4 + wave) * (SLOTS * 64);
    const rsrc_t scr = make_rsrc(wscr, SLOTS * 64 * 4);
    const uint32_t lo = 4u * lane;
    // slot byte offsets (soffset): c[sg][64] | h[sg][64] | partial[sg][20*16]
#define C_SL(sg, s) (256u * (uint32_t)(64 * (sg) + (s)))
#define H_SL(sg, s) (256u * (uint32_t)(128 + 64 * (sg) + (s)))
#define P_SL(sg, s) (256u * (uint32_t)(256 + 320 * (sg) + (s)))

    // matrix views (each bounded to its own rows so padding reads are zero)
    const int V1 = p.V1, F = p.F;
    Tile timg{make_rsrc(th + p.off_img_w, 4u * 128u * F), make_rsrc(nz + p.off_img_w, 4u * 128u * F),
              make_rsrc(th + p.off_img_b, 4u * 128u), make_rsrc(nz + p.off_img_b, 4u * 128u), 0, F, 0, 32, 0.f};
    Tile ti2h{make_rsrc(th + p.off_i2h_w, 4u * 640u * 128u), make_rsrc(nz + p.off_i2h_w, 4u * 640u * 128u),
              make_rsrc(th + p.off_i2h_b, 4u * 640u), make_rsrc(nz + p.off_i2h_b, 4u * 640u), 0, 128, 0, 32, 0.f};
    Tile th2h{make_rsrc(th + p.off_h2h_w, 4u * 640u * 128u), make_rsrc(nz + p.off_h2h_w, 4u * 640u * 128u),
              make_rsrc(th + p.off_h2h_b, 4u * 640u), make_rsrc(nz + p.off_h2h_b, 4u * 640u), 0, 128, 0, 32, 0.f};
    Tile tlog{make_rsrc(th + p.off_log_w, 4u * 128u * V1), make_rsrc(nz + p.off_log_w, 4u * 128u * V1),
              make_rsrc(th + p.off_log_b, 4u * V1), make_rsrc(nz + p.off_log_b, 4u * V1), 0, 128, 0, 32, NEG_INF};

    float xp[64], xm[64], hp[64], hm[64];
    Stage sr;

    // ========== t = 0: x = img_embed(fc) (nets.py:194-195) =================================
    {
        f32x16 ap_[4], am_[4];
        const int nK = F >> 7, ntile = 4 * nK;
        auto tile = [&](int n) { Tile d = timg; d.row0 = 32 * (n & 3); d.k0 = 128 * (n >> 2); return d; };
        stage_load(tile(0), tid, sr);
        stage_store(lds, tile(0), sigma, tid, sr);
        __syncthreads();
        for (int kc = 0; kc < nK; ++kc) {
            const uint32_t frow = 4u * (uint32_t)(bc * F + 128 * kc + 4 * hh);
#pragma unroll
            for (int U = 0; U < 4; ++U) {
                const int n = kc * 4 + U;
                stage_load(tile(min(n + 1, ntile - 1)), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_F;
                if (kc == 0) {
                    ap_[U] = bias_init(buf + 2 * SIGN_F, hh);
                    am_[U] = bias_init(buf + 2 * SIGN_F + 32, hh);
                }
                const float* rp = buf + li * LDS_ROW + hh * 16;
#pragma unroll
                for (int T = 0; T < 4; ++T) {
                    f32x4 a0[4], a1[4], bq[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        a0[c] = *reinterpret_cast<const f32x4*>(rp + T * 32 + 4 * c);
                        a1[c] = *reinterpret_cast<const f32x4*>(rp + SIGN_F + T * 32 + 4 * c);
                        bq[c] = ld4(fc_r, frow + 4u * (32 * T + 8 * c));
                    }
#pragma unroll
                    for (int jj = 0; jj < 16; ++jj) {
                        ap_[U] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], bq[jj >> 2][jj & 3], ap_[U], 0, 0, 0);
                        am_[U] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], bq[jj >> 2][jj & 3], am_[U], 0, 0, 0);
                    }
                }
                stage_store(lds + ((n + 1) & 1) * STAGE_F, tile(min(n + 1, ntile - 1)), sigma, tid, sr);
                __syncthreads();
            }
        }
#pragma unroll
        for (int U = 0; U < 4; ++U)
#pragma unroll
            for (int r = 0; r < 16; ++r) { xp[16 * U + r] = ap_[U][r]; xm[16 * U + r] = am_[U][r]; }
    }

    int itp = 0, itm = 0;
    bool unp = true, unm = true;
    for (int t = 0; t <= p.T; ++t) {
        // ========== x = embed(it) (nets.py:196-199) ========================================
        if (t > 0) {
            const uint32_t ep = 4u * ((uint32_t)p.off_emb_w + (uint32_t)itp * 128u + 4u * hh);
            const uint32_t em = 4u * ((uint32_t)p.off_emb_w + (uint32_t)itm * 128u + 4u * hh);
#pragma unroll
            for (int T = 0; T < 4; ++T)
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const uint32_t o = 4u * (32 * T + 8 * a);
                    const f32x4 w0 = ld4(theta_r, ep + o), z0 = ld4(noise_r, ep + o);
                    const f32x4 w1 = ld4(theta_r, em + o), z1 = ld4(noise_r, em + o);
                    const f32x4 x0 = w0 + sigma * z0, x1 = w1 - sigma * z1;
#pragma unroll
                    for (int c = 0; c < 4; ++c) { xp[16 * T + 4 * a + c] = x0[c]; xm[16 * T + 4 * a + c] = x1[c]; }
                }
        }
        // ========== LSTM cell (nets.py:98-134): s = ((b_i2h + Wi.x) + b_h2h) + Wh.h ========
        {
            auto tile = [&](int n) {
                const int m = n % 20, U = m / 5, q = m % 5;
                Tile d = n < 20 ? ti2h : th2h;
                d.row0 = q * 128 + 32 * U;
                return d;
            };
            stage_load(tile(0), tid, sr);
            stage_store(lds, tile(0), sigma, tid, sr);
            __syncthreads();
            for (int n = 0; n < 20; ++n) {                       // i2h partials (h not live)
                stage_load(tile(n + 1), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_F;
                f32x16 accp = bias_init(buf + 2 * SIGN_F, hh), accm = bias_init(buf + 2 * SIGN_F + 32, hh);
                mfma2(accp, accm, buf, xp, xm, lane);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    st1(scr, lo, P_SL(0, 16 * n + r), accp[r]);
                    st1(scr, lo, P_SL(1, 16 * n + r), accm[r]);
                }
                stage_store(lds + ((n + 1) & 1) * STAGE_F, tile(n + 1), sigma, tid, sr);
                __syncthreads();
            }
#pragma unroll
            for (int i = 0; i < 64; ++i) {
                hp[i] = (t == 0) ? 0.f : ld1(scr, lo, H_SL(0, i));
                hm[i] = (t == 0) ? 0.f : ld1(scr, lo, H_SL(1, i));
            }
            for (int n = 20; n < 40; ++n) {                      // + b_h2h + Wh.h (x not live)
                stage_load(tile(min(n + 1, 39)), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_F;
                const int m = n - 20;
                f32x16 accp, accm;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    accp[r] = ld1(scr, lo, P_SL(0, 16 * m + r));
                    accm[r] = ld1(scr, lo, P_SL(1, 16 * m + r));
                }
                accp = accp + bias_init(buf + 2 * SIGN_F, hh);
                accm = accm + bias_init(buf + 2 * SIGN_F + 32, hh);
                if (t > 0) mfma2(accp, accm, buf, hp, hm, lane);   // h = 0 at t = 0
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    st1(scr, lo, P_SL(0, 16 * m + r), accp[r]);
                    st1(scr, lo, P_SL(1, 16 * m + r), accm[r]);
                }
                stage_store(lds + ((n + 1) & 1) * STAGE_F, tile(min(n + 1, 39)), sigma, tid, sr);
                __syncthreads();
            }
            for (int sg = 0; sg < 2; ++sg)
                for (int U = 0; U < 4; ++U) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const uint32_t g = 16 * (5 * U) + r;
                        const float s0 = ld1(scr, lo, P_SL(sg, g)), s1 = ld1(scr, lo, P_SL(sg, g + 16));
                        const float s2 = ld1(scr, lo, P_SL(sg, g + 32)), s3 = ld1(scr, lo, P_SL(sg, g + 48));
                        const float s4 = ld1(scr, lo, P_SL(sg, g + 64));
                        const float cold = (t == 0) ? 0.f : ld1(scr, lo, C_SL(sg, 16 * U + r));
                        float cn, hn;
                        nn_lstm_cell(s0, s1, s2, s3, s4, cold, &cn, &hn);
                        st1(scr, lo, C_SL(sg, 16 * U + r), cn);
                        st1(scr, lo, H_SL(sg, 16 * U + r), hn);
                    }
                }
#pragma unroll
            for (int i = 0; i < 64; ++i) {
                hp[i] = ld1(scr, lo, H_SL(0, i));
                hm[i] = ld1(scr, lo, H_SL(1, i));
            }
        }
        if (t == 0) continue;           // t=0 logits are discarded (nets.py:205-206)

        // ========== logits + log_softmax + greedy argmax (nets.py:202,208-209) =============
        const int nvt = (V1 + 31) >> 5;
        auto ltile = [&](int n) { Tile d = tlog; d.row0 = 32 * n; d.nvalid = V1 - 32 * n; return d; };
        Row sp, sm;
        row_init(sp);
        row_init(sm);
        stage_load(ltile(0), tid, sr);
        stage_store(lds, ltile(0), sigma, tid, sr);
        __syncthreads();
        f32x16 Pp, Pm;
#pragma unroll
        for (int r = 0; r < 16; ++r) { Pp[r] = NEG_INF; Pm[r] = NEG_INF; }
        for (int n = 0; n < nvt; ++n) {
            const Tile nd = ltile(min(n + 1, nvt - 1));
            stage_load(nd, tid, sr);
            f32x16 accp, accm;
            logit_tile(accp, accm, lds + (n & 1) * STAGE_F, hp, hm, lane, sp, sm, Pp, Pm, 32 * (n - 1) + 4 * hh,
                       lds + ((n + 1) & 1) * STAGE_F, nd, sigma, tid, sr);
            __syncthreads();
            Pp = accp;
            Pm = accm;
        }
        epilogue(sp, Pp, 32 * (nvt - 1) + 4 * hh);
        epilogue(sm, Pm, 32 * (nvt - 1) + 4 * hh);
        float mp, lsep, mm, lsem;
        bool ovp, ovm;
        int tokp = finish_row(sp, mp, lsep, ovp);
        int tokm = finish_row(sm, mm, lsem, ovm);
        if (__syncthreads_or((ovp || ovm) ? 1 : 0)) {
            // rare: more records than tracked fall in the tie window -> exact second pass
            int bp = 0x7fffffff, bm = 0x7fffffff;
            stage_load(ltile(0), tid, sr);
            stage_store(lds, ltile(0), sigma, tid, sr);
            __syncthreads();
            for (int n = 0; n < nvt; ++n) {
                stage_load(ltile(min(n + 1, nvt - 1)), tid, sr);
                const float* buf = lds + (n & 1) * STAGE_F;
                f32x16 accp = bias_init(buf + 2 * SIGN_F, hh), accm = bias_init(buf + 2 * SIGN_F + 32, hh);
                mfma2(accp, accm, buf, hp, hm, lane);
                exact_op(bp, accp, 32 * n + 4 * hh, mp, lsep);
                exact_op(bm, accm, 32 * n + 4 * hh, mm, lsem);
                stage_store(lds + ((n + 1) & 1) * STAGE_F, ltile(min(n + 1, nvt - 1)), sigma, tid, sr);
                __syncthreads();
            }
            tokp = min(bp, __shfl_xor(bp, 32));
            tokm = min(bm, __shfl_xor(bm, 32));
            if (tid == 0) atomicAdd(p.stats + 0, 1);
        }
        if (tokp >= V1) tokp = 0;       // only when every logit is NaN
        if (tokm >= V1) tokm = 0;
        // finished mask (nets.py:236-243)
        unp = unp && (tokp > 0);
        unm = unm && (tokm > 0);
        itp = unp ? tokp : 0;
        itm = unm ? tokm : 0;
        if (hh == 0 && row_valid) {
            p.seq[(((size_t)member * 2 + 0) * p.B + b) * p.T + (t - 1)] = itp;
            p.seq[(((size_t)member * 2 + 1) * p.B + b) * p.T + (t - 1)] = itm;
        }
        if (t == p.T) break;
        if (!__syncthreads_or(((unp || unm) && row_valid) ? 1 : 0)) break;
    }
#undef C_SL
#undef H_SL
#undef P_SL
}

extern "C" hipError_t nicnes_launch_decode_w1(const DecodeParams* p, int member_count, int nslabs, hipStream_t stream) {
    const size_t lds_bytes = (size_t)(2 * STAGE_F) * sizeof(float);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)nicnes_decode_w1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds_bytes);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(nicnes_decode_w1_kernel, dim3(member_count, nslabs), dim3(NT), lds_bytes, stream, *p);
    return hipGetLastError();
}

extern "C" size_t nicnes_decode_w1_scratch_floats(int member_count, int nslabs) {
    return (size_t)member_count * nslabs * 4 * SLOTS * 64;
}
