// sensitivity.hip -- the SM-G-SUM sensitivity of safe mutations on the GPU, hand-written MFMA kernels.
//
// Replaces the per-task host computation of
//   Sensitivity._calc_sum_sensitivity (/root/reference/src/algorithm/safe_mutations.py:93-117) on
//   CaptionModel.forward_for_sensitivity (/root/reference/src/captioning/nets.py:22-70):
// O = [Bs, K] grouped log-prob norms after L = 5 greedy steps (vocabulary zero-padded to a multiple of
// split = 100, K groups, each reduced to its 2-norm); the reference runs K backward passes, one per
// column k of O summed over the batch, stacks the K gradients into a [K, D] Jacobian J and returns
// s_j = sqrt(sum_k J[k, j]^2) / Bs (safe_mutations.py:112-117).
//
// Here the K backward passes run at once and the Jacobian is never written: every weight gradient is a
// product G_k = A_k^T B over the batch (and the cells), and sq_tile (below) forms G_k tile by tile on
// fp32 MFMA and adds G_k^2 into its registers, k after k; only sum_k G_k^2 leaves the kernel (a few
// k-range partials, summed in a fixed order by sens_finish). The plain products of the forward and of
// the backward recurrence run on the same tile kernel (gemm mode). Structure used:
//   * the output seed of group k, dZ_k = d(sum_b O[b, k]) / d logits, is own_k - p * S_k (sens_seed):
//     own_k nonzero only inside group k. The logit.weight factor reads dZ from (lp, p, inv_g, S) as it
//     stages it (DzA, nothing [K, Bs, V] is stored), and dH_L = dZ_k Wl is inv_g (lp Wl restricted to
//     the group) - S_k (p Wl): one [Bs, V] x [V, R] product instead of K of them (sens_dh_logit);
//   * the embedding rows gather dX of the cells whose token is that row: a deterministic per-token sum
//     (sens_emb_sq), no atomics, so the vector is the same in every process.
// The forward picks its own greedy tokens (tok_internal: the logits of steps 1..L-1 in the decode's k order, the
// first id at the log_softmax maximum, fed back unmasked as forward_for_sensitivity does; before r04 a separate
// split-path decode of theta supplied them, ~1 ms per vector). Agreement with the reference's vector is to a stated tolerance (fp32 sums in
// another order), not bit for bit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "sensitivity.h"
#include "../../include/nicnes_math.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

// ---- the tile kernel -----------------------------------------------------------------------------
// C[m, n] = sum_r A(k, m, r) B(k, r, n) over a 64 x 64 tile per workgroup of 4 waves (wave w: rows
// 32 (w >> 1), columns 32 (w & 1) of the tile, one v_mfma_f32_32x32x2_f32 accumulator), the reduction
// staged through LDS in chunks of 16, the next chunk's global loads issued before this chunk's MFMAs.
// gemm mode: k = blockIdx.z (a batch), C written (beta 0) or accumulated (beta 1).
// sq mode: k runs over [k0, k1) of range blockIdx.z, C_k is formed for each k and C_k^2 accumulated;
// out[z][m, n] = sum over the range (sq partials, summed over ranges by sens_finish).
#define TM 64
#define TN 64
#define TR 32
#define LDS_P (TM + 1)

struct Strided {             // element (k, m, r) at p + k sk + m sm + r sr
    const float* p;
    int64_t sk, sm, sr;
    __device__ __forceinline__ float operator()(int k, int m, int r) const {
        return p[(int64_t)k * sk + (int64_t)m * sm + (int64_t)r * sr];
    }
    __device__ __forceinline__ bool m_unit() const { return sm == 1; }
};

// dZ_k[b, v] = [v in group k] lp[b, v] inv_g[b, k] - p[b, v] S[b, k] as A(k, m = v, r = b) (sens_seed's seed)
struct DzA {
    const float* lp;         // [Bs, V]
    const float* pr;         // [Bs, V] exp(lp)
    const float* ig;         // [Bs, K] 1 / |lp group k| (0 for an all-padding group)
    const float* S;          // [Bs, K] sum over group k of lp inv_g
    int V, K, split;
    __device__ __forceinline__ float operator()(int k, int v, int b) const {
        const int64_t o = (int64_t)b * V + v;
        const float own = (v / split == k) ? lp[o] * ig[b * K + k] : 0.f;
        return own - pr[o] * S[b * K + k];
    }
    __device__ __forceinline__ bool m_unit() const { return true; }
};

struct TileArgs {
    int M, N, R;             // tile problem: C [M, N], reduction R
    const float* B;          // element (k, r, n) at B + k sBk + r sBr + n sBn
    int64_t sBk, sBr, sBn;
    float* C;                // gemm: (k, m, n) at C + k sCk + m sCm + n sCn; sq: out + z sCk + m sCm + n sCn
    int64_t sCk, sCm, sCn;
    int beta;                // gemm: 1 accumulate into C
    int k0, kpr, k_end;      // sq: range z covers k in [k0 + z kpr, min(k0 + (z + 1) kpr, k_end))
    const float* bias;       // gemm (nullable): every column's chain starts from bias[n] (and beta is 0)
    int kperm;               // 1: the reduction visits r in the reference's fma-chain order (nn_kperm)
};

// nn_kperm inside a 16-aligned chunk: chain position p -> r (the 32-wide pattern keeps each half in its 16)
__device__ __forceinline__ int perm16(int p) { const int j = p >> 1; return (j & 3) + 8 * (j >> 2) + 4 * (p & 1); }

// chunk [r0, r0 + TR) of A (TM rows from m0) and B (TN columns from n0) into registers: NPT + NPT values per
// thread, the 256 threads laid along the operand's unit-stride dimension; with kperm, chain position p of the
// chunk holds r0 + (p & 16) + perm16(p & 15)
#define NPT (TM * TR / 256)
__device__ __forceinline__ int chunk_r(const TileArgs& t, int p) { return t.kperm ? (p & 16) + perm16(p & 15) : p; }

template <class AOp>
__device__ __forceinline__ void tile_load(const AOp& A, const TileArgs& t, int k, int m0, int n0, int r0, float (&ra)[NPT],
                                          float (&rb)[NPT]) {
    const int tid = threadIdx.x;
    const bool am = A.m_unit();
#pragma unroll
    for (int e = 0; e < NPT; ++e) {
        const int i = tid + 256 * e;
        const int m = am ? (i & (TM - 1)) : (i / TR), p = am ? (i / TM) : (i & (TR - 1));
        const int gm = m0 + m, gr = r0 + chunk_r(t, p);
        ra[e] = (gm < t.M && gr < t.R) ? A(k, gm, gr) : 0.f;
    }
    const bool bn = t.sBn == 1;
#pragma unroll
    for (int e = 0; e < NPT; ++e) {
        const int i = tid + 256 * e;
        const int n = bn ? (i & (TN - 1)) : (i / TR), p = bn ? (i / TN) : (i & (TR - 1));
        const int gn = n0 + n, gr = r0 + chunk_r(t, p);
        rb[e] = (gn < t.N && gr < t.R) ? t.B[(int64_t)k * t.sBk + (int64_t)gr * t.sBr + (int64_t)gn * t.sBn] : 0.f;
    }
}

template <class AOp>
__device__ __forceinline__ void tile_store(const AOp& A, const TileArgs& t, float* As, float* Bs, const float (&ra)[NPT],
                                           const float (&rb)[NPT]) {
    const int tid = threadIdx.x;
    const bool am = A.m_unit(), bn = t.sBn == 1;
#pragma unroll
    for (int e = 0; e < NPT; ++e) {
        const int i = tid + 256 * e;
        const int m = am ? (i & (TM - 1)) : (i / TR), p = am ? (i / TM) : (i & (TR - 1));
        As[p * LDS_P + m] = ra[e];
        const int n = bn ? (i & (TN - 1)) : (i / TR), q = bn ? (i / TN) : (i & (TR - 1));
        Bs[q * LDS_P + n] = rb[e];
    }
}

// acc += A(k)[tile rows, :] B(k)[:, tile columns] for this wave's 32 x 32 block
template <class AOp>
__device__ __forceinline__ void tile_product(const AOp& A, const TileArgs& t, int k, int m0, int n0, float* As, float* Bs,
                                             f32x16& acc) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = 32 * (w >> 1), wn = 32 * (w & 1), kh = lane >> 5, li = lane & 31;
    float ra[NPT], rb[NPT];
    tile_load(A, t, k, m0, n0, 0, ra, rb);
    for (int r0 = 0; r0 < t.R; r0 += TR) {
        __syncthreads();                                     // the previous chunk has been read
        tile_store(A, t, As, Bs, ra, rb);
        __syncthreads();
        if (r0 + TR < t.R) tile_load(A, t, k, m0, n0, r0 + TR, ra, rb);
#pragma unroll
        for (int j = 0; j < TR / 2; ++j) {
            const float a = As[(2 * j + kh) * LDS_P + wm + li];
            const float b = Bs[(2 * j + kh) * LDS_P + wn + li];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
    }
}

template <class AOp, bool SQ>
__global__ __launch_bounds__(256) void sens_tile(AOp A, TileArgs t) {
    __shared__ float As[TR * LDS_P], Bs[TR * LDS_P];
    const int m0 = blockIdx.x * TM, n0 = blockIdx.y * TN, z = blockIdx.z;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = 32 * (w >> 1), wn = 32 * (w & 1), kh = lane >> 5, li = lane & 31;
    f32x16 acc, sq;
#pragma unroll
    for (int i = 0; i < 16; ++i) sq[i] = 0.f;
    const int ka = SQ ? t.k0 + z * t.kpr : z, kb = SQ ? min(ka + t.kpr, t.k_end) : z + 1;
    // the bias the gemm's chains start from (the reference's addmm order: nicnes_math.h nn_kperm)
    const float b0 = (!SQ && t.bias && n0 + wn + li < t.N) ? t.bias[n0 + wn + li] : 0.f;
    for (int k = ka; k < kb; ++k) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = b0;
        tile_product(A, t, k, m0, n0, As, Bs, acc);
        if (SQ) {
#pragma unroll
            for (int i = 0; i < 16; ++i) sq[i] += acc[i] * acc[i];
        }
    }
    // accumulator element i of lane l: row 8 (i >> 2) + 4 (l >> 5) + (i & 3), column l & 31
    const int n = n0 + wn + li;
    if (n >= t.N) return;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int m = m0 + wm + 8 * (i >> 2) + 4 * kh + (i & 3);
        if (m >= t.M) continue;
        float* c = t.C + (int64_t)z * t.sCk + (int64_t)m * t.sCm + (int64_t)n * t.sCn;
        if (SQ) *c = sq[i];
        else *c = t.beta ? *c + acc[i] : acc[i];
    }
}

// ---- elementwise and small kernels ------------------------------------------------------------------
// X[b, :] = emb[token, :], token = tok[b * stride + col] (col < 0: the BOS token 0)
__global__ void sens_embed_gather(float* X, const float* emb, const int32_t* tok, int stride, int col, int Bs, int E) {
    const int b = blockIdx.x, e = threadIdx.x;
    if (b >= Bs || e >= E) return;
    const int t = col < 0 ? 0 : tok[(int64_t)b * stride + col];
    X[(int64_t)b * E + e] = emb[(int64_t)t * E + e];
}

// LSTMCore without vbn / layer norm (nets.py:98-134): S = [Bs, 5R] gate sums (i, f, o, g1, g2) = the i2h chain
// (in S) + the h2h chain (Sh, nullable: the bias alone, h = 0), then the cell as the decode runs it (nn_lstm_cell)
__global__ void sens_cell_fwd(float* S, const float* Sh, const float* bh, const float* Cprev, float* C, float* H, int Bs,
                              int R) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Bs * R) return;
    const int64_t b = i / R;
    const int r = (int)(i % R);
    float* s = S + b * 5 * R;
#pragma unroll
    for (int q = 0; q < 5; ++q) s[q * R + r] = s[q * R + r] + (Sh ? Sh[b * 5 * R + q * R + r] : bh[q * R + r]);
    float cn, hn;
    nn_lstm_cell(s[r], s[R + r], s[2 * R + r], s[3 * R + r], s[4 * R + r], Cprev ? Cprev[i] : 0.f, &cn, &hn);
    C[i] = cn;
    H[i] = hn;
}

// one block per row: LP = log_softmax(Z) (nets.py:202), P = exp(LP)
__global__ void sens_logsoftmax(const float* Z, float* LP, float* P, int V) {
    __shared__ float red[256];
    const float* z = Z + (int64_t)blockIdx.x * V;
    float* lp = LP + (int64_t)blockIdx.x * V;
    float* pr = P + (int64_t)blockIdx.x * V;
    float m = -INFINITY;
    for (int v = threadIdx.x; v < V; v += blockDim.x) m = fmaxf(m, z[v]);
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    m = red[0];
    __syncthreads();
    float s = 0.f;
    for (int v = threadIdx.x; v < V; v += blockDim.x) s += expf(z[v] - m);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const float lse = logf(red[0]);
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
        const float l = (z[v] - m) - lse;
        lp[v] = l;
        pr[v] = expf(l);
    }
}

// one block per row: the greedy token of a forward step, torch.max(log_softmax(Z)) (nets.py:61-63): the first id
// whose log-prob (z - m) - lse equals the maximum, -lse; m, the exp-sum and lse as sens_logsoftmax forms them
__global__ void sens_greedy(const float* Z, int V, int32_t* tok, int stride, int col) {
    __shared__ float red[256];
    __shared__ int redi[256];
    const float* z = Z + (int64_t)blockIdx.x * V;
    float m = -INFINITY;
    for (int v = threadIdx.x; v < V; v += blockDim.x) m = fmaxf(m, z[v]);
    red[threadIdx.x] = m;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    m = red[0];
    __syncthreads();
    float s = 0.f;
    for (int v = threadIdx.x; v < V; v += blockDim.x) s += expf(z[v] - m);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const float lse = logf(red[0]);
    int best = 0x7fffffff;
    for (int v = threadIdx.x; v < V; v += blockDim.x)
        if (((z[v] - m) - lse) == -lse) { best = v; break; }
    redi[threadIdx.x] = best;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) redi[threadIdx.x] = min(redi[threadIdx.x], redi[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) tok[(int64_t)blockIdx.x * stride + col] = redi[0] < V ? redi[0] : 0;
}

// block (b, k): the seed of output column k for row b through the 2-norm and log_softmax,
// dZ[k, b, v] = [v in group k] lp[b, v] / g_bk - exp(lp[b, v]) * sum_{u in group k} lp[b, u] / g_bk,
// kept as inv_g[b, k] = 1 / g_bk (0 for an all-padding group) and S[b, k] (DzA forms dZ from them)
__global__ void sens_seed(const float* LP, float* IG, float* Sg, int Bs, int V, int K, int split) {
    __shared__ float red[2][128];
    const int b = blockIdx.x, k = blockIdx.y;
    const float* lp = LP + (int64_t)b * V;
    const int v0 = k * split;
    float sq = 0.f, sm = 0.f;
    for (int u = threadIdx.x; u < split; u += blockDim.x) {
        const float x = (v0 + u < V) ? lp[v0 + u] : 0.f;          // the zero padding of extended_lp
        sq += x * x;
        sm += x;
    }
    red[0][threadIdx.x] = sq;
    red[1][threadIdx.x] = sm;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float g = sqrtf(red[0][0]);
        const float inv = g > 0.f ? 1.f / g : 0.f;
        IG[b * K + k] = inv;
        Sg[b * K + k] = red[1][0] * inv;
    }
}

// dH_L[k, b, r] = sum_v dZ[k, b, v] Wl[v, r] = inv_g[b, k] sum_{v in group k} lp[b, v] Wl[v, r] - S[b, k] PW[b, r],
// PW = p Wl (one product for every k). Block (b, k), thread r.
__global__ void sens_dh_logit(const float* LP, const float* IG, const float* Sg, const float* PW, const float* Wl,
                              float* dH, int Bs, int V, int K, int R, int split) {
    const int b = blockIdx.x, k = blockIdx.y, r = threadIdx.x;
    if (r >= R) return;
    const float* lp = LP + (int64_t)b * V;
    const int v0 = k * split, v1 = min(v0 + split, V);
    float own = 0.f;
    for (int v = v0; v < v1; ++v) own += lp[v] * Wl[(int64_t)v * R + r];
    dH[((int64_t)k * Bs + b) * R + r] = own * IG[b * K + k] - Sg[b * K + k] * PW[(int64_t)b * R + r];
}

// LSTM cell backward for the K seeds at once: dH, dC [K, Bs, R] -> dS of cell i (dS_all [K][L + 1][Bs][5R]),
// dC <- d c_prev. torch.max(a, b) (nets.py:121) splits the gradient of an exact tie in halves (aten maximum
// backward).
__global__ void sens_cell_bwd(const float* dH, float* dC, const float* S, const float* C, const float* Cprev,
                              float* dS, int64_t sdk, int K, int Bs, int R) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)K * Bs * R) return;
    const int64_t kb = i / R;                                    // k * Bs + b
    const int r = (int)(i % R);
    const int64_t b = kb % Bs, k = kb / Bs;
    const float* s = S + b * 5 * R;
    // the forward's activations as it computed them (nn_lstm_cell)
    const float ig = nn_sigmoidf(s[r]), fg = nn_sigmoidf(s[R + r]), og = nn_sigmoidf(s[2 * R + r]);
    const float g1 = s[3 * R + r], g2 = s[4 * R + r], g = g1 > g2 ? g1 : g2;
    const float c = C[b * R + r], cp = Cprev ? Cprev[b * R + r] : 0.f;
    const float th = nn_tanhf(c);
    const float dh = dH[i];
    const float dc = dC[i] + dh * og * (1.f - th * th);
    const float dog = dh * th;
    float* d = dS + k * sdk + b * 5 * R;
    d[r] = dc * g * ig * (1.f - ig);
    d[R + r] = dc * cp * fg * (1.f - fg);
    d[2 * R + r] = dog * og * (1.f - og);
    const float dg = dc * ig;
    d[3 * R + r] = g1 > g2 ? dg : (g1 == g2 ? 0.5f * dg : 0.f);
    d[4 * R + r] = g2 > g1 ? dg : (g1 == g2 ? 0.5f * dg : 0.f);
    dC[i] = dc * fg;
}

// sums[k][c] = sum_{r < rows} X[k sk + r sr + c] (a bias gradient for each of the K seeds): block (64 columns, k),
// 4 row groups summed in a fixed order
__global__ __launch_bounds__(256) void sens_colsum_k(const float* X, int rows, int cols, int64_t sr, int64_t sk,
                                                     float* sums) {
    __shared__ float red[4][64];
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6, k = blockIdx.y;
    const int c = blockIdx.x * 64 + cl;
    float s = 0.f;
    if (c < cols) {
        const float* x = X + (int64_t)k * sk + c;
        for (int r = g; r < rows; r += 4) s += x[(int64_t)r * sr];
    }
    red[g][cl] = s;
    __syncthreads();
    if (g == 0 && c < cols) sums[(int64_t)k * cols + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

// out[c] = sum_k sums[k][c]^2 (out2, nullable, gets the same)
__global__ void sens_sq_over_k(const float* sums, int cols, int K, float* out, float* out2) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= cols) return;
    float sq = 0.f;
    for (int k = 0; k < K; ++k) {
        const float v = sums[(int64_t)k * cols + c];
        sq += v * v;
    }
    out[c] = sq;
    if (out2) out2[c] = sq;
}

// logit.bias: out[v] = sum_k (sum_b dZ_k[b, v])^2 with sum_b dZ_k[b, v] = [k = group(v)] sum_b lp[b, v] inv_g[b, k]
// - PS[v, k], PS = p^T S (a tile product)
__global__ void sens_logb_sq(const float* LP, const float* IG, const float* PS, int Bs, int V, int K, int split,
                             float* out) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= V) return;
    const int kv = v / split;
    float own = 0.f;
    for (int b = 0; b < Bs; ++b) own += LP[(int64_t)b * V + v] * IG[b * K + kv];
    float sq = 0.f;
    for (int k = 0; k < K; ++k) {
        const float g = (k == kv ? own : 0.f) - PS[(int64_t)v * K + k];
        sq += g * g;
    }
    out[v] = sq;
}

// PW = sum over the split partials (fixed order)
__global__ void sens_sum_parts(const float* parts, int nparts, int64_t n, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
    for (int z = 0; z < nparts; ++z) s += parts[(int64_t)z * n + i];
    out[i] = s;
}

// embedding rows: row t gathers dX of every (cell i >= 1, row b) fed token t (BOS at cell 1, else the greedy
// token of logit step i - 1), G_k[t, e] = sum over those (i, b), in order, of dX[k, i, b, e]. Block (p, kc), with
// pair p = (i - 1) Bs + b: if p is its token's first pair, the token's pairs are listed in LDS and the block adds
// G_k[t, e]^2 over k in range kc into out[kc][t E + e] (thread e; partial rows summed by sens_finish).
// dX_all [K][L + 1][Bs][E]; npair <= EMB_MAXP.
#define EMB_MAXP 4096
#define EMB_KC 8
__global__ __launch_bounds__(256) void sens_emb_sq(const float* dX, const int32_t* tok, int stride, int L, int Bs, int E,
                                                   int K, int64_t D, float* out) {
    __shared__ int tq[EMB_MAXP];
    __shared__ int list[EMB_MAXP];
    __shared__ int cnt;
    const int p = blockIdx.x, kc = blockIdx.y, e = threadIdx.x;
    const int npair = L * Bs;
    for (int q = threadIdx.x; q < npair; q += blockDim.x) {
        const int i = q / Bs + 1, b = q % Bs;
        tq[q] = i == 1 ? 0 : tok[(int64_t)b * stride + (i - 2)];
    }
    __syncthreads();
    const int t = tq[p];
    int earlier = 0;
    for (int q = threadIdx.x; q < p; q += blockDim.x) earlier |= tq[q] == t;
    if (__syncthreads_or(earlier)) return;                   // not the first pair of this token
    if (threadIdx.x == 0) {
        int n = 0;
        for (int q = p; q < npair; ++q)
            if (tq[q] == t) list[n++] = (q / Bs + 1) * Bs + q % Bs;    // (cell, row) -> row of dX_all
        cnt = n;
    }
    __syncthreads();
    if (e >= E) return;
    const int64_t sk = (int64_t)(L + 1) * Bs * E;
    const int kpr = (K + EMB_KC - 1) / EMB_KC, k0 = kc * kpr, k1 = min(k0 + kpr, K);
    float sq = 0.f;
    for (int k = k0; k < k1; ++k) {
        float s = 0.f;
        for (int j = 0; j < cnt; ++j) s += dX[(int64_t)k * sk + (int64_t)list[j] * E + e];
        sq += s * s;
    }
    out[(int64_t)kc * D + (int64_t)t * E + e] = sq;
}

// s_j = sqrt(sum over the segment's range partials of part[z][j]) / Bs, then s < underflow -> underflow,
// s /= underflow (safe_mutations.py:63-65). Segment q = [off[q], off[q + 1]) has nz[q] partial rows.
struct Segs {
    int64_t off[10];
    int nz[9];
};
__global__ void sens_finish(const float* part, int64_t D, Segs sg, float inv_bs, float underflow, float* out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= D) return;
    int q = 0;
    while (q < 8 && j >= sg.off[q + 1]) ++q;
    float acc = 0.f;
    for (int z = 0; z < sg.nz[q]; ++z) acc += part[(int64_t)z * D + j];
    float s = sqrtf(acc) * inv_bs;
    if (underflow > 0.f) {
        s = s < underflow ? underflow : s;
        s /= underflow;
    }
    out[j] = s;
}

inline unsigned blocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

#define SENS_NZ 16           // k-range partial rows of the square sums

struct SensWork {
    int Bs = 0, K = 0, L = 0;
    int64_t D = 0;
    float* X = nullptr;     // [L + 1][Bs, E] cell inputs
    float* S = nullptr;     // [L + 1][Bs, 5R] gate sums
    float* Sh = nullptr;    // [Bs, 5R] the h2h chain of the current cell
    float* C = nullptr;     // [L + 1][Bs, R]
    float* H = nullptr;     // [L + 1][Bs, R]
    float* Z = nullptr;     // [Bs, V] logits
    float* LP = nullptr;    // [Bs, V] log-probs
    float* P = nullptr;     // [Bs, V] exp(log-probs)
    float* IG = nullptr;    // [Bs, K]
    float* SG = nullptr;    // [Bs, K]
    float* PW = nullptr;    // [Bs, R] p Wl
    float* PWp = nullptr;   // [32][Bs, R] its split partials
    float* PS = nullptr;    // [V, K] p^T S
    float* CS = nullptr;    // [K, 5R] per-seed bias column sums
    float* dH = nullptr;    // [K, Bs, R]
    float* dC = nullptr;    // [K, Bs, R]
    float* dS = nullptr;    // [K][L + 1][Bs][5R]
    float* dX = nullptr;    // [K][L + 1][Bs][E]
    float* part = nullptr;  // [SENS_NZ][D] square-sum partials
};

namespace {

void free_all(SensWork* w) {
    float* ps[] = {w->X, w->S, w->Sh, w->C, w->H, w->Z, w->LP, w->P, w->IG, w->SG, w->PW, w->PWp, w->PS, w->CS, w->dH, w->dC, w->dS, w->dX, w->part};
    for (float* p : ps)
        if (p) (void)hipFree(p);
    w->X = w->S = w->Sh = w->C = w->H = w->Z = w->LP = w->P = w->IG = w->SG = w->PW = w->PWp = w->PS = w->CS = nullptr;
    w->dH = w->dC = w->dS = w->dX = w->part = nullptr;
    w->Bs = w->K = w->L = 0;
    w->D = 0;
}

hipError_t grow(SensWork* w, const SensParams* p) {
    if (w->Bs >= p->Bs && w->K >= p->K && w->L >= p->L && w->D == p->D) return hipSuccess;
    free_all(w);
    const int64_t L1 = p->L + 1, Bs = p->Bs, K = p->K, E = p->E, R = p->R, V = p->V1;
    const struct { float** q; int64_t n; } a[] = {
        {&w->X, L1 * Bs * E}, {&w->S, L1 * Bs * 5 * R}, {&w->Sh, Bs * 5 * R}, {&w->C, L1 * Bs * R}, {&w->H, L1 * Bs * R},
        {&w->Z, Bs * V}, {&w->LP, Bs * V}, {&w->P, Bs * V}, {&w->IG, Bs * K}, {&w->SG, Bs * K}, {&w->PW, Bs * R}, {&w->PWp, 32 * Bs * R}, {&w->PS, V * K}, {&w->CS, K * 5 * R},
        {&w->dH, K * Bs * R}, {&w->dC, K * Bs * R}, {&w->dS, K * L1 * Bs * 5 * R}, {&w->dX, K * L1 * Bs * E},
        {&w->part, SENS_NZ * p->D}};
    for (const auto& x : a) {
        hipError_t e = hipMalloc((void**)x.q, (size_t)x.n * sizeof(float));
        if (e != hipSuccess) {
            free_all(w);
            return e;
        }
    }
    w->Bs = p->Bs;
    w->K = p->K;
    w->L = p->L;
    w->D = p->D;
    return hipSuccess;
}

TileArgs targs(int M, int N, int R, const float* B, int64_t sBk, int64_t sBr, int64_t sBn, float* C, int64_t sCk,
               int64_t sCm, int64_t sCn, int beta = 0) {
    TileArgs t;
    t.M = M; t.N = N; t.R = R;
    t.B = B; t.sBk = sBk; t.sBr = sBr; t.sBn = sBn;
    t.C = C; t.sCk = sCk; t.sCm = sCm; t.sCn = sCn;
    t.beta = beta;
    t.k0 = 0; t.kpr = 1; t.k_end = 1;
    t.bias = nullptr;
    t.kperm = 0;
    return t;
}

// the forward products in the reference's arithmetic: every chain from its bias, r in the nn_kperm order, as the
// engine's decode (bit-exact with the reference): the activations, and so the max-out choices of the cells, are
// the reference's own
TileArgs fwd(TileArgs t, const float* bias) {
    t.bias = bias;
    t.kperm = 1;
    return t;
}

// C_k = A_k B_k for k < batch
template <class AOp>
void gemm(const AOp& A, const TileArgs& t, int batch, hipStream_t st) {
    hipLaunchKernelGGL((sens_tile<AOp, false>), dim3(blocks(t.M, TM), blocks(t.N, TN), batch), dim3(256), 0, st, A, t);
}

// part[z][out + m sCm + n] = sum over the k of range z of (A_k B)[m, n]^2, nz ranges over k < K
template <class AOp>
void sqsum(const AOp& A, TileArgs t, int K, int nz, hipStream_t st) {
    t.k0 = 0;
    t.kpr = (K + nz - 1) / nz;
    t.k_end = K;
    const int z = (K + t.kpr - 1) / t.kpr;
    hipLaunchKernelGGL((sens_tile<AOp, true>), dim3(blocks(t.M, TM), blocks(t.N, TN), z), dim3(256), 0, st, A, t);
}

Strided sa(const float* p, int64_t sk, int64_t sm, int64_t sr) {
    Strided s;
    s.p = p; s.sk = sk; s.sm = sm; s.sr = sr;
    return s;
}

}  // namespace

extern "C" SensWork* nicnes_sens_create() { return new SensWork(); }

extern "C" void nicnes_sens_destroy(SensWork* w) {
    if (!w) return;
    free_all(w);
    delete w;
}

extern "C" int nicnes_sens_run(SensWork* w, const SensParams* p, hipStream_t st) {
    if (!w || !p || p->Bs < 1 || p->L < 1 || p->split < 1) return 1;
    if (p->E > 256 || p->R > 256) return 1;                     // thread-per-column kernels
    if ((int64_t)p->L * p->Bs > EMB_MAXP) return 1;             // sens_emb_sq's pair list
    if (grow(w, p) != hipSuccess) return 3;
    const int Bs = p->Bs, E = p->E, R = p->R, F = p->F, V = p->V1, K = p->K, L = p->L, G5 = 5 * R;
    const int64_t D = p->D, L1 = L + 1;
    const float* th = p->theta;
    const float *Wimg = th + p->off_img_w, *bimg = th + p->off_img_b, *Wemb = th + p->off_emb_w;
    const float *Wl = th + p->off_log_w, *bl = th + p->off_log_b;
    const float *Wi = th + p->off_i2h_w, *bi = th + p->off_i2h_b, *Wh = th + p->off_h2h_w, *bh = th + p->off_h2h_b;
    auto Xs = [&](int i) { return w->X + (int64_t)i * Bs * E; };
    auto Ss = [&](int i) { return w->S + (int64_t)i * Bs * G5; };
    auto Cs = [&](int i) { return w->C + (int64_t)i * Bs * R; };
    auto Hs = [&](int i) { return w->H + (int64_t)i * Bs * R; };
    // token fed to cell i (1..L): BOS for i = 1, else the greedy token of logit step i - 1
    auto tok_col = [&](int i) { return i == 1 ? -1 : i - 2; };

    // ---- forward: image cell, then L token cells (forward_for_sensitivity, nets.py:48-64); C = A B with
    // A row-major [rows, red] and B = W^T of a row-major [out, in] weight
    gemm(sa(p->fc, 0, F, 1), fwd(targs(Bs, E, F, Wimg, 0, 1, F, Xs(0), 0, E, 1), bimg), 1, st);   // img_embed
    for (int i = 0; i <= L; ++i) {
        if (i >= 1)
            hipLaunchKernelGGL(sens_embed_gather, dim3(Bs), dim3(E), 0, st, Xs(i), Wemb, p->tok, p->tok_stride,
                               tok_col(i), Bs, E);
        gemm(sa(Xs(i), 0, E, 1), fwd(targs(Bs, G5, E, Wi, 0, 1, E, Ss(i), 0, G5, 1), bi), 1, st);          // i2h
        if (i >= 1) gemm(sa(Hs(i - 1), 0, R, 1), fwd(targs(Bs, G5, R, Wh, 0, 1, R, w->Sh, 0, G5, 1), bh), 1, st);   // h2h
        hipLaunchKernelGGL(sens_cell_fwd, dim3(blocks((int64_t)Bs * R, 256)), dim3(256), 0, st, Ss(i),
                           i ? (const float*)w->Sh : (const float*)nullptr, bh,
                           i ? (const float*)Cs(i - 1) : (const float*)nullptr, Cs(i), Hs(i), Bs, R);
        if (p->tok_internal && i >= 1 && i < L) {      // the token fed to cell i + 1 (nets.py:60-63)
            gemm(sa(Hs(i), 0, R, 1), fwd(targs(Bs, V, R, Wl, 0, 1, R, w->Z, 0, V, 1), bl), 1, st);
            hipLaunchKernelGGL(sens_greedy, dim3(Bs), dim3(256), 0, st, w->Z, V, p->tok, p->tok_stride, i - 1);
        }
    }
    gemm(sa(Hs(L), 0, R, 1), fwd(targs(Bs, V, R, Wl, 0, 1, R, w->Z, 0, V, 1), bl), 1, st);             // logit
    hipLaunchKernelGGL(sens_logsoftmax, dim3(Bs), dim3(256), 0, st, w->Z, w->LP, w->P, V);

    // ---- the K backward passes at once
    hipLaunchKernelGGL(sens_seed, dim3(Bs, K), dim3(128), 0, st, w->LP, w->IG, w->SG, Bs, V, K, p->split);
    DzA dz;
    dz.lp = w->LP; dz.pr = w->P; dz.ig = w->IG; dz.S = w->SG; dz.V = V; dz.K = K; dz.split = p->split;
    float* part = w->part;
    // logit.weight: G_k[v, r] = sum_b dZ_k[b, v] H_L[b, r]; logit.bias
    sqsum(dz, targs(V, R, Bs, Hs(L), 0, R, 1, part + p->off_log_w, D, R, 1), K, SENS_NZ, st);
    // logit.bias: PS = p^T S over the batch, then the group terms
    gemm(sa(w->P, 0, 1, V), targs(V, K, Bs, w->SG, 0, K, 1, w->PS, 0, K, 1), 1, st);
    hipLaunchKernelGGL(sens_logb_sq, dim3(blocks(V, 256)), dim3(256), 0, st, w->LP, w->IG, w->PS, Bs, V, K, p->split,
                       part + p->off_log_b);
    // dH of the last cell: p Wl once (split over the vocabulary: nsp partial products, summed in order), then the
    // group terms
    {
        int nsp = 1;
        for (int d = 32; d > 1; --d)
            if (V % d == 0 && V / d >= TR) { nsp = d; break; }
        const int cl = V / nsp;
        gemm(sa(w->P, cl, V, 1), targs(Bs, R, cl, Wl, (int64_t)cl * R, R, 1, w->PWp, (int64_t)Bs * R, R, 1), nsp, st);
        hipLaunchKernelGGL(sens_sum_parts, dim3(blocks((int64_t)Bs * R, 256)), dim3(256), 0, st, w->PWp, nsp,
                           (int64_t)Bs * R, w->PW);
    }
    hipLaunchKernelGGL(sens_dh_logit, dim3(Bs, K), dim3(R), 0, st, w->LP, w->IG, w->SG, w->PW, Wl, w->dH, Bs, V, K, R,
                       p->split);
    if (hipMemsetAsync(w->dC, 0, (size_t)K * Bs * R * sizeof(float), st) != hipSuccess) return 4;
    const int64_t sdk = L1 * Bs * G5, sxk = L1 * Bs * E;
    for (int i = L; i >= 0; --i) {
        float* dSi = w->dS + (int64_t)i * Bs * G5;
        hipLaunchKernelGGL(sens_cell_bwd, dim3(blocks((int64_t)K * Bs * R, 256)), dim3(256), 0, st, w->dH, w->dC, Ss(i),
                           Cs(i), i ? (const float*)Cs(i - 1) : (const float*)nullptr, dSi, sdk, K, Bs, R);
        // dX_i = dS_i Wi ([5R, E] row-major), dH_{i-1} = dS_i Wh
        gemm(sa(dSi, sdk, G5, 1), targs(Bs, E, G5, Wi, 0, E, 1, w->dX + (int64_t)i * Bs * E, sxk, E, 1), K, st);
        if (i >= 1)
            gemm(sa(dSi, sdk, G5, 1), targs(Bs, R, G5, Wh, 0, R, 1, w->dH, (int64_t)Bs * R, R, 1), K, st);
    }
    // gate weights: G_k[g, e] = sum over (cell i, b) of dS_k[i, b, g] X_i[b, e] (h2h: cells 1..L with H_{i-1})
    sqsum(sa(w->dS, sdk, 1, G5), targs(G5, E, (int)(L1 * Bs), w->X, 0, E, 1, part + p->off_i2h_w, D, E, 1), K, SENS_NZ, st);
    sqsum(sa(w->dS + (int64_t)Bs * G5, sdk, 1, G5), targs(G5, R, L * Bs, w->H, 0, R, 1, part + p->off_h2h_w, D, R, 1), K,
          SENS_NZ, st);
    // both gate biases take every cell's dS (h2h's bias is added at cell 0 too, where h = 0)
    hipLaunchKernelGGL(sens_colsum_k, dim3(blocks(G5, 64), K), dim3(256), 0, st, w->dS, (int)(L1 * Bs), G5, (int64_t)G5,
                       sdk, w->CS);
    hipLaunchKernelGGL(sens_sq_over_k, dim3(blocks(G5, 256)), dim3(256), 0, st, w->CS, G5, K, part + p->off_i2h_b,
                       part + p->off_h2h_b);
    // img_embed: G_k[e, f] = sum_b dX_k[0, b, e] fc[b, f]; its bias
    sqsum(sa(w->dX, sxk, 1, E), targs(E, F, Bs, p->fc, 0, F, 1, part + p->off_img_w, D, F, 1), K, SENS_NZ, st);
    hipLaunchKernelGGL(sens_colsum_k, dim3(blocks(E, 64), K), dim3(256), 0, st, w->dX, Bs, E, (int64_t)E, sxk, w->CS);
    hipLaunchKernelGGL(sens_sq_over_k, dim3(blocks(E, 256)), dim3(256), 0, st, w->CS, E, K, part + p->off_img_b,
                       (float*)nullptr);
    // embedding rows never fed stay 0 (in every partial row)
    for (int z = 0; z < EMB_KC; ++z)
        if (hipMemsetAsync(part + (int64_t)z * D + p->off_emb_w, 0, (size_t)(p->off_log_w - p->off_emb_w) * sizeof(float),
                           st) != hipSuccess)
            return 4;
    hipLaunchKernelGGL(sens_emb_sq, dim3(L * Bs, EMB_KC), dim3(256), 0, st, w->dX, p->tok, p->tok_stride, L, Bs, E, K, D,
                       part + p->off_emb_w);
    Segs sg;
    const int64_t offs[10] = {p->off_img_w, p->off_img_b, p->off_emb_w, p->off_log_w, p->off_log_b,
                              p->off_i2h_w, p->off_i2h_b, p->off_h2h_w, p->off_h2h_b, D};
    const int kpr = (K + SENS_NZ - 1) / SENS_NZ, nzk = (K + kpr - 1) / kpr;
    const int nz[9] = {nzk, 1, EMB_KC, nzk, 1, nzk, 1, nzk, 1};   // k-range partial rows per segment
    for (int q = 0; q < 10; ++q) sg.off[q] = offs[q];
    for (int q = 0; q < 9; ++q) sg.nz[q] = nz[q];
    hipLaunchKernelGGL(sens_finish, dim3(blocks(D, 256)), dim3(256), 0, st, part, D, sg, 1.f / (float)Bs, p->underflow,
                       p->out);
    return hipGetLastError() == hipSuccess ? 0 : 6;
}
