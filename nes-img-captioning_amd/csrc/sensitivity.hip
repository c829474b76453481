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

#include <algorithm>
#include <type_traits>

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
#define SENS_TR 32        // reduction chunk of the tile kernel (sens_tile<..., TR>; 64 measured slower: fewer waves)
#define TR_MIN 32        // the smallest chunk: the logit split below keeps V / nsp >= TR_MIN
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

// nn_kperm inside a 16-aligned block: chain position p -> r (the pattern keeps each 16 in place)
__device__ __forceinline__ int perm16(int p) { const int j = p >> 1; return (j & 3) + 8 * (j >> 2) + 4 * (p & 1); }

// chunk [r0, r0 + TR) of A (TM rows from m0) and B (TN columns from n0) into registers: NPT + NPT values per
// thread, the 256 threads laid along the operand's unit-stride dimension; with kperm, chain position p of the
// chunk holds r0 + (p & ~15) + perm16(p & 15). TR = 64: a wave's 32 MFMAs per chunk cover the next chunk's
// loads better (at 32 the chunk loop was load-latency bound: a 640-long reduction took 20 load -> barrier rounds)
__device__ __forceinline__ int chunk_r(const TileArgs& t, int p) { return t.kperm ? (p & ~15) + perm16(p & 15) : p; }

template <int TR, class AOp>
__device__ __forceinline__ void tile_load(const AOp& A, const TileArgs& t, int k, int m0, int n0, int r0, float (&ra)[TM * TR / 256],
                                          float (&rb)[TM * TR / 256]) {
    const int tid = threadIdx.x;
    const bool am = A.m_unit();
#pragma unroll
    for (int e = 0; e < TM * TR / 256; ++e) {
        const int i = tid + 256 * e;
        const int m = am ? (i & (TM - 1)) : (i / TR), p = am ? (i / TM) : (i & (TR - 1));
        const int gm = m0 + m, gr = r0 + chunk_r(t, p);
        ra[e] = (gm < t.M && gr < t.R) ? A(k, gm, gr) : 0.f;
    }
    const bool bn = t.sBn == 1;
#pragma unroll
    for (int e = 0; e < TM * TR / 256; ++e) {
        const int i = tid + 256 * e;
        const int n = bn ? (i & (TN - 1)) : (i / TR), p = bn ? (i / TN) : (i & (TR - 1));
        const int gn = n0 + n, gr = r0 + chunk_r(t, p);
        rb[e] = (gn < t.N && gr < t.R) ? t.B[(int64_t)k * t.sBk + (int64_t)gr * t.sBr + (int64_t)gn * t.sBn] : 0.f;
    }
}

template <int TR, class AOp>
__device__ __forceinline__ void tile_store(const AOp& A, const TileArgs& t, float* As, float* Bs, const float (&ra)[TM * TR / 256],
                                           const float (&rb)[TM * TR / 256]) {
    const int tid = threadIdx.x;
    const bool am = A.m_unit(), bn = t.sBn == 1;
#pragma unroll
    for (int e = 0; e < TM * TR / 256; ++e) {
        const int i = tid + 256 * e;
        const int m = am ? (i & (TM - 1)) : (i / TR), p = am ? (i / TM) : (i & (TR - 1));
        As[p * LDS_P + m] = ra[e];
        const int n = bn ? (i & (TN - 1)) : (i / TR), q = bn ? (i / TN) : (i & (TR - 1));
        Bs[q * LDS_P + n] = rb[e];
    }
}

// the same chunk through 16-byte loads along each operand's unit-stride dimension (Strided A only; the host checks
// alignment and unit-dimension extents, tile_fits4): 2 + 2 float4 per thread at TR = 32. Loaded along r, the four
// values sit at chain positions chunk_p(r) (the inverse of chunk_r).
__device__ __forceinline__ int inv16(int x) { return 2 * ((x >> 3) * 4 + (x & 3)) + ((x >> 2) & 1); }
__device__ __forceinline__ int chunk_p(const TileArgs& t, int r) { return t.kperm ? (r & ~15) + inv16(r & 15) : r; }

template <int TR>
__device__ __forceinline__ void tile_load4(const Strided& A, const TileArgs& t, int k, int m0, int n0, int r0,
                                           float4 (&ra)[TM * TR / 1024], float4 (&rb)[TM * TR / 1024]) {
    const int tid = threadIdx.x;
    const bool am = A.sm == 1, bn = t.sBn == 1;
#pragma unroll
    for (int e = 0; e < TM * TR / 1024; ++e) {
        const int f = tid + 256 * e;
        int gm, gr;
        if (am) { gm = m0 + 4 * (f & (TM / 4 - 1)); gr = r0 + chunk_r(t, f / (TM / 4)); }
        else    { gm = m0 + f / (TR / 4);           gr = r0 + 4 * (f & (TR / 4 - 1)); }
        ra[e] = (gm < t.M && gr < t.R) ? *reinterpret_cast<const float4*>(A.p + (int64_t)k * A.sk + (int64_t)gm * A.sm +
                                                                          (int64_t)gr * A.sr)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        int gn;
        if (bn) { gn = n0 + 4 * (f & (TN / 4 - 1)); gr = r0 + chunk_r(t, f / (TN / 4)); }
        else    { gn = n0 + f / (TR / 4);           gr = r0 + 4 * (f & (TR / 4 - 1)); }
        rb[e] = (gn < t.N && gr < t.R) ? *reinterpret_cast<const float4*>(t.B + (int64_t)k * t.sBk + (int64_t)gr * t.sBr +
                                                                          (int64_t)gn * t.sBn)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

template <int TR>
__device__ __forceinline__ void tile_store4(const Strided& A, const TileArgs& t, float* As, float* Bs,
                                            const float4 (&ra)[TM * TR / 1024], const float4 (&rb)[TM * TR / 1024]) {
    const int tid = threadIdx.x;
    const bool am = A.sm == 1, bn = t.sBn == 1;
#pragma unroll
    for (int e = 0; e < TM * TR / 1024; ++e) {
        const int f = tid + 256 * e;
        const float va[4] = {ra[e].x, ra[e].y, ra[e].z, ra[e].w}, vb[4] = {rb[e].x, rb[e].y, rb[e].z, rb[e].w};
        if (am) {
            const int m = 4 * (f & (TM / 4 - 1)), q = f / (TM / 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) As[q * LDS_P + m + u] = va[u];
        } else {
            const int m = f / (TR / 4), r = 4 * (f & (TR / 4 - 1));
#pragma unroll
            for (int u = 0; u < 4; ++u) As[chunk_p(t, r + u) * LDS_P + m] = va[u];
        }
        if (bn) {
            const int n = 4 * (f & (TN / 4 - 1)), q = f / (TN / 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) Bs[q * LDS_P + n + u] = vb[u];
        } else {
            const int n = f / (TR / 4), r = 4 * (f & (TR / 4 - 1));
#pragma unroll
            for (int u = 0; u < 4; ++u) Bs[chunk_p(t, r + u) * LDS_P + n] = vb[u];
        }
    }
}

// acc += A(k)[tile rows, :] B(k)[:, tile columns] for this wave's 32 x 32 block
template <int TR, bool V4, class AOp>
__device__ __forceinline__ void tile_product(const AOp& A, const TileArgs& t, int k, int m0, int n0, float* As, float* Bs,
                                             f32x16& acc) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = 32 * (w >> 1), wn = 32 * (w & 1), kh = lane >> 5, li = lane & 31;
    float ra[V4 ? 1 : TM * TR / 256], rb[V4 ? 1 : TM * TR / 256];
    float4 ra4[V4 ? TM * TR / 1024 : 1], rb4[V4 ? TM * TR / 1024 : 1];
    if constexpr (V4) tile_load4<TR>(A, t, k, m0, n0, 0, ra4, rb4);
    else tile_load<TR>(A, t, k, m0, n0, 0, ra, rb);
    for (int r0 = 0; r0 < t.R; r0 += TR) {
        __syncthreads();                                     // the previous chunk has been read
        if constexpr (V4) tile_store4<TR>(A, t, As, Bs, ra4, rb4);
        else tile_store<TR>(A, t, As, Bs, ra, rb);
        __syncthreads();
        if (r0 + TR < t.R) {
            if constexpr (V4) tile_load4<TR>(A, t, k, m0, n0, r0 + TR, ra4, rb4);
            else tile_load<TR>(A, t, k, m0, n0, r0 + TR, ra, rb);
        }
#pragma unroll
        for (int j = 0; j < TR / 2; ++j) {
            const float a = As[(2 * j + kh) * LDS_P + wm + li];
            const float b = Bs[(2 * j + kh) * LDS_P + wn + li];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
    }
}

template <class AOp, bool SQ, int TR = SENS_TR, bool V4 = false>
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
        tile_product<TR, V4>(A, t, k, m0, n0, As, Bs, acc);
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

// ---- products with a k-invariant B --------------------------------------------------------------------
// C_k = A_k B for a range of seeds k, where only A (the per-seed dS or dX) changes with k: the gate- and
// image-weight square sums (SQ: out[z][m, n] = sum over the range z of C_k[m, n]^2) and the backward recurrence's
// dX_i = dS_i Wi, dH_{i-1} = dS_i Wh (gemm: out + k sOz, both products in one launch: columns n >= N1 come from
// the second (B2, out2)). sens_tile re-staged B for every k; here a workgroup (32 rows m x 128 columns n, 4 waves
// of 32 columns) stages each 32-long chunk of the reduction once -- B's chunk and the range's A chunks (BSQ_KMAX
// of them) -- and keeps one accumulator per k. Each (k, tile) chain runs over r in the same chunk order as
// sens_tile's, so the products are those of the tile kernel. A is m-unit (sm = 1), B row-major (sBr).
#define BSQ_KMAX 6          // accumulators (seeds) per workgroup at most
#define BSQ_RC 32
#define BSQ_AP (32 + 4)
#define BSQ_BP (128 + 4)
template <bool SQ, int KK>
__global__ __launch_bounds__(256) void sens_bsq(Strided A, const float* B, const float* B2, int64_t sBr, int M, int N1,
                                                int N, int Rr, int K, int kpr, float* out, float* out2, int64_t sOz,
                                                int64_t sOz2, int64_t sOm) {
    __shared__ __attribute__((aligned(16))) float As[KK * BSQ_RC * BSQ_AP];
    __shared__ __attribute__((aligned(16))) float Bs[BSQ_RC * BSQ_BP];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, kh = lane >> 5, li = lane & 31;
    const int m0 = blockIdx.x * 32, z = blockIdx.z;
    int n0 = blockIdx.y * 128, Nb = N1;
    if (n0 >= N1) {                                              // the second product's columns
        B = B2;
        out = out2;
        sOz = sOz2;
        n0 -= N1;
        Nb = N - N1;
    }
    const bool am = A.m_unit();                                  // lanes along m (else along r) for the loads
    const int ka = z * kpr, nk = min(ka + kpr, K) - ka;
    float4 ra[KK], rb[4];
    // 16-byte loads along each operand's unit-stride dimension (the host checks alignment and extents: bsq_fits)
    auto load = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {                        // A: 32 x 32 of seed ka + kk, one float4 per thread
            const int u = tid >> 3, c4 = 4 * (tid & 7);          // u: the strided index, c4: along the unit dimension
            const int m = am ? c4 : u, r = am ? u : c4;
            const bool ok = kk < nk && m0 + m < M && r0 + r < Rr;
            ra[kk] = ok ? *reinterpret_cast<const float4*>(A.p + (int64_t)(ka + kk) * A.sk + (int64_t)(m0 + m) * A.sm +
                                                           (int64_t)(r0 + r) * A.sr)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {                            // B: 32 x 128, four float4 per thread
            const int f = tid + 256 * e, r = f >> 5, n4 = 4 * (f & 31);
            rb[e] = (n0 + n4 < Nb && r0 + r < Rr) ? *reinterpret_cast<const float4*>(B + (int64_t)(r0 + r) * sBr + n0 + n4)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    f32x16 acc[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[kk][i] = 0.f;
    load(0);
    for (int r0 = 0; r0 < Rr; r0 += BSQ_RC) {
        __syncthreads();                                         // the previous chunk has been read
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
            const int u = tid >> 3, c4 = 4 * (tid & 7);
            float* a = As + kk * BSQ_RC * BSQ_AP;
            if (am) {
                *reinterpret_cast<float4*>(a + u * BSQ_AP + c4) = ra[kk];          // row r = u, columns m = c4 ..
            } else {
                a[(c4 + 0) * BSQ_AP + u] = ra[kk].x;                            // rows r = c4 .., column m = u
                a[(c4 + 1) * BSQ_AP + u] = ra[kk].y;
                a[(c4 + 2) * BSQ_AP + u] = ra[kk].z;
                a[(c4 + 3) * BSQ_AP + u] = ra[kk].w;
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int f = tid + 256 * e, r = f >> 5, n4 = 4 * (f & 31);
            *reinterpret_cast<float4*>(Bs + r * BSQ_BP + n4) = rb[e];
        }
        __syncthreads();
        if (r0 + BSQ_RC < Rr) load(r0 + BSQ_RC);
        // operands read one k-step ahead, so the MFMAs never wait on LDS
        const float* bl = Bs + kh * BSQ_BP + 32 * w + li;
        const float* al = As + kh * BSQ_AP + li;
        float bn = bl[0], an[KK];
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) an[kk] = al[kk * BSQ_RC * BSQ_AP];
#pragma unroll
        for (int j = 0; j < BSQ_RC / 2; ++j) {
            const float b = bn;
            float a[KK];
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) a[kk] = an[kk];
            if (j + 1 < BSQ_RC / 2) {
                bn = bl[(2 * j + 2) * BSQ_BP];
#pragma unroll
                for (int kk = 0; kk < KK; ++kk) an[kk] = al[(kk * BSQ_RC + 2 * j + 2) * BSQ_AP];
            }
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) acc[kk] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk], b, acc[kk], 0, 0, 0);
        }
    }
    // accumulator element i of lane l: row 8 (i >> 2) + 4 (l >> 5) + (i & 3), column l & 31 (of this wave's block)
    const int n = n0 + 32 * w + li;
    if (n >= Nb) return;
    if (SQ) {
        f32x16 sq;
#pragma unroll
        for (int i = 0; i < 16; ++i) sq[i] = 0.f;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
            if (kk < nk)
#pragma unroll
                for (int i = 0; i < 16; ++i) sq[i] += acc[kk][i] * acc[kk][i];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int m = m0 + 8 * (i >> 2) + 4 * kh + (i & 3);
            if (m < M) out[(int64_t)z * sOz + (int64_t)m * sOm + n] = sq[i];
        }
    } else {
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
            if (kk < nk)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int m = m0 + 8 * (i >> 2) + 4 * kh + (i & 3);
                    if (m < M) out[(int64_t)(ka + kk) * sOz + (int64_t)m * sOm + n] = acc[kk][i];
                }
    }
}

// ---- elementwise and small kernels
// rows[z][0 .. n) = 0 for the grid's y rows (stride D): the embedding rows no token fed, in every partial row
__global__ __launch_bounds__(256) void sens_zero_rows(float* rows, int64_t D, int64_t n) {
    float* r = rows + (int64_t)blockIdx.y * D;
    const int64_t i0 = (int64_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i0 + 256 * u < n) r[i0 + 256 * u] = 0.f;
}

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
#define ROW_T 1024           // threads per row of the row kernels (sens_logsoftmax, sens_greedy): 128 rows, 9488 wide
__global__ __launch_bounds__(ROW_T) void sens_logsoftmax(const float* Z, float* LP, float* P, int V) {
    __shared__ float red[ROW_T];
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
// whose log-prob (z - m) - lse equals the maximum, -lse
__global__ __launch_bounds__(ROW_T) void sens_greedy(const float* Z, int V, int32_t* tok, int stride, int col) {
    // two passes: the running (max, exp-sum) of each thread (the sum rescaled when the max rises), combined over the
    // block; then the first id at the maximum log-prob
    __shared__ float red[ROW_T], reds[ROW_T];
    __shared__ int redi[ROW_T];
    const float* z = Z + (int64_t)blockIdx.x * V;
    float m = -INFINITY, s = 0.f;
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
        const float x = z[v];
        if (x > m) {
            s = s * expf(m - x) + 1.f;
            m = x;
        } else {
            s += expf(x - m);
        }
    }
    red[threadIdx.x] = m;
    reds[threadIdx.x] = s;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            const float ma = red[threadIdx.x], mb = red[threadIdx.x + o];
            const float mx = fmaxf(ma, mb);
            const float sa = ma == -INFINITY ? 0.f : reds[threadIdx.x] * expf(ma - mx);
            const float sb = mb == -INFINITY ? 0.f : reds[threadIdx.x + o] * expf(mb - mx);
            red[threadIdx.x] = mx;
            reds[threadIdx.x] = sa + sb;
        }
        __syncthreads();
    }
    m = red[0];
    const float lse = logf(reds[0]);
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
// PW = p Wl (one product for every k). The group products O_k = lp[:, group k] Wl[group k, :] are a batched tile
// product written into dH (groups 0 .. kown - 1; a group past the vocabulary's end is 0); this kernel finishes
// dH = O_k inv_g - S PW in place. Thread per (k, b, r).
__global__ void sens_dh_logit(const float* IG, const float* Sg, const float* PW, float* dH, int Bs, int K, int R,
                              int kown) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)K * Bs * R) return;
    const int64_t kb = i / R;
    const int r = (int)(i % R), b = (int)(kb % Bs), k = (int)(kb / Bs);
    const float own = k < kown ? dH[i] : 0.f;
    dH[i] = own * IG[b * K + k] - Sg[b * K + k] * PW[(int64_t)b * R + r];
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
__global__ __launch_bounds__(1024) void sens_colsum_k(const float* X, int rows, int cols, int64_t sr, int64_t sk,
                                                      float* sums) {
    __shared__ float red[16][64];
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6, k = blockIdx.y;
    const int c = blockIdx.x * 64 + cl;
    float s = 0.f;
    if (c < cols) {
        const float* x = X + (int64_t)k * sk + c;
        for (int r = g; r < rows; r += 16) s += x[(int64_t)r * sr];
    }
    red[g][cl] = s;
    __syncthreads();
    if (g == 0 && c < cols) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) t += red[q][cl];
        sums[(int64_t)k * cols + c] = t;
    }
}

// out[c] = sum_k sums[k][c]^2 (out2, nullable, gets the same): 64 columns x 16 k lanes per block, lanes added in order
__global__ __launch_bounds__(1024) void sens_sq_over_k(const float* sums, int cols, int K, float* out, float* out2) {
    __shared__ float red[16][64];
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    float sq = 0.f;
    if (c < cols)
        for (int k = g; k < K; k += 16) {
            const float v = sums[(int64_t)k * cols + c];
            sq += v * v;
        }
    red[g][cl] = sq;
    __syncthreads();
    if (g == 0 && c < cols) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) t += red[q][cl];
        out[c] = t;
        if (out2) out2[c] = t;
    }
}

// logit.weight, the square sums without the seed ever formed (Bs <= LSQ_BMAX, R = 128): G_k[v, r] = sum_b dZ_k[b, v]
// H[b, r] with dZ_k[b, v] = -p[b, v] S[b, k] + [v in group k] lp[b, v] inv_g[b, k]. Only S[:, k] and inv_g[:, k]
// change with k, so both operands are loaded into LDS once per workgroup and stay there for its k range: p^T of the
// workgroup's 128 vocabulary rows (the MFMA A operand, scaled by -S[b, k] as it is read) and H (the B operand). The
// own term runs a second chain from lp only for the (at most two) groups that meet a wave's rows. Workgroup: 8
// waves; wave w takes vocabulary rows 32 (w & 3) and all 128 columns (four 32 x 32 accumulators, so each A value
// feeds 4 MFMAs), and the range's k of parity w >> 2; the two parities' square sums are added at the end (in LDS).
// Grid (V / 128, k ranges). out[z][v R + r] = sum over the range of G_k^2 (summed by sens_finish).
#define LSQ_BMAX 128
#define LSQ_R 128
#define LSQ_HP (LSQ_R + 4)
#define LSQ_KMAX 12
__global__ __launch_bounds__(512) void sens_logit_sq(const float* P, const float* LP, const float* IG, const float* SG,
                                                     const float* H, int Bs, int V, int K, int split, int kpr,
                                                     int64_t D, float* out) {
    extern __shared__ __attribute__((aligned(16))) float lsq[];
    float* Hs = lsq;                                             // [b][r]  H rows (zero past Bs)
    float* Ps = lsq + LSQ_BMAX * LSQ_HP;                         // [b][v]  p of the workgroup's 128 rows
    float* St = Ps + LSQ_BMAX * LSQ_HP;                          // [k - ka][b]  -S[b, k]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, kh = lane >> 5, li = lane & 31;
    const int z = blockIdx.y, ka = z * kpr, kb = min(ka + kpr, K);
    const int v0 = blockIdx.x * 128, vl = 32 * (w & 3);         // the workgroup's and this wave's first rows
    const int vw = v0 + vl, v = vw + li;                         // v: the row this lane supplies to the A operand
    const int par = w >> 2;                                      // this wave's k parity
    // Hs holds row b's column r = 32 q + c at b HP + 4 c + q: a lane's four B values (q = 0..3) are one b128 read
    for (int i = tid; i < LSQ_BMAX * LSQ_R; i += 512) {
        const int b = i / LSQ_R, r = i % LSQ_R;
        Hs[b * LSQ_HP + 4 * (r & 31) + (r >> 5)] = b < Bs ? H[(int64_t)b * LSQ_R + r] : 0.f;
    }
    for (int i = tid; i < LSQ_BMAX * 128; i += 512) {
        const int b = i / 128, c = i % 128;
        Ps[b * LSQ_HP + c] = (b < Bs && v0 + c < V) ? P[(int64_t)b * V + v0 + c] : 0.f;
    }
    for (int i = tid; i < LSQ_KMAX * LSQ_BMAX; i += 512) {
        const int kk = i / LSQ_BMAX, b = i % LSQ_BMAX;
        St[i] = (ka + kk < kb && b < Bs) ? -SG[b * K + ka + kk] : 0.f;
    }
    __syncthreads();
    const float* hl = Hs + 4 * li;                               // this lane's B values: hl[b HP + q]
    const int jn = (Bs + 1) >> 1;                                // k-steps that carry rows (the own chain)
    f32x16 sq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 16; ++i) sq[q][i] = 0.f;
    for (int k = ka + par; k < kb; k += 2) {
        f32x16 acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[q][i] = 0.f;
        const float* st = St + (k - ka) * LSQ_BMAX + kh;
        const float* pl = Ps + kh * LSQ_HP + vl + li;
        // each k-step's operands are read one step ahead, so the four MFMAs never wait on LDS
        float4 hn = *reinterpret_cast<const float4*>(hl + kh * LSQ_HP);
        float pn = pl[0], sn = st[0];
#pragma unroll 8
        for (int j = 0; j < LSQ_BMAX / 2; ++j) {                 // (rows past Bs are zero in Ps, St and Hs)
            const float4 h = hn;
            const float x = pn * sn;
            if (j + 1 < LSQ_BMAX / 2) {
                hn = *reinterpret_cast<const float4*>(hl + (2 * j + 2 + kh) * LSQ_HP);
                pn = pl[(2 * j + 2) * LSQ_HP];
                sn = st[2 * j + 2];
            }
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.x, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.y, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.z, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.w, acc[3], 0, 0, 0);
        }
        // the own term of group k, for the waves whose rows meet it: lp[b, v] inv_g[b, k] on [k split, (k + 1) split)
        if (k * split < vw + 32 && (k + 1) * split > vw) {
            const bool own = v < V && v / split == k;
            for (int j = 0; j < jn; ++j) {
                const int b = 2 * j + kh;
                const float x = (own && b < Bs) ? LP[(int64_t)b * V + v] * IG[b * K + k] : 0.f;
                const float4 h = *reinterpret_cast<const float4*>(hl + b * LSQ_HP);
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.x, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.y, acc[1], 0, 0, 0);
                acc[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.z, acc[2], 0, 0, 0);
                acc[3] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, h.w, acc[3], 0, 0, 0);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 16; ++i) sq[q][i] += acc[q][i] * acc[q][i];
    }
    // odd-parity waves hand their sums to the even ones through LDS (Ps is free now)
    __syncthreads();
    float* xs = Ps + (w & 3) * (64 * 64) + lane;
    if (par) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int i = 0; i < 16; ++i) xs[(16 * q + i) * 64] = sq[q][i];
    }
    __syncthreads();
    if (par) return;
    // accumulator element i of lane l: row 8 (i >> 2) + 4 (l >> 5) + (i & 3), column l & 31 (of block q)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int vv = vw + 8 * (i >> 2) + 4 * kh + (i & 3);
        if (vv >= V) continue;
        float* o = out + (int64_t)z * D + (int64_t)vv * LSQ_R + li;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[32 * q] = sq[q][i] + xs[(16 * q + i) * 64];
    }
}
#define LSQ_LDS_BYTES ((2 * LSQ_BMAX * LSQ_HP + LSQ_KMAX * LSQ_BMAX) * 4)

// logit.bias: out[v] = sum_k (sum_b dZ_k[b, v])^2 with sum_b dZ_k[b, v] = [k = group(v)] sum_b lp[b, v] inv_g[b, k]
// - PS[k, v], PS = (p^T S)^T (a tile product; k-major so the threads of a k read consecutive v)
__global__ __launch_bounds__(256) void sens_logb_sq(const float* LP, const float* IG, const float* PS, int Bs, int V,
                                                    int K, int split, float* out) {
    // block: 64 consecutive v x 4 parts; part g sums the rows b = g mod 4 of own, then the seeds k = g mod 4
    __shared__ float red[4][64];
    const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int v = blockIdx.x * 64 + cl;
    const bool ok = v < V;
    const int kv = ok ? v / split : 0;
    float own = 0.f;
    if (ok)
        for (int b = g; b < Bs; b += 4) own += LP[(int64_t)b * V + v] * IG[b * K + kv];
    red[g][cl] = own;
    __syncthreads();
    own = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
    __syncthreads();
    float sq = 0.f;
    if (ok)
        for (int k = g; k < K; k += 4) {
            const float gk = (k == kv ? own : 0.f) - PS[(int64_t)k * V + v];
            sq += gk * gk;
        }
    red[g][cl] = sq;
    __syncthreads();
    if (g == 0 && ok) out[v] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
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
// the pairs grouped by token, once per vector (one block): keys token * EMB_MAXP + pair sorted in LDS (bitonic), so a
// token's pairs are contiguous and in increasing pair order. runs[0] = the number of tokens fed, runs[1 + u] = the
// first sorted position of token u's pairs (runs[1 + n] = npair), rtok[u] its token, list[pos] its dX row.
#define EMB_CH 16            // pairs per chunk of the two-pass embedding sums
#define EMB_KPR2 12          // seeds per k lane (8 lanes: K <= 96)
__global__ __launch_bounds__(1024) void sens_emb_runs(const int32_t* tok, int stride, int L, int Bs, int* runs, int* rtok,
                                                      int* list, int* rchunk) {
    __shared__ uint32_t key[EMB_MAXP];
    __shared__ int rstart[EMB_MAXP + 1];
    __shared__ int wcnt[16];
    const int npair = L * Bs, tid = threadIdx.x;
    int n2 = 1;
    while (n2 < npair) n2 <<= 1;
    for (int q = tid; q < n2; q += 1024) {
        uint32_t k = 0xffffffffu;                                // padding sorts last
        if (q < npair) {
            const int i = q / Bs + 1, b = q % Bs;
            const int t = i == 1 ? 0 : tok[(int64_t)b * stride + (i - 2)];
            k = (uint32_t)t * EMB_MAXP + (uint32_t)q;
        }
        key[q] = k;
    }
    __syncthreads();
    for (int size = 2; size <= n2; size <<= 1)
        for (int stride2 = size >> 1; stride2 > 0; stride2 >>= 1) {
            for (int q = tid; q < n2; q += 1024) {
                const int o = q ^ stride2;
                if (o > q) {
                    const bool up = (q & size) == 0;
                    const uint32_t a = key[q], b = key[o];
                    if ((a > b) == up) { key[q] = b; key[o] = a; }
                }
            }
            __syncthreads();
        }
    // run starts: positions whose token differs from the previous one, numbered in order
    int nr = 0;
    for (int q0 = 0; q0 < npair; q0 += 1024) {
        const int q = q0 + tid;
        const bool st = q < npair && (q == 0 || key[q] / EMB_MAXP != key[q - 1] / EMB_MAXP);
        const uint64_t bal = __ballot(st);
        if ((tid & 63) == 0) wcnt[tid >> 6] = __popcll(bal);
        __syncthreads();
        int base = nr;
        for (int u = 0; u < (tid >> 6); ++u) base += wcnt[u];
        const int pos = base + __popcll(bal & ((1ull << (tid & 63)) - 1));
        if (st) {
            runs[1 + pos] = q;
            rstart[pos] = q;
            rtok[pos] = (int)(key[q] / EMB_MAXP);
        }
        if (q < npair) {
            const int pq = (int)(key[q] % EMB_MAXP);
            list[q] = (pq / Bs + 1) * Bs + pq % Bs;             // (cell, row) -> row of dX_all
        }
        for (int u = 0; u < 16; ++u) nr += wcnt[u];
        __syncthreads();
    }
    if (tid == 0) {
        runs[0] = nr;
        runs[1 + nr] = npair;
    }
    // chunks of at most EMB_CH pairs per run (sens_emb_part): rchunk[u] = the run's first chunk, rchunk[nr] = total
    if (rchunk != nullptr && tid == 0) {
        int c = 0;
        for (int u = 0; u < nr; ++u) {
            rchunk[u] = c;
            c += ((u + 1 < nr ? rstart[u + 1] : npair) - rstart[u] + EMB_CH - 1) / EMB_CH;
        }
        rchunk[nr] = c;
    }
}

// pass 1 of the two-pass embedding sums: chunk c (of run u: pairs j0 + EMB_CH q ..) -> part[c][k][e] = the chunk's
// sum over its pairs, in pair order, for every seed k (1024 threads = 8 k lanes x 128 e, EMB_KPR2 seeds each).
// Grid: an upper bound of the chunk count; blocks past rchunk[runs[0]] exit.
__global__ __launch_bounds__(1024) void sens_emb_part(const float* dX, const int* runs, const int* rchunk, const int* list,
                                                      int L, int Bs, int E, int K, float* part) {
    const int c = blockIdx.x, e = threadIdx.x & 127, kl = threadIdx.x >> 7;
    const int nr = runs[0];
    if (c >= rchunk[nr] || e >= E) return;
    int lo = 0, hi = nr - 1;                                     // the run holding chunk c
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rchunk[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const int j0 = runs[1 + lo] + EMB_CH * (c - rchunk[lo]), j1 = min(j0 + EMB_CH, runs[2 + lo]);
    const int64_t sk = (int64_t)(L + 1) * Bs * E;
    const int k0 = kl * EMB_KPR2;
    if (k0 >= K) return;                                         // small vocabularies: this k lane has no seeds
    float acc[EMB_KPR2];
#pragma unroll
    for (int q = 0; q < EMB_KPR2; ++q) acc[q] = 0.f;
    const float* base = dX + (int64_t)k0 * sk + e;
    int64_t koff[EMB_KPR2];
#pragma unroll
    for (int q = 0; q < EMB_KPR2; ++q) koff[q] = (k0 + q < K ? (int64_t)q : 0) * sk;
    for (int j = j0; j < j1; ++j) {
        const float* row = base + (int64_t)list[j] * E;
        float x[EMB_KPR2];
#pragma unroll
        for (int q = 0; q < EMB_KPR2; ++q) x[q] = row[koff[q]];
#pragma unroll
        for (int q = 0; q < EMB_KPR2; ++q) acc[q] += x[q];
    }
    float* o = part + ((int64_t)c * K + k0) * E + e;
#pragma unroll
    for (int q = 0; q < EMB_KPR2; ++q)
        if (k0 + q < K) o[(int64_t)q * E] = acc[q];
}

// pass 2: run u -> out[t E + e] = sum_k (sum over the run's chunks, in order, of part[c][k][e])^2; the 8 k lanes'
// square sums added in lane order
__global__ __launch_bounds__(1024) void sens_emb_fin(const float* part, const int* runs, const int* rtok, const int* rchunk,
                                                     int E, int K, float* out) {
    __shared__ float red[8][128];
    const int u = blockIdx.x, e = threadIdx.x & 127, kl = threadIdx.x >> 7;
    if (u >= runs[0]) return;
    const int c0 = rchunk[u], c1 = rchunk[u + 1];
    float sq = 0.f;
    if (e < E)
        for (int q = 0; q < EMB_KPR2; ++q) {
            const int k = kl * EMB_KPR2 + q;
            if (k >= K) break;
            float s = 0.f;
            for (int c = c0; c < c1; ++c) s += part[((int64_t)c * K + k) * E + e];
            sq += s * s;
        }
    red[kl][e] = sq;
    __syncthreads();
    if (kl == 0 && e < E) {
        float tot = 0.f;
#pragma unroll
        for (int z = 0; z < 8; ++z) tot += red[z][e];
        out[(int64_t)rtok[u] * E + e] = tot;
    }
}

// embedding rows: row t gathers dX of every (cell i >= 1, row b) fed token t (BOS at cell 1, else the greedy token
// of logit step i - 1), G_k[t, e] = sum over those (i, b), in pair order, of dX[k, i, b, e]. Block (run u, kc),
// thread e: out[kc][t E + e] = sum over k in range kc of G_k[t, e]^2 (partial rows summed by sens_finish).
// dX_all [K][L + 1][Bs][E]; blocks past the number of runs exit.
__global__ __launch_bounds__(256) void sens_emb_sq(const float* dX, const int* runs, const int* rtok, const int* list,
                                                   int L, int Bs, int E, int K, int64_t D, float* out) {
    const int u = blockIdx.x, kc = blockIdx.y, e = threadIdx.x;
    if (u >= runs[0] || e >= E) return;
    const int j0 = runs[1 + u], j1 = runs[2 + u], t = rtok[u];
    const int64_t sk = (int64_t)(L + 1) * Bs * E;
    const int kpr = (K + EMB_KC - 1) / EMB_KC, k0 = kc * kpr, k1 = min(k0 + kpr, K);
    float sq = 0.f;
    for (int k = k0; k < k1; ++k) {
        const float* base = dX + (int64_t)k * sk + e;
        float s = 0.f;
        int j = j0;
        for (; j + 8 <= j1; j += 8) {                            // 8 loads in flight, added in pair order
            float x[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = base[(int64_t)list[j + q] * E];
#pragma unroll
            for (int q = 0; q < 8; ++q) s += x[q];
        }
        for (; j < j1; ++j) s += base[(int64_t)list[j] * E];
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

// an A/B switch of the timing runs (scripts/gpu_r05_sens.sh): set and not "0"
inline bool env_on(const char* name) {
    const char* v = getenv(name);
    return v && v[0] && !(v[0] == '0' && v[1] == 0);
}

}  // namespace

#define SENS_NZ 16           // k-range partial rows of the square sums (tile kernel)
#define SENS_NZ_MAX 32       // ... at most (the gate weights' sens_bsq ranges)

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
    float* PS = nullptr;    // [K, V] (p^T S)^T
    float* CS = nullptr;    // [K, 5R] per-seed bias column sums
    float* dH = nullptr;    // [K, Bs, R]
    float* dC = nullptr;    // [K, Bs, R]
    float* dS = nullptr;    // [K][L + 1][Bs][5R]
    float* dX = nullptr;    // [K][L + 1][Bs][E]
    float* part = nullptr;  // [SENS_NZ_MAX][D] square-sum partials
    int* runs = nullptr;    // [EMB_MAXP + 2] sens_emb_runs: run count, run starts
    int* rtok = nullptr;    // [EMB_MAXP] each run's token
    int* elist = nullptr;   // [EMB_MAXP] dX rows in token-then-pair order
    int* rchunk = nullptr;  // [EMB_MAXP + 2] each run's first chunk (sens_emb_part)
    float* echunk = nullptr;  // [chunks][K][E] the chunks' sums
};

namespace {

void free_all(SensWork* w) {
    float* ps[] = {w->X, w->S, w->Sh, w->C, w->H, w->Z, w->LP, w->P, w->IG, w->SG, w->PW, w->PWp, w->PS, w->CS, w->dH, w->dC, w->dS, w->dX, w->part};
    for (float* p : ps)
        if (p) (void)hipFree(p);
    for (int* p : {w->runs, w->rtok, w->elist, w->rchunk})
        if (p) (void)hipFree(p);
    w->runs = w->rtok = w->elist = w->rchunk = nullptr;
    if (w->echunk) (void)hipFree(w->echunk);
    w->echunk = nullptr;
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
        {&w->part, SENS_NZ_MAX * p->D}};
    for (const auto& x : a) {
        hipError_t e = hipMalloc((void**)x.q, (size_t)x.n * sizeof(float));
        if (e != hipSuccess) {
            free_all(w);
            return e;
        }
    }
    for (int** q : {&w->runs, &w->rtok, &w->elist, &w->rchunk}) {
        hipError_t e = hipMalloc((void**)q, (EMB_MAXP + 2) * sizeof(int));
        if (e != hipSuccess) {
            free_all(w);
            return e;
        }
    }
    {
        const int64_t npair = L1 * Bs, maxch = npair / EMB_CH + npair;
        hipError_t e = hipMalloc((void**)&w->echunk, (size_t)(maxch * K * E) * sizeof(float));
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
// sens_tile's 16-byte loads (Strided A): aligned bases, strides of whole float4s, unit-dimension extents in float4s
inline bool tile_fits4(const Strided& A, const TileArgs& t) {
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    const bool am = A.sm == 1, ar = A.sr == 1, bn = t.sBn == 1, br = t.sBr == 1;
    return !env_on("NICNES_SENS_TILE_SCALAR") && al(A.p) && al(t.B) && (am || ar) && (bn || br) && A.sk % 4 == 0 &&
           t.sBk % 4 == 0 && (am ? A.sr % 4 == 0 && t.M % 4 == 0 : A.sm % 4 == 0 && t.R % 4 == 0) &&
           (bn ? t.sBr % 4 == 0 && t.N % 4 == 0 : t.sBn % 4 == 0 && t.R % 4 == 0);
}

template <class AOp>
void gemm(const AOp& A, const TileArgs& t, int batch, hipStream_t st) {
    if constexpr (std::is_same<AOp, Strided>::value) {
        if (tile_fits4(A, t)) {
            // 64-long chunks: with 16-byte loads the registers allow them (4 + 4 float4 per thread), and a wave's 32
            // MFMAs per chunk cover the next chunk's loads (the image projection's 2048-long chains: 32 chunks, not 64)
            hipLaunchKernelGGL((sens_tile<Strided, false, 64, true>), dim3(blocks(t.M, TM), blocks(t.N, TN), batch),
                               dim3(256), 0, st, A, t);
            return;
        }
    }
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
            hipLaunchKernelGGL(sens_greedy, dim3(Bs), dim3(ROW_T), 0, st, w->Z, V, p->tok, p->tok_stride, i - 1);
        }
    }
    gemm(sa(Hs(L), 0, R, 1), fwd(targs(Bs, V, R, Wl, 0, 1, R, w->Z, 0, V, 1), bl), 1, st);             // logit
    hipLaunchKernelGGL(sens_logsoftmax, dim3(Bs), dim3(ROW_T), 0, st, w->Z, w->LP, w->P, V);

    // ---- the K backward passes at once
    hipLaunchKernelGGL(sens_seed, dim3(Bs, K), dim3(128), 0, st, w->LP, w->IG, w->SG, Bs, V, K, p->split);
    DzA dz;
    dz.lp = w->LP; dz.pr = w->P; dz.ig = w->IG; dz.S = w->SG; dz.V = V; dz.K = K; dz.split = p->split;
    float* part = w->part;
    // sens_bsq's 16-byte loads: 16-byte aligned bases, strides and unit-dimension extents in whole float4s
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    auto bsq_fits = [&](const Strided& A, int M, int Rr, const float* Bm, int64_t sBr, int N) {
        const bool am = A.sm == 1, ar = A.sr == 1;
        return al(A.p) && al(Bm) && (am || ar) && A.sk % 4 == 0 && (am ? A.sr % 4 == 0 && M % 4 == 0
                                                                         : A.sm % 4 == 0 && Rr % 4 == 0) &&
               sBr % 4 == 0 && N % 4 == 0;
    };
    // logit.weight: G_k[v, r] = sum_b dZ_k[b, v] H_L[b, r]; logit.bias
    // (its own k ranges: 10 k per workgroup -> 75 x 10 workgroups for 3 full rounds of one per CU at K = 95)
    const int kpr_l = std::min((K + 9) / 10, LSQ_KMAX), nz_l = (K + kpr_l - 1) / kpr_l;
    bool lsq_used = false;
    {
        const int kpr = kpr_l, nz = nz_l;
        static const bool lsq_ok = hipFuncSetAttribute((const void*)sens_logit_sq,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       LSQ_LDS_BYTES) == hipSuccess;
        lsq_used = lsq_ok && Bs <= LSQ_BMAX && R == LSQ_R && nz <= SENS_NZ && !env_on("NICNES_SENS_TILE_LOGIT");
        if (lsq_used)
            hipLaunchKernelGGL(sens_logit_sq, dim3(blocks(V, 128), nz), dim3(512), LSQ_LDS_BYTES, st, w->P, w->LP, w->IG, w->SG,
                               Hs(L), Bs, V, K, p->split, kpr, D, part + p->off_log_w);
        else
            sqsum(dz, targs(V, R, Bs, Hs(L), 0, R, 1, part + p->off_log_w, D, R, 1), K, SENS_NZ, st);
    }
    // logit.bias: PS = p^T S over the batch, then the group terms
    gemm(sa(w->P, 0, 1, V), targs(V, K, Bs, w->SG, 0, K, 1, w->PS, 0, 1, V), 1, st);          // PS^T [K, V]
    hipLaunchKernelGGL(sens_logb_sq, dim3(blocks(V, 64)), dim3(256), 0, st, w->LP, w->IG, w->PS, Bs, V, K, p->split,
                       part + p->off_log_b);
    // dH of the last cell: p Wl once (split over the vocabulary: nsp partial products, summed in order), then the
    // group terms
    {
        int nsp = 1;
        for (int d = 32; d > 1; --d)
            if (V % d == 0 && V / d >= TR_MIN) { nsp = d; break; }
        const int cl = V / nsp;
        gemm(sa(w->P, cl, V, 1), targs(Bs, R, cl, Wl, (int64_t)cl * R, R, 1, w->PWp, (int64_t)Bs * R, R, 1), nsp, st);
        hipLaunchKernelGGL(sens_sum_parts, dim3(blocks((int64_t)Bs * R, 256)), dim3(256), 0, st, w->PWp, nsp,
                           (int64_t)Bs * R, w->PW);
    }
    {
        const int sp = p->split, kfull = V / sp, rem = V - kfull * sp;
        if (kfull > 0)           // the full groups: O_k [Bs, R] = lp[:, k sp .. + sp] Wl[k sp .. + sp, :]
            gemm(sa(w->LP, sp, V, 1), targs(Bs, R, sp, Wl, (int64_t)sp * R, R, 1, w->dH, (int64_t)Bs * R, R, 1), kfull, st);
        if (rem > 0)             // the last group's rows inside the vocabulary
            gemm(sa(w->LP + (int64_t)kfull * sp, 0, V, 1),
                 targs(Bs, R, rem, Wl + (int64_t)kfull * sp * R, 0, R, 1, w->dH + (int64_t)kfull * Bs * R, 0, R, 1), 1, st);
        const int kown = std::min(K, kfull + (rem > 0 ? 1 : 0));
        hipLaunchKernelGGL(sens_dh_logit, dim3(blocks((int64_t)K * Bs * R, 256)), dim3(256), 0, st, w->IG, w->SG, w->PW,
                           w->dH, Bs, K, R, kown);
    }
    if (hipMemsetAsync(w->dC, 0, (size_t)K * Bs * R * sizeof(float), st) != hipSuccess) return 4;
    const int64_t sdk = L1 * Bs * G5, sxk = L1 * Bs * E;
    for (int i = L; i >= 0; --i) {
        float* dSi = w->dS + (int64_t)i * Bs * G5;
        hipLaunchKernelGGL(sens_cell_bwd, dim3(blocks((int64_t)K * Bs * R, 256)), dim3(256), 0, st, w->dH, w->dC, Ss(i),
                           Cs(i), i ? (const float*)Cs(i - 1) : (const float*)nullptr, dSi, sdk, K, Bs, R);
        // dX_i = dS_i Wi ([5R, E] row-major), dH_{i-1} = dS_i Wh: one launch of both (Wi, Wh stay put over k), 2 seeds
        // per workgroup (4 x (1 or 2) x 32 workgroups at Bs = 128, K = 95); the tile kernel with NICNES_SENS_TILE_BWD
        // (the fused launch puts dH's columns at the second 128-column tile: E == R == 128 exactly)
        if (E == R && E == 128 && !env_on("NICNES_SENS_TILE_BWD") && bsq_fits(sa(dSi, sdk, G5, 1), Bs, G5, Wi, E, E) &&
            al(Wh)) {
            const int kb2 = 2, nzb = (K + kb2 - 1) / kb2;
            hipLaunchKernelGGL((sens_bsq<false, 2>), dim3(blocks(Bs, 32), i >= 1 ? 2 : 1, nzb), dim3(256), 0, st,
                               sa(dSi, sdk, G5, 1), Wi, Wh, (int64_t)E, Bs, E, i >= 1 ? 2 * E : E, G5, K, kb2,
                               w->dX + (int64_t)i * Bs * E, w->dH, sxk, (int64_t)Bs * R, (int64_t)E);
        } else {
            gemm(sa(dSi, sdk, G5, 1), targs(Bs, E, G5, Wi, 0, E, 1, w->dX + (int64_t)i * Bs * E, sxk, E, 1), K, st);
            if (i >= 1)
                gemm(sa(dSi, sdk, G5, 1), targs(Bs, R, G5, Wh, 0, R, 1, w->dH, (int64_t)Bs * R, R, 1), K, st);
        }
    }
    // gate weights: G_k[g, e] = sum over (cell i, b) of dS_k[i, b, g] X_i[b, e] (h2h: cells 1..L with H_{i-1})
    // (B = X, H, fc does not change with k: sens_bsq stages each chunk of it once for a range of BSQ_KMAX seeds)
    // (3 seeds per workgroup, up to SENS_NZ_MAX k ranges: 640 workgroups for the gate weights at K = 95)
    const int kpr_g = (K + SENS_NZ_MAX - 1) / SENS_NZ_MAX, nz_g = (K + kpr_g - 1) / kpr_g;
    const bool bsq = kpr_g <= 3 && !env_on("NICNES_SENS_TILE_GATES") &&
                     bsq_fits(sa(w->dS, sdk, 1, G5), G5, (int)(L1 * Bs), w->X, E, E) &&
                     bsq_fits(sa(w->dS + (int64_t)Bs * G5, sdk, 1, G5), G5, L * Bs, w->H, R, R) &&
                     bsq_fits(sa(w->dX, sxk, 1, E), E, Bs, p->fc, F, F);
    auto bsq_run = [&](Strided A, const float* Bm, int M, int N, int Rr, float* out) {
        hipLaunchKernelGGL((sens_bsq<true, 3>), dim3(blocks(M, 32), blocks(N, 128), nz_g), dim3(256), 0, st,
                           A, Bm, Bm, (int64_t)N, M, N, N, Rr, K, kpr_g, out, out, D, D, (int64_t)N);
    };
    if (bsq) {
        bsq_run(sa(w->dS, sdk, 1, G5), w->X, G5, E, (int)(L1 * Bs), part + p->off_i2h_w);
        bsq_run(sa(w->dS + (int64_t)Bs * G5, sdk, 1, G5), w->H, G5, R, L * Bs, part + p->off_h2h_w);
    } else {
        sqsum(sa(w->dS, sdk, 1, G5), targs(G5, E, (int)(L1 * Bs), w->X, 0, E, 1, part + p->off_i2h_w, D, E, 1), K, SENS_NZ, st);
        sqsum(sa(w->dS + (int64_t)Bs * G5, sdk, 1, G5), targs(G5, R, L * Bs, w->H, 0, R, 1, part + p->off_h2h_w, D, R, 1), K,
              SENS_NZ, st);
    }
    // both gate biases take every cell's dS (h2h's bias is added at cell 0 too, where h = 0)
    hipLaunchKernelGGL(sens_colsum_k, dim3(blocks(G5, 64), K), dim3(1024), 0, st, w->dS, (int)(L1 * Bs), G5, (int64_t)G5,
                       sdk, w->CS);
    hipLaunchKernelGGL(sens_sq_over_k, dim3(blocks(G5, 64)), dim3(1024), 0, st, w->CS, G5, K, part + p->off_i2h_b,
                       part + p->off_h2h_b);
    // img_embed: G_k[e, f] = sum_b dX_k[0, b, e] fc[b, f]; its bias
    if (bsq)
        bsq_run(sa(w->dX, sxk, 1, E), p->fc, E, F, Bs, part + p->off_img_w);
    else
        sqsum(sa(w->dX, sxk, 1, E), targs(E, F, Bs, p->fc, 0, F, 1, part + p->off_img_w, D, F, 1), K, SENS_NZ, st);
    hipLaunchKernelGGL(sens_colsum_k, dim3(blocks(E, 64), K), dim3(1024), 0, st, w->dX, Bs, E, (int64_t)E, sxk, w->CS);
    hipLaunchKernelGGL(sens_sq_over_k, dim3(blocks(E, 64)), dim3(1024), 0, st, w->CS, E, K, part + p->off_img_b,
                       (float*)nullptr);
    // embedding rows never fed stay 0 (in every partial row)
    const bool emb1 = E <= 128 && K <= 8 * EMB_KPR2 && !env_on("NICNES_SENS_EMB_KC");   // one partial row
    const int nz_emb = emb1 ? 1 : EMB_KC;
    hipLaunchKernelGGL(sens_zero_rows, dim3(blocks(p->off_log_w - p->off_emb_w, 1024), nz_emb), dim3(256), 0, st,
                       part + p->off_emb_w, D, p->off_log_w - p->off_emb_w);
    hipLaunchKernelGGL(sens_emb_runs, dim3(1), dim3(1024), 0, st, p->tok, p->tok_stride, L, Bs, w->runs, w->rtok, w->elist,
                       w->rchunk);
    if (emb1) {
        // two passes: every run cut into chunks of EMB_CH pairs (the BOS run has >= Bs pairs), the chunk sums added
        // per run in order
        const int npair = L * Bs, maxch = npair / EMB_CH + npair;
        hipLaunchKernelGGL(sens_emb_part, dim3(maxch), dim3(1024), 0, st, w->dX, w->runs, w->rchunk, w->elist, L, Bs, E, K,
                           w->echunk);
        hipLaunchKernelGGL(sens_emb_fin, dim3(npair), dim3(1024), 0, st, w->echunk, w->runs, w->rtok, w->rchunk, E, K,
                           part + p->off_emb_w);
    } else
        hipLaunchKernelGGL(sens_emb_sq, dim3(L * Bs, EMB_KC), dim3(std::max(E, 64)), 0, st, w->dX, w->runs, w->rtok,
                           w->elist, L, Bs, E, K, D, part + p->off_emb_w);
    Segs sg;
    const int64_t offs[10] = {p->off_img_w, p->off_img_b, p->off_emb_w, p->off_log_w, p->off_log_b,
                              p->off_i2h_w, p->off_i2h_b, p->off_h2h_w, p->off_h2h_b, D};
    const int kpr = (K + SENS_NZ - 1) / SENS_NZ, nzk = (K + kpr - 1) / kpr;
    const int nzgw = bsq ? nz_g : nzk;
    const int nz[9] = {nzgw, 1, nz_emb, lsq_used ? nz_l : nzk, 1, nzgw, 1, nzgw, 1};   // k-range partial rows per segment
    for (int q = 0; q < 10; ++q) sg.off[q] = offs[q];
    for (int q = 0; q < 9; ++q) sg.nz[q] = nz[q];
    hipLaunchKernelGGL(sens_finish, dim3(blocks(D, 256)), dim3(256), 0, st, part, D, sg, 1.f / (float)Bs, p->underflow,
                       p->out);
    return hipGetLastError() == hipSuccess ? 0 : 6;
}
