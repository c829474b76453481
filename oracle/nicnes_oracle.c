/*
 * nicnes_oracle.c -- CPU restatement of the reference fc_caption greedy decode.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (nes-img-captioning_amd/) links,
 * loads or calls this file; it is the checker used by tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg.
 *
 * Restates (op for op, one row at a time):
 *   FCModel._sample        /root/reference/src/captioning/nets.py:183-245 (greedy and sampled)
 *   LSTMCore.forward       /root/reference/src/captioning/nets.py:98-134   (vbn = layer_n = false)
 *   F.log_softmax + torch.max (first index on ties)   nets.py:202,208-209
 * Dense products are fp32 fma chains started from the bias in the order nn_kperm()
 * defines (include/nicnes_math.h); transcendental functions are the shared nn_* ones.
 * The HIP kernels follow the same definitions, so GPU tokens are compared bit-exactly
 * against this file; this file is compared margin-aware against the imported reference
 * (tests/golden/, made by scripts/make_golden.py).
 *
 * Build: oracle/Makefile (gcc -O3 -mavx2 -mfma -ffp-contract=off -fopenmp).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nicnes_math.h"

typedef struct {
    int32_t V1;   /* vocab_size + 1 (logit width), nets.py:151-152 */
    int32_t E;    /* input_encoding_size */
    int32_t R;    /* rnn_size */
    int32_t F;    /* fc_feat_size */
    int32_t T;    /* seq_length (16), nets.py:147 */
} od_dims;

typedef struct {
    int64_t img_w, img_b, emb_w, log_w, log_b, i2h_w, i2h_b, h2h_w, h2h_b, D;
} od_layout;

/* flat theta order = module registration order, nets.py:150-153 then LSTMCore :81-82 */
static od_layout od_make_layout(const od_dims* d) {
    od_layout L;
    int64_t o = 0;
    L.img_w = o; o += (int64_t)d->E * d->F;
    L.img_b = o; o += d->E;
    L.emb_w = o; o += (int64_t)d->V1 * d->E;
    L.log_w = o; o += (int64_t)d->V1 * d->R;
    L.log_b = o; o += d->V1;
    L.i2h_w = o; o += (int64_t)5 * d->R * d->E;
    L.i2h_b = o; o += 5 * d->R;
    L.h2h_w = o; o += (int64_t)5 * d->R * d->R;
    L.h2h_b = o; o += 5 * d->R;
    L.D = o;
    return L;
}

int64_t od_param_count(const od_dims* d) { return od_make_layout(d).D; }

void od_layout_offsets(const od_dims* d, int64_t* out10) {
    od_layout L = od_make_layout(d);
    int64_t v[10] = {L.img_w, L.img_b, L.emb_w, L.log_w, L.log_b, L.i2h_w, L.i2h_b, L.h2h_w, L.h2h_b, L.D};
    memcpy(out10, v, sizeof v);
}

/* position in the fma chain -> k; half_order = 1 swaps the two halves of every MFMA step */
static int perm_pos(int pos, int K, int half_order) {
    if ((K & 31) != 0) return pos;                       /* tiny dims: ascending */
    return nn_kperm(half_order ? (pos ^ 1) : pos);
}

/* W [rows][K] row-major -> WT[pos][rows] with columns visited in chain order */
static float* transpose_perm(const float* W, int rows, int K, int half_order) {
    float* WT = (float*)malloc(sizeof(float) * (size_t)rows * K);
    for (int p = 0; p < K; ++p) {
        int k = perm_pos(p, K, half_order);
        float* dst = WT + (size_t)p * rows;
        for (int r = 0; r < rows; ++r) dst[r] = W[(size_t)r * K + k];
    }
    return WT;
}

/* acc[r] continues its fmaf chain over the chain positions; x[k] read through the permutation */
static void gemv_chain_acc(const float* WT, const float* x, int rows, int K, int half_order, float* acc) {
    for (int p = 0; p < K; ++p) {
        const float xv = x[perm_pos(p, K, half_order)];
        const float* w = WT + (size_t)p * rows;
        for (int r = 0; r < rows; ++r) acc[r] = fmaf(w[r], xv, acc[r]);
    }
}

/* acc[r] = fmaf-chain over chain positions started from the bias */
static void gemv_chain(const float* WT, const float* bias, const float* x, int rows, int K,
                       int half_order, float* acc) {
    for (int r = 0; r < rows; ++r) acc[r] = bias[r];
    for (int p = 0; p < K; ++p) {
        const float xv = x[perm_pos(p, K, half_order)];
        const float* w = WT + (size_t)p * rows;
        for (int r = 0; r < rows; ++r) acc[r] = fmaf(w[r], xv, acc[r]);
    }
}

/* greedy pick: torch log_softmax (x - max) - lse, then first index of the max lp.
 * Returns token; *lp = max log-prob; *fragile = 1 if moving lse by +-2 ulp changes the
 * tie set (the GPU's lse is summed in another order and may differ in the last bits). */
static int greedy_pick(const float* logits, int V1, float* lp_out, uint8_t* fragile) {
    float m = logits[0];
    for (int v = 1; v < V1; ++v) if (logits[v] > m) m = logits[v];
    double s = 0.0;
    for (int v = 0; v < V1; ++v) s += exp((double)(logits[v] - m));
    float lse = (float)log(s);
    float best = -lse;                        /* lp at the max: (0) - lse */
    int tok = -1;
    for (int v = 0; v < V1; ++v) {
        float lp = (logits[v] - m) - lse;
        if (lp == best) { tok = v; break; }
    }
    /* fragility check on the near-max elements only */
    *fragile = 0;
    float l2[4];
    l2[0] = nextafterf(lse, INFINITY); l2[1] = nextafterf(l2[0], INFINITY);
    l2[2] = nextafterf(lse, -INFINITY); l2[3] = nextafterf(l2[2], -INFINITY);
    for (int q = 0; q < 4; ++q) {
        int t2 = -1;
        for (int v = 0; v < V1; ++v) {
            float d = logits[v] - m;
            if (d < -1e-5f) continue;
            if (d - l2[q] == -l2[q]) { t2 = v; break; }
        }
        if (t2 != tok) *fragile = 1;
    }
    *lp_out = best;
    return tok;
}

/* sampled pick (nets.py:210-231, greedy=False): p = exp(log_softmax) in fp32 (torch.exp), n = p /
 * sum(p) in fp32 (np.linalg.norm(row, ord=1)), then RandomState.choice(len, 1, p=n): cdf = cumsum(n)
 * in fp64 divided by its last entry, pick = first index with cdf > u (searchsorted side='right').
 * lp = the pick's log-prob (logprobs.gather). fragile = u within 1e-6 of the cdf boundary below or at
 * the pick (a different summation order of p moves the boundaries by ~1e-7). pbuf/cdf: [V1] scratch. */
static int sample_pick(const float* logits, int V1, double u, float* pbuf, double* cdf, float* lp_out,
                       uint8_t* fragile) {
    float m = logits[0];
    for (int v = 1; v < V1; ++v) if (logits[v] > m) m = logits[v];
    double s = 0.0;
    for (int v = 0; v < V1; ++v) s += exp((double)(logits[v] - m));
    const float lse = (float)log(s);
    double norm = 0.0;
    for (int v = 0; v < V1; ++v) { pbuf[v] = nn_expf((logits[v] - m) - lse); norm += pbuf[v]; }
    const float normf = (float)norm;
    double c = 0.0;
    for (int v = 0; v < V1; ++v) { c += (double)(pbuf[v] / normf); cdf[v] = c; }
    const double last = cdf[V1 - 1];
    int tok = V1 - 1;
    for (int v = 0; v < V1; ++v) if (cdf[v] / last > u) { tok = v; break; }
    const double hi = cdf[tok] / last, lo = tok > 0 ? cdf[tok - 1] / last : 0.0;
    *fragile = (fabs(hi - u) < 1e-6 || fabs(u - lo) < 1e-6) ? 1 : 0;
    *lp_out = (logits[tok] - m) - lse;
    return tok;
}

static int decode_core(const od_dims* d, const float* theta, const float* fc, int B, const double* u,
                       int32_t* seq, float* lp, uint8_t* fragile, int half_order);

/*
 * Greedy decode of B unique rows with a (possibly perturbed) fp32 theta.
 * seq[B*T] (int32), lp[B*T] (max log-prob per step; 0 after the global early exit, as
 * nets.py:242-243 leaves it), fragile[B*T]. Returns the number of logit steps run.
 */
int od_decode(const od_dims* d, const float* theta, const float* fc, int B,
              int32_t* seq, float* lp, uint8_t* fragile, int half_order) {
    return decode_core(d, theta, fc, B, NULL, seq, lp, fragile, half_order);
}

/*
 * Sampled decode (FCModel._sample with greedy=False, nets.py:210-243): row b draws u[b*T + t-1] at logit
 * step t, every row at every step until the whole batch has finished, as the reference draws one uniform
 * per row and step (np.random.choice per row, nets.py:220-224). lp = log-prob of the sampled token (also
 * for rows already finished, as seq_logprobs keeps it), 0 after the global early exit.
 */
int od_decode_sample(const od_dims* d, const float* theta, const float* fc, int B, const double* u,
                     int32_t* seq, float* lp, uint8_t* fragile, int half_order) {
    return decode_core(d, theta, fc, B, u, seq, lp, fragile, half_order);
}

static int decode_core(const od_dims* d, const float* theta, const float* fc, int B, const double* u,
                       int32_t* seq, float* lp, uint8_t* fragile, int half_order) {
    const od_layout L = od_make_layout(d);
    const int E = d->E, R = d->R, F = d->F, V1 = d->V1, T = d->T, G = 5 * R;
    float* WimgT = transpose_perm(theta + L.img_w, E, F, half_order);
    float* WiT = transpose_perm(theta + L.i2h_w, G, E, half_order);
    float* WhT = transpose_perm(theta + L.h2h_w, G, R, half_order);
    float* WlT = transpose_perm(theta + L.log_w, V1, R, half_order);
    int32_t* fin_step = (int32_t*)malloc(sizeof(int32_t) * (size_t)B);
    memset(seq, 0, sizeof(int32_t) * (size_t)B * T);
    memset(lp, 0, sizeof(float) * (size_t)B * T);
    memset(fragile, 0, (size_t)B * T);

#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
        float* x = (float*)malloc(sizeof(float) * (size_t)(E > R ? E : R));
        float* h = (float*)calloc((size_t)R, sizeof(float));
        float* c = (float*)calloc((size_t)R, sizeof(float));
        float* si = (float*)malloc(sizeof(float) * (size_t)G);
        float* sh = (float*)malloc(sizeof(float) * (size_t)G);
        float* logits = (float*)malloc(sizeof(float) * (size_t)V1);
        float* pbuf = u ? (float*)malloc(sizeof(float) * (size_t)V1) : NULL;
        double* cdf = u ? (double*)malloc(sizeof(double) * (size_t)V1) : NULL;
        int unfinished = 1, it = 0;
        fin_step[b] = T;
        for (int t = 0; t <= T; ++t) {
            if (t == 0) gemv_chain(WimgT, theta + L.img_b, fc + (size_t)b * F, E, F, half_order, x);
            else memcpy(x, theta + L.emb_w + (size_t)it * E, sizeof(float) * (size_t)E);
            /* gate sums as LSTMCore forms them, all_input_sums = i2h(xt) + h2h(prev_h)
             * (nets.py:109-111): two chains, (b_i2h + Wi.x) and (b_h2h + Wh.h), then one add.
             * At t = 0, h = 0 and the h2h chain runs over zeros. */
            gemv_chain(WiT, theta + L.i2h_b, x, G, E, half_order, si);
            gemv_chain(WhT, theta + L.h2h_b, h, G, R, half_order, sh);
            for (int u = 0; u < G; ++u) sh[u] = si[u] + sh[u];
            for (int u = 0; u < R; ++u) {
                float cn, hn;
                nn_lstm_cell(sh[u], sh[R + u], sh[2 * R + u], sh[3 * R + u], sh[4 * R + u], c[u], &cn, &hn);
                c[u] = cn;
                h[u] = hn;
            }
            if (t == 0) continue;                       /* t=0 logits are discarded */
            gemv_chain(WlT, theta + L.log_b, h, V1, R, half_order, logits);
            float lpv;
            uint8_t fr;
            int tok = u ? sample_pick(logits, V1, u[(size_t)b * T + t - 1], pbuf, cdf, &lpv, &fr)
                        : greedy_pick(logits, V1, &lpv, &fr);
            if (tok > 0 && unfinished) unfinished = 1; else unfinished = 0;
            it = tok * unfinished;
            seq[(size_t)b * T + t - 1] = it;
            lp[(size_t)b * T + t - 1] = lpv;
            fragile[(size_t)b * T + t - 1] = fr;
            if (!unfinished && fin_step[b] == T) fin_step[b] = t;
            if (t == T) break;
        }
        free(x); free(h); free(c); free(si); free(sh); free(logits); free(pbuf); free(cdf);
    }
    /* global early exit (nets.py:242-243): steps after every row finished stay 0 */
    int last = 0;
    for (int b = 0; b < B; ++b) if (fin_step[b] > last) last = fin_step[b];
    for (int b = 0; b < B; ++b)
        for (int t = last; t < T; ++t) { lp[(size_t)b * T + t] = 0.0f; fragile[(size_t)b * T + t] = 0; }
    free(fin_step); free(WimgT); free(WiT); free(WhT); free(WlT);
    return last;
}

/* single dense product, exposed for the MFMA-order probe test: out[r] = chain(W[r,:], x) */
void od_gemv(const float* W, const float* bias, const float* x, int rows, int K, int half_order,
             float* out) {
    float* WT = transpose_perm(W, rows, K, half_order);
    gemv_chain(WT, bias, x, rows, K, half_order, out);
    free(WT);
}

/* shared elementwise math, exposed for accuracy tests */
void od_vec_math(int which, const float* in, float* out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        switch (which) {
            case 0: out[i] = nn_expf(in[i]); break;
            case 1: out[i] = nn_sigmoidf(in[i]); break;
            default: out[i] = nn_tanhf(in[i]); break;
        }
    }
}

void od_noise_indices(uint64_t seed, uint64_t iteration, uint64_t member0, int64_t count,
                      uint64_t table_len, uint64_t dim, uint64_t* out) {
    for (int64_t i = 0; i < count; ++i)
        out[i] = nn_noise_index(seed, iteration, member0 + (uint64_t)i, table_len, dim);
}
