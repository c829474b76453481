/*
 * nicnes_math.h -- the engine's elementwise-math and indexing contract.
 *
 * Every function here is compiled twice: by hipcc for the gfx950 kernels and by
 * gcc for the CPU oracle (oracle/). Both builds use -ffp-contract=off and only
 * IEEE-exact primitives (fmaf, +, -, *, /, floorf, bit casts), so a given input
 * produces the same bits on the GPU and on the host. That is what makes the
 * GPU-vs-oracle greedy-token comparison bit-exact.
 *
 * What the reference uses instead (and why it is only margin-comparable):
 *   LSTMCore.forward  src/captioning/nets.py:98-134   torch.sigmoid / torch.tanh (Sleef, CPU)
 *   PolicyNet.evolve  src/algorithm/nets.py:101-113   torch.normal_ (global RNG; replaced by the
 *                                                     noise table + index rule below)
 */
#ifndef NICNES_MATH_H
#define NICNES_MATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define NN_FN __host__ __device__ static inline
#else
#define NN_FN static inline
#endif

/* ---- bit casts (union punning works in C and in clang/gcc C++) ---------------------- */
NN_FN float nn_i2f(int32_t i) { union { int32_t i; float f; } u; u.i = i; return u.f; }
NN_FN int32_t nn_f2i(float f) { union { int32_t i; float f; } u; u.f = f; return u.i; }

NN_FN float nn_floorf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_floorf(x);
#else
    return __builtin_floorf(x);
#endif
}

/* 2^n as a float for n in [-126, 127] */
NN_FN float nn_pow2i(int32_t n) { return nn_i2f((n + 127) << 23); }

/*
 * nn_expf: e^x, <= ~1 ulp on the range the hot path uses. Cody-Waite reduction x = n ln2 + r,
 * |r| <= ln2/2, degree-7 Taylor in Horner form with fmaf, one scale by 2^n. The argument is
 * clamped to [-87, 88] so the scale stays a normal power of two (below -87 the result is e^-87
 * instead of a subnormal or 0: every caller adds it to 1 or multiplies a bounded value by it);
 * above 88.72 the result is +inf and NaN passes through. Branch-free (one instruction stream for
 * every lane of a wavefront).
 */
NN_FN float nn_expf_core(float xc) {                   /* xc in [-87, 88], not NaN */
    const float log2e = 1.44269502162933349609375f;
    const float ln2_hi = 0.693145751953125f;          /* 12 significant bits: n*ln2_hi exact */
    const float ln2_lo = 1.428606765330187045e-06f;
    float n = nn_floorf(xc * log2e + 0.5f);
    float r = fmaf(-n, ln2_hi, xc);
    r = fmaf(-n, ln2_lo, r);
    float p = 1.98412701138295233250e-4f;             /* 1/7! */
    p = fmaf(p, r, 1.38888892251998186111e-3f);       /* 1/6! */
    p = fmaf(p, r, 8.33333376795053482056e-3f);       /* 1/5! */
    p = fmaf(p, r, 4.16666679084300994873e-2f);       /* 1/4! */
    p = fmaf(p, r, 1.66666671633720397949e-1f);       /* 1/3! */
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    return p * nn_pow2i((int32_t)n);                  /* n in [-126, 127] */
}

NN_FN float nn_expf(float x) {
    const float xc = fminf(fmaxf(x, -87.0f), 88.0f);  /* NaN -> -87 (replaced below) */
    float y = nn_expf_core(xc);
    y = x > 88.72283935546875f ? nn_i2f(0x7f800000) : y;
    return x != x ? x : y;
}

/*
 * nn_rcp1f: 1/d for d in [1, 2^120], <= ~1 ulp: integer first guess (relative error < 12.5 %) and
 * three Newton steps e = 1 - d y, y += y e in fmaf (error squares each step: 1.6e-2, 2.4e-4,
 * 5.9e-8 before the last rounding). Deterministic IEEE operations only, so host and GPU agree.
 */
NN_FN float nn_rcp1f(float d) {
    float y = nn_i2f(0x7EF311C3 - nn_f2i(d));
    float e = fmaf(-d, y, 1.0f);
    y = fmaf(y, e, y);
    e = fmaf(-d, y, 1.0f);
    y = fmaf(y, e, y);
    e = fmaf(-d, y, 1.0f);
    return fmaf(y, e, y);
}

/* sigmoid as torch.sigmoid defines it (src/captioning/nets.py:117): 1 / (1 + e^-x); the argument is
 * clamped to [-80, 80] (sigmoid there is 1 - 2^-115 .. 2^-115 off its limit) so 1 + e^-x stays in the
 * reciprocal's range */
NN_FN float nn_sigmoidf(float x) {
    const float xc = fminf(fmaxf(x, -80.0f), 80.0f);   /* NaN -> -80 (replaced below) */
    const float y = nn_rcp1f(1.0f + nn_expf_core(-xc)); /* = nn_expf(-xc): -xc is in range */
    return x != x ? x : y;
}

/*
 * nn_tanhf: odd; |x| < 0.6 -> x * P(x^2) (least-squares fit of tanh(x)/x in double,
 * abs err 3.6e-10 before fp32 rounding), else 1 - 2/(e^{2|x|} + 1) (exactly 1 past 9.5).
 * Both branches are evaluated and one is selected (branch-free, as nn_expf).
 */
NN_FN float nn_tanhf(float x) {
    const float a = x < 0.0f ? -x : x;
    const float u = x * x;
    float p = 0.0022306744940578938f;
    p = fmaf(p, u, -0.008266338147222996f);
    p = fmaf(p, u, 0.021733924746513367f);
    p = fmaf(p, u, -0.05395231395959854f);
    p = fmaf(p, u, 0.13333244621753693f);
    p = fmaf(p, u, -0.3333333134651184f);
    p = fmaf(p, u, 1.0f);
    const float small = x * p;
    const float ac = fminf(a, 9.5f);                  /* e^19 + 1 < 2^28: in the reciprocal's range; */
    float y = 1.0f - 2.0f * nn_rcp1f(nn_expf_core(2.0f * ac) + 1.0f);   /* NaN -> 9.5, replaced below */
    /* past 9.5 the formula already gives exactly 1: 2 / (e^19 + 1) < ulp(1) / 2 below 1 */
    y = x < 0.0f ? -y : y;
    y = a < 0.6f ? small : y;
    return x != x ? x : y;
}

/*
 * LSTM cell element (src/captioning/nets.py:113-132 with vbn=layer_n=false):
 *   c' = f*c + i*max(g1,g2) ; h' = o * tanh(c')      (each product/sum rounded separately)
 * s_* are the pre-activation gate sums.
 */
NN_FN void nn_lstm_cell(float s_in, float s_forget, float s_out, float s_g1, float s_g2,
                        float c, float* c_new, float* h_new) {
    float ig = nn_sigmoidf(s_in);
    float fg = nn_sigmoidf(s_forget);
    float og = nn_sigmoidf(s_out);
    float g = s_g1 > s_g2 ? s_g1 : s_g2;     /* torch.max(a, b): NaN-free inputs */
    float fc = fg * c;                       /* both builds use -ffp-contract=off: the two */
    float igv = ig * g;                      /* products stay unfused, as in torch         */
    float cn = fc + igv;
    *c_new = cn;
    *h_new = og * nn_tanhf(cn);
}

/* ---- noise-table index rule (the contract that replaces shipping 11 MB noise vectors,
 *      src/algorithm/nic_nes/nic_nes_worker.py:156-161) ---------------------------------- */
NN_FN uint64_t nn_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define NN_NOISE_ALIGN 64u   /* slice starts are multiples of 64 floats (256 B) */

/* idx = 64 * (splitmix64(seed ^ (iter<<32 | member)) mod n_slots), n_slots = floor((T-D)/64)+1 */
NN_FN uint64_t nn_noise_index(uint64_t seed, uint64_t iteration, uint64_t member,
                              uint64_t table_len, uint64_t dim) {
    uint64_t n_slots = (table_len - dim) / NN_NOISE_ALIGN + 1u;
    uint64_t h = nn_splitmix64(seed ^ ((iteration << 32) | (member & 0xffffffffull)));
    return (h % n_slots) * NN_NOISE_ALIGN;
}

/*
 * Dot-product order ("k permutation"). The engine's dense products are fp32 fma chains
 * acc = fmaf(w[k], x[k], acc) started from the bias, visiting k in this order inside each
 * 32-wide chunk: for j = 0..15: k0 = (j&3) + 8*(j>>2), then k0 + 4.  It is the order in
 * which v_mfma_f32_32x32x2_f32 consumes an operand held in the 32x32 accumulator layout
 * (half 0 lanes: rows (r&3)+8(r>>2), half 1 lanes: +4), so the GPU needs no transpose.
 */
NN_FN int nn_kperm(int pos) {
    int chunk = pos >> 5, w = pos & 31, j = w >> 1, half = w & 1;
    return (chunk << 5) + (j & 3) + 8 * (j >> 2) + 4 * half;
}

#endif /* NICNES_MATH_H */
