// sensitivity.hip -- the SM-G-SUM sensitivity of safe mutations on the GPU.
//
// Replaces the per-task host computation of
//   Sensitivity._calc_sum_sensitivity (/root/reference/src/algorithm/safe_mutations.py:86-110) on
//   CaptionModel.forward_for_sensitivity (/root/reference/src/captioning/nets.py:22-70):
// O = [Bs, K] grouped log-prob norms after L = 5 greedy steps (vocabulary zero-padded to a multiple of
// split = 100, K groups, each reduced to its 2-norm); the reference runs K backward passes, one per
// column k of O summed over the batch, and returns s_j = sqrt(sum_k (dO_k / dtheta_j)^2) / Bs.
//
// Here the K backward passes run at once: the K output seeds dZ_k = d(sum_b O[b, k]) / d logits are
// formed in one kernel, and every backward product is one strided-batched GEMM over k (rocBLAS, fp32:
// plain library GEMMs), with the per-k gradients G[k, :] laid out in the flat theta order;
// one last pass reduces sqrt(sum_k G[k, j]^2) / Bs and applies the clamp of calc_sensitivity
// (safe_mutations.py:63-65). The greedy tokens of the forward come from the engine's bit-exact decode
// (unmasked, as forward_for_sensitivity feeds argmax back without the finished mask); the forward
// activations the backward needs are recomputed here in fp32. Agreement with the reference's vector is
// to a stated tolerance (fp32 sums in another order), not bit for bit.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <stdint.h>

#include "sensitivity.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// Y[r, c] += b1[c] (+ b2[c])
__global__ void sens_bias_rows(float* Y, const float* b1, const float* b2, int rows, int cols) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)rows * cols) return;
    const int c = (int)(i % cols);
    Y[i] += b1[c] + (b2 ? b2[c] : 0.f);
}

// X[b, :] = emb[token, :], token = tok[b * stride + col] (col < 0: the BOS token 0)
__global__ void sens_embed_gather(float* X, const float* emb, const int32_t* tok, int stride, int col, int Bs, int E) {
    const int b = blockIdx.x, e = threadIdx.x;
    if (b >= Bs || e >= E) return;
    const int t = col < 0 ? 0 : tok[(int64_t)b * stride + col];
    X[(int64_t)b * E + e] = emb[(int64_t)t * E + e];
}

// LSTMCore without vbn / layer norm (nets.py:98-134): S = [Bs, 5R] gate sums (i, f, o, g1, g2)
__global__ void sens_cell_fwd(const float* S, const float* Cprev, float* C, float* H, int Bs, int R) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Bs * R) return;
    const int64_t b = i / R;
    const int r = (int)(i % R);
    const float* s = S + b * 5 * R;
    const float ig = sigm(s[r]), fg = sigm(s[R + r]), og = sigm(s[2 * R + r]);
    const float g = fmaxf(s[3 * R + r], s[4 * R + r]);
    const float c = fg * (Cprev ? Cprev[i] : 0.f) + ig * g;
    C[i] = c;
    H[i] = og * tanhf(c);
}

// one block per row: LP = log_softmax(Z) (nets.py:202)
__global__ void sens_logsoftmax(const float* Z, float* LP, int V) {
    __shared__ float red[256];
    const float* z = Z + (int64_t)blockIdx.x * V;
    float* lp = LP + (int64_t)blockIdx.x * V;
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
    for (int v = threadIdx.x; v < V; v += blockDim.x) lp[v] = (z[v] - m) - lse;
}

// block (b, k): the seed of output column k for row b through the 2-norm and log_softmax:
// dZ[k, b, v] = [v in group k] lp[b, v] / g_bk - exp(lp[b, v]) * sum_{u in group k} lp[b, u] / g_bk
__global__ void sens_seed(const float* LP, float* dZ, int Bs, int V, int split) {
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
    const float g = sqrtf(red[0][0]);
    const float inv = g > 0.f ? 1.f / g : 0.f;                   // an all-padding group: no gradient
    const float S = red[1][0] * inv;
    float* d = dZ + ((int64_t)k * Bs + b) * V;
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
        const float own = (v >= v0 && v < v0 + split) ? lp[v] * inv : 0.f;
        d[v] = own - expf(lp[v]) * S;
    }
}

// out[k][c] (+)= sum_r X[k][r][c], optionally into a second destination too
__global__ void sens_colsum(const float* X, int rows, int cols, int64_t sX, float* out, float* out2, int64_t sO,
                            int accumulate) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, k = blockIdx.y;
    if (c >= cols) return;
    const float* x = X + (int64_t)k * sX + c;
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += x[(int64_t)r * cols];
    float* o = out + (int64_t)k * sO + c;
    *o = accumulate ? *o + s : s;
    if (out2) {
        float* o2 = out2 + (int64_t)k * sO + c;
        *o2 = accumulate ? *o2 + s : s;
    }
}

// LSTM cell backward for the K seeds at once: dH, dC [K, Bs, R] -> dS [K, Bs, 5R], dC <- d c_prev.
// torch.max(a, b) (nets.py:121) splits the gradient of an exact tie in halves (aten maximum backward).
__global__ void sens_cell_bwd(const float* dH, float* dC, const float* S, const float* C, const float* Cprev,
                              float* dS, int K, int Bs, int R) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)K * Bs * R) return;
    const int64_t kb = i / R;                                    // k * Bs + b
    const int r = (int)(i % R);
    const int64_t b = kb % Bs;
    const float* s = S + b * 5 * R;
    const float ig = sigm(s[r]), fg = sigm(s[R + r]), og = sigm(s[2 * R + r]);
    const float g1 = s[3 * R + r], g2 = s[4 * R + r], g = fmaxf(g1, g2);
    const float c = C[b * R + r], cp = Cprev ? Cprev[b * R + r] : 0.f;
    const float th = tanhf(c);
    const float dh = dH[i];
    const float dc = dC[i] + dh * og * (1.f - th * th);
    const float dog = dh * th;
    float* d = dS + kb * 5 * R;
    d[r] = dc * g * ig * (1.f - ig);
    d[R + r] = dc * cp * fg * (1.f - fg);
    d[2 * R + r] = dog * og * (1.f - og);
    const float dg = dc * ig;
    d[3 * R + r] = g1 > g2 ? dg : (g1 == g2 ? 0.5f * dg : 0.f);
    d[4 * R + r] = g2 > g1 ? dg : (g1 == g2 ? 0.5f * dg : 0.f);
    dC[i] = dc * fg;
}

// embedding rows: G[k, off + token(b) * E + e] += dX[k, b, e] (token = tok[b * stride + col], col < 0: BOS)
__global__ void sens_embed_scatter(const float* dX, const int32_t* tok, int stride, int col, float* G, int64_t D,
                                   int64_t off, int K, int Bs, int E) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)K * Bs * E) return;
    const int e = (int)(i % E);
    const int64_t kb = i / E;
    const int b = (int)(kb % Bs), k = (int)(kb / Bs);
    const int t = col < 0 ? 0 : tok[(int64_t)b * stride + col];
    atomicAdd(G + (int64_t)k * D + off + (int64_t)t * E + e, dX[i]);
}

// s_j = sqrt(sum_k G[k, j]^2) / Bs, then s < underflow -> underflow, s /= underflow (safe_mutations.py:63-65)
__global__ void sens_reduce(const float* G, int K, int64_t D, float inv_bs, float underflow, float* out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= D) return;
    float acc = 0.f;
    for (int k = 0; k < K; ++k) {
        const float g = G[(int64_t)k * D + j];
        acc += g * g;
    }
    float s = sqrtf(acc) * inv_bs;
    if (underflow > 0.f) {
        s = s < underflow ? underflow : s;
        s /= underflow;
    }
    out[j] = s;
}

inline unsigned blocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

struct SensWork {
    rocblas_handle blas = nullptr;
    int Bs = 0, K = 0;
    int64_t D = 0;
    float* X = nullptr;     // [L + 1][Bs, E] cell inputs
    float* S = nullptr;     // [L + 1][Bs, 5R] gate sums
    float* C = nullptr;     // [L + 1][Bs, R]
    float* H = nullptr;     // [L + 1][Bs, R]
    float* Z = nullptr;     // [Bs, V] logits -> log-probs in LP
    float* LP = nullptr;
    float* dZ = nullptr;    // [K, Bs, V]
    float* G = nullptr;     // [K, D] per-seed gradients, flat theta order
    float* dH = nullptr;    // [K, Bs, R]
    float* dC = nullptr;    // [K, Bs, R]
    float* dS = nullptr;    // [K, Bs, 5R]
    float* dX = nullptr;    // [K, Bs, E]
};

namespace {

void free_all(SensWork* w) {
    float* ps[] = {w->X, w->S, w->C, w->H, w->Z, w->LP, w->dZ, w->G, w->dH, w->dC, w->dS, w->dX};
    for (float* p : ps)
        if (p) (void)hipFree(p);
    w->X = w->S = w->C = w->H = w->Z = w->LP = w->dZ = w->G = w->dH = w->dC = w->dS = w->dX = nullptr;
    w->Bs = w->K = 0;
    w->D = 0;
}

hipError_t grow(SensWork* w, const SensParams* p) {
    if (w->Bs >= p->Bs && w->K >= p->K && w->D == p->D) return hipSuccess;
    free_all(w);
    const int64_t L1 = p->L + 1, Bs = p->Bs, K = p->K, E = p->E, R = p->R, V = p->V1;
    const struct { float** q; int64_t n; } a[] = {
        {&w->X, L1 * Bs * E}, {&w->S, L1 * Bs * 5 * R}, {&w->C, L1 * Bs * R}, {&w->H, L1 * Bs * R},
        {&w->Z, Bs * V}, {&w->LP, Bs * V}, {&w->dZ, K * Bs * V}, {&w->G, K * p->D},
        {&w->dH, K * Bs * R}, {&w->dC, K * Bs * R}, {&w->dS, K * Bs * 5 * R}, {&w->dX, K * Bs * E}};
    for (const auto& x : a) {
        hipError_t e = hipMalloc((void**)x.q, (size_t)x.n * sizeof(float));
        if (e != hipSuccess) {
            free_all(w);
            return e;
        }
    }
    w->Bs = p->Bs;
    w->K = p->K;
    w->D = p->D;
    return hipSuccess;
}

// row-major C[b] (M x N, ldc) = op(A[b]) (M x K) . op(B[b]) (K x N) + beta C[b], via the column-major
// product C^T = op(B)^T op(A)^T
rocblas_status gemm_rm(rocblas_handle hb, bool tA, bool tB, int M, int N, int Kd, const float* A, int lda,
                       int64_t sA, const float* B, int ldb, int64_t sB, float beta, float* C, int ldc, int64_t sC,
                       int batch) {
    const float one = 1.f;
    return rocblas_sgemm_strided_batched(hb, tB ? rocblas_operation_transpose : rocblas_operation_none,
                                         tA ? rocblas_operation_transpose : rocblas_operation_none, N, M, Kd, &one, B,
                                         ldb, sB, A, lda, sA, &beta, C, ldc, sC, batch);
}

}  // namespace

extern "C" SensWork* nicnes_sens_create() { return new SensWork(); }

extern "C" void nicnes_sens_destroy(SensWork* w) {
    if (!w) return;
    free_all(w);
    if (w->blas) (void)rocblas_destroy_handle(w->blas);
    delete w;
}

extern "C" int nicnes_sens_run(SensWork* w, const SensParams* p, hipStream_t st) {
    if (!w || !p || p->Bs < 1 || p->L < 1 || p->split < 1) return 1;
    if (!w->blas) {
        if (rocblas_create_handle(&w->blas) != rocblas_status_success) return 2;
    }
    if (rocblas_set_stream(w->blas, st) != rocblas_status_success) return 2;
    if (grow(w, p) != hipSuccess) return 3;
    const int Bs = p->Bs, E = p->E, R = p->R, F = p->F, V = p->V1, K = p->K, L = p->L;
    const int64_t D = p->D;
    const float* th = p->theta;
    const float *Wimg = th + p->off_img_w, *bimg = th + p->off_img_b, *Wemb = th + p->off_emb_w;
    const float *Wl = th + p->off_log_w, *bl = th + p->off_log_b;
    const float *Wi = th + p->off_i2h_w, *bi = th + p->off_i2h_b, *Wh = th + p->off_h2h_w, *bh = th + p->off_h2h_b;
    auto Xs = [&](int i) { return w->X + (int64_t)i * Bs * E; };
    auto Ss = [&](int i) { return w->S + (int64_t)i * Bs * 5 * R; };
    auto Cs = [&](int i) { return w->C + (int64_t)i * Bs * R; };
    auto Hs = [&](int i) { return w->H + (int64_t)i * Bs * R; };
    // token fed to cell i (1..L): BOS for i = 1, else the greedy token of logit step i - 1
    auto tok_col = [&](int i) { return i == 1 ? -1 : i - 2; };
    rocblas_status bs = rocblas_status_success;
    auto G = [&](rocblas_status s) { if (s != rocblas_status_success) bs = s; };

    // ---- forward: image cell, then L token cells (forward_for_sensitivity, nets.py:48-64)
    G(gemm_rm(w->blas, false, true, Bs, E, F, p->fc, F, 0, Wimg, F, 0, 0.f, Xs(0), E, 0, 1));   // img_embed
    hipLaunchKernelGGL(sens_bias_rows, dim3(blocks((int64_t)Bs * E, 256)), dim3(256), 0, st, Xs(0), bimg,
                       (const float*)nullptr, Bs, E);
    for (int i = 0; i <= L; ++i) {
        if (i >= 1)
            hipLaunchKernelGGL(sens_embed_gather, dim3(Bs), dim3(E), 0, st, Xs(i), Wemb, p->tok, p->tok_stride,
                               tok_col(i), Bs, E);
        G(gemm_rm(w->blas, false, true, Bs, 5 * R, E, Xs(i), E, 0, Wi, E, 0, 0.f, Ss(i), 5 * R, 0, 1));
        if (i >= 1) G(gemm_rm(w->blas, false, true, Bs, 5 * R, R, Hs(i - 1), R, 0, Wh, R, 0, 1.f, Ss(i), 5 * R, 0, 1));
        hipLaunchKernelGGL(sens_bias_rows, dim3(blocks((int64_t)Bs * 5 * R, 256)), dim3(256), 0, st, Ss(i), bi, bh,
                           Bs, 5 * R);
        hipLaunchKernelGGL(sens_cell_fwd, dim3(blocks((int64_t)Bs * R, 256)), dim3(256), 0, st, Ss(i),
                           i ? (const float*)Cs(i - 1) : (const float*)nullptr, Cs(i), Hs(i), Bs, R);
    }
    G(gemm_rm(w->blas, false, true, Bs, V, R, Hs(L), R, 0, Wl, R, 0, 0.f, w->Z, V, 0, 1));        // logit
    hipLaunchKernelGGL(sens_bias_rows, dim3(blocks((int64_t)Bs * V, 256)), dim3(256), 0, st, w->Z, bl,
                       (const float*)nullptr, Bs, V);
    hipLaunchKernelGGL(sens_logsoftmax, dim3(Bs), dim3(256), 0, st, w->Z, w->LP, V);

    // ---- the K backward passes at once
    hipLaunchKernelGGL(sens_seed, dim3(Bs, K), dim3(128), 0, st, w->LP, w->dZ, Bs, V, p->split);
    if (hipMemsetAsync(w->G, 0, (size_t)K * D * sizeof(float), st) != hipSuccess) return 4;
    const int64_t sZ = (int64_t)Bs * V;
    // logit.weight / .bias, dh of the last cell
    G(gemm_rm(w->blas, true, false, V, R, Bs, w->dZ, V, sZ, Hs(L), R, 0, 0.f, w->G + p->off_log_w, R, D, K));
    hipLaunchKernelGGL(sens_colsum, dim3(blocks(V, 256), K), dim3(256), 0, st, w->dZ, Bs, V, sZ, w->G + p->off_log_b,
                       (float*)nullptr, D, 0);
    G(gemm_rm(w->blas, false, false, Bs, R, V, w->dZ, V, sZ, Wl, R, 0, 0.f, w->dH, R, (int64_t)Bs * R, K));
    if (hipMemsetAsync(w->dC, 0, (size_t)K * Bs * R * sizeof(float), st) != hipSuccess) return 4;
    const int64_t sS = (int64_t)Bs * 5 * R, sX = (int64_t)Bs * E, sH = (int64_t)Bs * R;
    for (int i = L; i >= 0; --i) {
        hipLaunchKernelGGL(sens_cell_bwd, dim3(blocks((int64_t)K * Bs * R, 256)), dim3(256), 0, st, w->dH, w->dC, Ss(i),
                           Cs(i), i ? (const float*)Cs(i - 1) : (const float*)nullptr, w->dS, K, Bs, R);
        G(gemm_rm(w->blas, true, false, 5 * R, E, Bs, w->dS, 5 * R, sS, Xs(i), E, 0, 1.f, w->G + p->off_i2h_w, E, D, K));
        if (i >= 1)
            G(gemm_rm(w->blas, true, false, 5 * R, R, Bs, w->dS, 5 * R, sS, Hs(i - 1), R, 0, 1.f, w->G + p->off_h2h_w,
                      R, D, K));
        hipLaunchKernelGGL(sens_colsum, dim3(blocks(5 * R, 256), K), dim3(256), 0, st, w->dS, Bs, 5 * R, sS,
                           w->G + p->off_i2h_b, w->G + p->off_h2h_b, D, 1);
        G(gemm_rm(w->blas, false, false, Bs, E, 5 * R, w->dS, 5 * R, sS, Wi, E, 0, 0.f, w->dX, E, sX, K));
        if (i >= 1) {
            G(gemm_rm(w->blas, false, false, Bs, R, 5 * R, w->dS, 5 * R, sS, Wh, R, 0, 0.f, w->dH, R, sH, K));
            hipLaunchKernelGGL(sens_embed_scatter, dim3(blocks((int64_t)K * Bs * E, 256)), dim3(256), 0, st, w->dX,
                               p->tok, p->tok_stride, tok_col(i), w->G, D, p->off_emb_w, K, Bs, E);
        } else {
            G(gemm_rm(w->blas, true, false, E, F, Bs, w->dX, E, sX, p->fc, F, 0, 0.f, w->G + p->off_img_w, F, D, K));
            hipLaunchKernelGGL(sens_colsum, dim3(blocks(E, 256), K), dim3(256), 0, st, w->dX, Bs, E, sX,
                               w->G + p->off_img_b, (float*)nullptr, D, 0);
        }
    }
    hipLaunchKernelGGL(sens_reduce, dim3(blocks(D, 256)), dim3(256), 0, st, w->G, K, D, 1.f / (float)Bs, p->underflow,
                       p->out);
    if (bs != rocblas_status_success) return 5;
    return hipGetLastError() == hipSuccess ? 0 : 6;
}
