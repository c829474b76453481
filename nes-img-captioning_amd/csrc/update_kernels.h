// Internal (non-ABI) interface of the master-side kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct AdamParams {
    double* theta64;        // fp64 master theta (updated in place)
    float* theta32;         // fp32 evaluation copy (written)
    double* m;
    double* v;
    const float* gsum;      // sum over members of w_i * delta_i (all ranks), fp32
    double* partials;       // [2 * nicnes_adam_blocks(dim)]
    int64_t dim;
    float two_f;            // 2F: ranked_fitnesses.size
    int32_t theta_is_fp32;  // 1 before the first update (reference theta is still fp32)
    double l2coeff;
    float l2coeff32;
    double a;               // stepsize * sqrt(1 - b2^t) / (1 - b1^t), computed on the host
    double beta1, beta2, one_minus_beta1, one_minus_beta2, epsilon;
    float one_minus_beta1_32, one_minus_beta2_32;
    int32_t kind;           // 0 Adam, 1 SGD with momentum (beta1 = momentum)
    double neg_stepsize;    // SGD: -stepsize
    const double* globalg;  // non-null: Optimizer.update(globalg) form (gsum / l2coeff unused)
    int32_t g_is_fp32;      // globalg was an fp32 array: (1 - b) * g' products stay fp32 (NEP 50)
    const int32_t* fault;   // nullable: the handle's decode counters (decode_fault: the step is skipped)
    double* skip_out;       // 1.0 when this step was skipped (a fault), 0.0 when applied
};

extern "C" hipError_t nicnes_launch_noise_index(uint64_t seed, uint64_t iteration, uint64_t member0, int count,
                                                uint64_t table_len, uint64_t dim, uint64_t* out, hipStream_t s);
extern "C" hipError_t nicnes_launch_sample_draws(uint64_t seed, uint64_t iteration, uint64_t member0, int count, int B,
                                                 int T, double* out, hipStream_t s);
extern "C" hipError_t nicnes_launch_noise_vectors(const float* noise, const uint64_t* idx, int count, int64_t dim,
                                                  float sigma, float* out, hipStream_t s);
extern "C" hipError_t nicnes_launch_mutate(const float* noise, const uint64_t* idx, int count, int64_t dim, float sigma,
                                           const float* vec, int mode, float* out, int64_t out_stride, hipStream_t s);
extern "C" hipError_t nicnes_launch_proportional(const float* theta, int64_t n, float mean_abs, float* out,
                                                 hipStream_t s);
extern "C" hipError_t nicnes_launch_count_zeros(const float* theta, int64_t n, unsigned long long* out, hipStream_t s);
extern "C" hipError_t nicnes_launch_iota_stride(uint64_t* out, int n, uint64_t stride, hipStream_t s);
extern "C" size_t nicnes_rank_scratch_pairs(int n);
extern "C" hipError_t nicnes_launch_rank(const double* fit, int n, uint64_t* skey, uint32_t* sidx, double* cr_out,
                                         float* w_out, hipStream_t s);
// mode 0: delta = fp32(sigma * z); 1: delta / vec[j]; 2: delta * vec[j] (safe / proportional mutations)
// fault (nullable): the handle's decode counters; after a faulted decode every gsum entry is NaN
extern "C" hipError_t nicnes_launch_grad(const float* noise, const uint64_t* idx, const float* w, int count, float sigma,
                                         int64_t dim, const float* vec, int mode, float* gsum, hipStream_t s,
                                         const int32_t* fault = nullptr);
extern "C" int nicnes_adam_blocks(int64_t dim);
extern "C" hipError_t nicnes_launch_adam(const AdamParams* p, double* norms_out, hipStream_t s);
// out[i] = fp32(sigma * in[i]), i < n (the decode's sigma-scaled noise table)
extern "C" hipError_t nicnes_launch_scale(const float* in, float* out, uint64_t n, float sigma, hipStream_t s);
