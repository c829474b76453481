// update_kernels.hip -- master side of one NIC-NES iteration on gfx950.
//
//   noise indices          new contract replacing the shipped noise vectors
//                          (nic_nes_worker.py:142,156-161; include/nicnes_math.h nn_noise_index)
//   centred ranks          NESMaster.compute_ranks / compute_centered_ranks (nic_nes_master.py:184-205),
//                          stable (value, index) order
//   weighted noise sum     NESMaster.gradient_estimate + batched_weighted_sum (nic_nes_master.py:170-221),
//                          delta_i re-read from the table, fp64 accumulation in member order
//   Adam                   Optimizer.update + Adam._compute_step (optimizers.py:15-22,78-83) with the
//                          master's g' = -g + l2coeff*theta (nic_nes_master.py:126,133), fp64 state,
//                          evaluated with the same IEEE op sequence numpy uses (no fma contraction)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>

#include "../../include/nicnes_math.h"
#include "cider_kernel.h"
#include "update_kernels.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void nicnes_noise_index_kernel(uint64_t seed, uint64_t iteration, uint64_t member0, int count,
                                          uint64_t table_len, uint64_t dim, uint64_t* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) out[i] = nn_noise_index(seed, iteration, member0 + (uint64_t)i, table_len, dim);
}

// ---- centred ranks: rank_i = #{j : (x_j, j) < (x_i, i)} over the ravelled (P, 2) fitness -----
// The reference sorts with numpy's default argsort (compute_ranks, nic_nes_master.py:196-205); the
// engine's order is the stable one, (value, index), identical whenever values are distinct. Values
// map to an order-preserving uint64 (-0.0 as +0.0, every NaN as one NaN sorting last, as numpy's
// argsort places NaN). Pass 1: each workgroup bitonic-sorts a chunk of RANK_CHUNK (key, index)
// pairs in LDS. Pass 2: a pair's rank is the sum over chunks of its lower bound in that chunk
// (binary search); keys are unique with the index, so this is the stable rank. Any population size.
#define RANK_CHUNK 2048

__device__ __forceinline__ uint64_t rank_key(double x) {
    if (x != x) x = __builtin_nan("");                      // one canonical (positive) NaN: last
    if (x == 0.0) x = 0.0;                                  // -0.0 == 0.0
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ bool pair_less(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
    return ka < kb || (ka == kb && ia < ib);
}

__global__ __launch_bounds__(1024) void nicnes_rank_sort_kernel(const double* fit, int n, uint64_t* skey, uint32_t* sidx) {
    __shared__ uint64_t k[RANK_CHUNK];
    __shared__ uint32_t ix[RANK_CHUNK];
    const int base = blockIdx.x * RANK_CHUNK;
    for (int e = threadIdx.x; e < RANK_CHUNK; e += blockDim.x) {
        const int g = base + e;
        k[e] = g < n ? rank_key(fit[g]) : ~0ull;            // padding sorts after every real pair
        ix[e] = g < n ? (uint32_t)g : 0xffffffffu;
    }
    __syncthreads();
    for (int size = 2; size <= RANK_CHUNK; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const int t = threadIdx.x;                      // one compare-exchange per thread
            const int a = 2 * t - (t & (stride - 1));
            const int b = a + stride;
            const bool up = (a & size) == 0;
            const uint64_t ka = k[a], kb = k[b];
            const uint32_t ia = ix[a], ib = ix[b];
            if (pair_less(kb, ib, ka, ia) == up) {
                k[a] = kb; k[b] = ka;
                ix[a] = ib; ix[b] = ia;
            }
            __syncthreads();
        }
    }
    for (int e = threadIdx.x; e < RANK_CHUNK; e += blockDim.x) {
        skey[base + e] = k[e];
        sidx[base + e] = ix[e];
    }
}

// n <= RANK_CHUNK (every population up to 1024 members): no sort. Workgroup g holds all n keys in LDS and ranks
// its 32 entries (16 members): 8 groups of 32 lanes count the pairs below each entry over an eighth of the keys
// each, then the counts are added. The same stable rank as the two passes below, in one launch of n / 32
// workgroups (round 5: the sort pass and the search pass took 29.5 us per iteration at P = 64, 31 at P = 512)
#define RANK_SMALL_E 32
#define RANK_SMALL_G (256 / RANK_SMALL_E)
__global__ __launch_bounds__(256) void nicnes_rank_small_kernel(const double* fit, int n, double* cr_out, float* w_out) {
    __shared__ uint64_t k[RANK_CHUNK];
    __shared__ int cnt[RANK_SMALL_G][RANK_SMALL_E];
    __shared__ double cr[RANK_SMALL_E];
    for (int e = threadIdx.x; e < n; e += blockDim.x) k[e] = rank_key(fit[e]);
    __syncthreads();
    const int l = threadIdx.x % RANK_SMALL_E, g = threadIdx.x / RANK_SMALL_E;
    const int e = blockIdx.x * RANK_SMALL_E + l;
    if (e < n) {
        const uint64_t ke = k[e];
        const int j0 = g * n / RANK_SMALL_G, j1 = (g + 1) * n / RANK_SMALL_G;
        int r = 0;
#pragma unroll 4
        for (int j = j0; j < j1; ++j)             // every lane of the group reads the same key: an LDS broadcast
            r += pair_less(k[j], (uint32_t)j, ke, (uint32_t)e) ? 1 : 0;
        cnt[g][l] = r;
    }
    __syncthreads();
    if (g == 0 && e < n) {
        int r = 0;
#pragma unroll
        for (int q = 0; q < RANK_SMALL_G; ++q) r += cnt[q][l];
        double y = (double)r;
        y /= (double)(n - 1);                      // y /= (x.size - 1)   (compute_centered_ranks)
        y -= 0.5;                                  // y -= .5
        cr[l] = y;
        if (cr_out) cr_out[e] = y;
    }
    __syncthreads();
    const int pl = threadIdx.x, p = blockIdx.x * (RANK_SMALL_E / 2) + pl;
    if (pl < RANK_SMALL_E / 2 && 2 * p < n)
        w_out[p] = (float)(cr[2 * pl] - cr[2 * pl + 1]);   // cr[:, 0] - cr[:, 1], then fp32 (gradient_estimate)
}

__device__ __forceinline__ int chunk_lower_bound(const uint64_t* key, const uint32_t* idx, uint64_t kq, uint32_t iq) {
    int lo = 0, hi = RANK_CHUNK;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pair_less(key[mid], idx[mid], kq, iq)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void nicnes_rank_kernel(const double* fit, int n, const uint64_t* skey,
                                                          const uint32_t* sidx, double* cr_out, float* w_out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * p >= n) return;
    const int nchunks = (n + RANK_CHUNK - 1) / RANK_CHUNK;
    double cr[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int e = 2 * p + s;
        const uint64_t kq = rank_key(fit[e]);
        int rank = 0;
        for (int c = 0; c < nchunks; ++c)
            rank += chunk_lower_bound(skey + (size_t)c * RANK_CHUNK, sidx + (size_t)c * RANK_CHUNK, kq, (uint32_t)e);
        double y = (double)rank;
        y /= (double)(n - 1);                  // y /= (x.size - 1)   (compute_centered_ranks)
        y -= 0.5;                              // y -= .5
        cr[s] = y;
        if (cr_out) cr_out[e] = y;
    }
    w_out[p] = (float)(cr[0] - cr[1]);         // cr[:, 0] - cr[:, 1], then fp32 (gradient_estimate)
}

// gsum[j] = fp32( sum_i w_i * delta_i[j] ), fp64 accumulation in member order, with
// delta_i[j] = fp32(sigma * z[idx_i + j]) transformed by the mutation MODE (0 none, 1 / v[j], 2 * v[j]):
// safe / proportional mutations are applied on the fly, the per-member deltas are never stored
template <int MODE>
__device__ __forceinline__ float grad_delta(float sigma, float z, float v) {
    const float d = sigma * z;
    return MODE == 1 ? d / v : (MODE == 2 ? d * v : d);
}

// A faulted decode on this handle (decode_fault) poisons the sum instead: every entry NaN, so the all-reduce
// carries the fault to every rank and each rank's optimizer step skips (nicnes_adam_kernel).
template <int MODE>
// (restrict, and the fault test at the store: no store may precede the loop's loads, so idx[i] and w[i] stay
// scalar loads and the loop keeps several members' rows in flight; with a NaN-store branch in front of the loop
// they became dependent vector loads, 0.88 -> 1.09 ms at P = 512)
__global__ __launch_bounds__(256) void nicnes_grad_kernel(const float* __restrict__ noise,
                                                          const uint64_t* __restrict__ idx, const float* __restrict__ w,
                                                          int count, float sigma, int64_t dim,
                                                          const float* __restrict__ vec, float* __restrict__ gsum,
                                                          const int32_t* __restrict__ fault) {
    const int64_t j4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (j4 >= dim) return;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const bool full = j4 + 4 <= dim;
    f32x4 v = {1.f, 1.f, 1.f, 1.f};
    if (MODE) {
        if (full) v = *reinterpret_cast<const f32x4*>(vec + j4);
        else
            for (int q = 0; q < 3; ++q)
                if (j4 + q < dim) v[q] = vec[j4 + q];
    }
    if (full) {
#pragma unroll 4
        for (int i = 0; i < count; ++i) {
            const f32x4 zz = *reinterpret_cast<const f32x4*>(noise + idx[i] + j4);
            const double wi = (double)w[i];
            a0 += wi * (double)grad_delta<MODE>(sigma, zz[0], v[0]);
            a1 += wi * (double)grad_delta<MODE>(sigma, zz[1], v[1]);
            a2 += wi * (double)grad_delta<MODE>(sigma, zz[2], v[2]);
            a3 += wi * (double)grad_delta<MODE>(sigma, zz[3], v[3]);
        }
    } else {
        for (int i = 0; i < count; ++i) {
            const float* z = noise + idx[i] + j4;
            const double wi = (double)w[i];
            a0 += wi * (double)grad_delta<MODE>(sigma, z[0], v[0]);
            if (j4 + 1 < dim) a1 += wi * (double)grad_delta<MODE>(sigma, z[1], v[1]);
            if (j4 + 2 < dim) a2 += wi * (double)grad_delta<MODE>(sigma, z[2], v[2]);
        }
    }
    if (decode_fault(fault)) a0 = a1 = a2 = a3 = __builtin_nan("");   // a faulted decode: NaN everywhere
    gsum[j4] = (float)a0;
    if (j4 + 1 < dim) gsum[j4 + 1] = (float)a1;
    if (j4 + 2 < dim) gsum[j4 + 2] = (float)a2;
    if (j4 + 3 < dim) gsum[j4 + 3] = (float)a3;
}

// one Adam step; partial sums of step^2 and theta_old^2 per block for the update ratio.
// No-op (theta, m, v untouched; ratio NaN) after a faulted decode: this handle's counters (p.fault), or a NaN
// first entry of the noise sum, which a faulted rank's nicnes_grad_kernel writes and the all-reduce spreads
__device__ __forceinline__ void adam_one(const AdamParams& p, int64_t j, double& s2, double& t2) {
    const double th = p.theta64[j];
    // globalg g' = -g + l2coeff * theta (nic_nes_master.py:311-318), or given directly
    // (Optimizer.update(globalg)). Before the first update theta, and so g', are fp32 arrays.
    float gp32 = 0.f;
    double gp64;
    if (p.globalg) {
        gp64 = p.globalg[j];
        gp32 = (float)gp64;
    } else {
        const float g = p.gsum[j] / p.two_f;             // gradient_est /= ranked_fitnesses.size (fp32)
        if (p.theta_is_fp32) {
            gp32 = -g + p.l2coeff32 * (float)th;
            gp64 = gp32;
        } else {
            gp64 = (double)(-g) + p.l2coeff * th;
        }
    }
    // numpy keeps python_float * fp32_array in fp32 (NEP 50): at the first update the
    // (1 - b) * g' products are fp32, added to the fp64 state (optimizers.py:45,81-82)
    double step;
    if (p.kind == 0) {                                   // Adam._compute_step, optimizers.py:78-83
        double m, v;
        if (p.g_is_fp32) {
            m = p.beta1 * p.m[j] + (double)(p.one_minus_beta1_32 * gp32);
            v = p.beta2 * p.v[j] + (double)(p.one_minus_beta2_32 * (gp32 * gp32));
        } else {
            m = p.beta1 * p.m[j] + p.one_minus_beta1 * gp64;
            v = p.beta2 * p.v[j] + p.one_minus_beta2 * (gp64 * gp64);
        }
        step = (-p.a * m) / (sqrt(v) + p.epsilon);
        p.m[j] = m;
        p.v[j] = v;
    } else {                                             // SGD._compute_step, optimizers.py:44-47
        const double v = p.g_is_fp32 ? p.beta1 * p.v[j] + (double)(p.one_minus_beta1_32 * gp32)
                                         : p.beta1 * p.v[j] + p.one_minus_beta1 * gp64;
        step = p.neg_stepsize * v;
        p.v[j] = v;
    }
    const double nt = th + step;
    p.theta64[j] = nt;
    p.theta32[j] = (float)nt;
    s2 += step * step;
    t2 += th * th;
}

// grid-stride over the parameters (ADAM_BLOCKS workgroups, so the fixed-order sum of the partials below reads
// 2 x ADAM_BLOCKS doubles instead of 2 x D / 256: 13 us of one workgroup's dependent loads at D = 2.87 M)
__global__ __launch_bounds__(256) void nicnes_adam_kernel(AdamParams p) {
    __shared__ double red[2][256];
    double s2 = 0.0, t2 = 0.0;
    const bool skip = decode_fault(p.fault) || (p.gsum != nullptr && p.gsum[0] != p.gsum[0]);
    // the explicit skip flag beside the norms (norms[2]): the host raises the fault error only when it is set,
    // not for a NaN ratio of an applied step (0/0 at theta = step = 0, or a NaN entry past index 0)
    if (blockIdx.x == 0 && threadIdx.x == 0) p.skip_out[0] = skip ? 1.0 : 0.0;
    if (skip) {
        s2 = t2 = __builtin_nan("");
    } else {
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < p.dim; j += stride) adam_one(p, j, s2, t2);
    }
    red[0][threadIdx.x] = s2;
    red[1][threadIdx.x] = t2;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        p.partials[2 * blockIdx.x] = red[0][0];
        p.partials[2 * blockIdx.x + 1] = red[1][0];
    }
}

// fixed-order sum of the per-block partials -> out[0] = |step|^2, out[1] = |theta_old|^2
__global__ __launch_bounds__(256) void nicnes_sum_partials_kernel(const double* partials, int nblocks, double* out) {
    __shared__ double red[2][256];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < nblocks; i += 256) {
        a += partials[2 * i];
        b += partials[2 * i + 1];
    }
    red[0][threadIdx.x] = a;
    red[1][threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            red[0][threadIdx.x] += red[0][threadIdx.x + o];
            red[1][threadIdx.x] += red[1][threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = red[0][0];
        out[1] = red[1][0];
    }
}

extern "C" hipError_t nicnes_launch_noise_index(uint64_t seed, uint64_t iteration, uint64_t member0, int count,
                                                uint64_t table_len, uint64_t dim, uint64_t* out, hipStream_t s) {
    if (count <= 0) return hipSuccess;
    hipLaunchKernelGGL(nicnes_noise_index_kernel, dim3((count + 255) / 256), dim3(256), 0, s, seed, iteration, member0,
                       count, table_len, dim, out);
    return hipGetLastError();
}

// the uniforms of a sampled decode (RandomState.choice's one random_sample per row and logit step,
// nets.py:220-224): u of (member member0 + k, sign s, row b, step t) from a counter-based hash of the
// noise seed, the iteration and those coordinates, 53-bit like numpy's random_sample; [count, 2, B, T]
__global__ void nicnes_sample_draws_kernel(uint64_t seed, uint64_t iteration, uint64_t member0, int count, int B,
                                           int T, double* out) {
    const int64_t n = (int64_t)count * 2 * B * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = i / (2 * (int64_t)B * T), r = i % (2 * (int64_t)B * T);
        const uint64_t key = nn_splitmix64(seed ^ 0x6a09e667f3bcc909ull ^ ((iteration << 32) | (member0 + (uint64_t)k)));
        const uint64_t x = nn_splitmix64(key ^ (uint64_t)r);
        out[i] = (double)(x >> 11) * (1.0 / 9007199254740992.0);
    }
}

extern "C" hipError_t nicnes_launch_sample_draws(uint64_t seed, uint64_t iteration, uint64_t member0, int count, int B,
                                                 int T, double* out, hipStream_t s) {
    const int64_t n = (int64_t)count * 2 * B * T;
    if (n <= 0) return hipSuccess;
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(nicnes_sample_draws_kernel, dim3(blocks), dim3(256), 0, s, seed, iteration, member0, count, B, T,
                       out);
    return hipGetLastError();
}

extern "C" size_t nicnes_rank_scratch_pairs(int n) { return (size_t)((n + RANK_CHUNK - 1) / RANK_CHUNK) * RANK_CHUNK; }

extern "C" hipError_t nicnes_launch_rank(const double* fit, int n, uint64_t* skey, uint32_t* sidx, double* cr_out,
                                         float* w_out, hipStream_t s) {
    if (n <= RANK_CHUNK) {
        hipLaunchKernelGGL(nicnes_rank_small_kernel, dim3((n + RANK_SMALL_E - 1) / RANK_SMALL_E), dim3(256), 0, s, fit, n,
                           cr_out, w_out);
        return hipGetLastError();
    }
    const int nchunks = (n + RANK_CHUNK - 1) / RANK_CHUNK;
    hipLaunchKernelGGL(nicnes_rank_sort_kernel, dim3(nchunks), dim3(RANK_CHUNK / 2), 0, s, fit, n, skey, sidx);
    hipLaunchKernelGGL(nicnes_rank_kernel, dim3((n / 2 + 255) / 256), dim3(256), 0, s, fit, n, skey, sidx, cr_out, w_out);
    return hipGetLastError();
}

extern "C" hipError_t nicnes_launch_grad(const float* noise, const uint64_t* idx, const float* w, int count, float sigma,
                                         int64_t dim, const float* vec, int mode, float* gsum, hipStream_t s,
                                         const int32_t* fault) {
    const int64_t n4 = (dim + 3) / 4;
    const dim3 grid((unsigned)((n4 + 255) / 256));
    if (mode == 1)
        hipLaunchKernelGGL(nicnes_grad_kernel<1>, grid, dim3(256), 0, s, noise, idx, w, count, sigma, dim, vec, gsum, fault);
    else if (mode == 2)
        hipLaunchKernelGGL(nicnes_grad_kernel<2>, grid, dim3(256), 0, s, noise, idx, w, count, sigma, dim, vec, gsum, fault);
    else
        hipLaunchKernelGGL(nicnes_grad_kernel<0>, grid, dim3(256), 0, s, noise, idx, w, count, sigma, dim, vec, gsum, fault);
    return hipGetLastError();
}

// delta_k = fp32(sigma * z[idx_k + j]) for k < count, j < dim: the vectors PolicyNet.evolve returns
// (src/algorithm/nets.py:101-102) rebuilt from the table, for the reference-format NESResult
// (nic_nes_worker.py:156-161). Coalesced over j, one row of the grid per member.
__global__ __launch_bounds__(256) void nicnes_noise_vectors_kernel(const float* noise, const uint64_t* idx, int64_t dim,
                                                                   float sigma, float* out) {
    const int k = blockIdx.y;
    const float* z = noise + idx[k];
    float* o = out + (size_t)k * dim;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < dim; j += (int64_t)gridDim.x * blockDim.x)
        o[j] = sigma * z[j];
}

extern "C" hipError_t nicnes_launch_noise_vectors(const float* noise, const uint64_t* idx, int count, int64_t dim,
                                                  float sigma, float* out, hipStream_t s) {
    hipLaunchKernelGGL(nicnes_noise_vectors_kernel, dim3(512, count), dim3(256), 0, s, noise, idx, dim, sigma, out);
    return hipGetLastError();
}

// Safe / proportional mutations (src/algorithm/nets.py:96-113): delta'_k = fp32(fp32(sigma * z) / vec)
// (mode 1: SM-G-SUM, SM-G-ABS, SM-VECTOR divide the noise by the sensitivity) or fp32(fp32(sigma * z) *
// vec) (mode 2: SM-PROPORTIONAL multiplies it by |theta|), IEEE division as torch's in-place /=.
// out row k at out + k * out_stride.
__device__ __forceinline__ float mutate1(float z, float sigma, float v, int mode) {
    const float d = sigma * z;
    return mode == 1 ? d / v : d * v;
}

// VEC: 4 consecutive parameters per thread and one 16-byte store (the member's table slice starts at any float:
// its loads stay dword-aligned 16-byte loads); the same per-element arithmetic as the scalar form
#ifndef MUTATE_NT
#define MUTATE_NT 1         // the delta' rows written with nontemporal stores (measured: 2.10 -> 1.97 ms at P = 512)
#endif
template <bool VEC>
__global__ __launch_bounds__(256) void nicnes_mutate_kernel(const float* noise, const uint64_t* idx, int64_t dim,
                                                            float sigma, const float* vec, int mode, float* out,
                                                            int64_t out_stride) {
    const int k = blockIdx.y;
    const float* z = noise + idx[k];
    float* o = out + (size_t)k * out_stride;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    int64_t j0 = 0;
    if constexpr (VEC) {
        const int64_t n4 = dim / 4;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += step) {
            f32x4 zv, r;
            __builtin_memcpy(&zv, z + 4 * i, 16);
            const f32x4 vv = reinterpret_cast<const f32x4*>(vec)[i];
#pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = mutate1(zv[e], sigma, vv[e], mode);
#if MUTATE_NT
            __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(o) + i);   // (the decode re-reads it from HBM)
#else
            reinterpret_cast<f32x4*>(o)[i] = r;
#endif
        }
        j0 = 4 * n4;
    }
    for (int64_t j = j0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < dim; j += step)
        o[j] = mutate1(z[j], sigma, vec[j], mode);
}

extern "C" hipError_t nicnes_launch_mutate(const float* noise, const uint64_t* idx, int count, int64_t dim, float sigma,
                                           const float* vec, int mode, float* out, int64_t out_stride, hipStream_t s) {
    if (out_stride % 4 == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)vec & 15) == 0)
        hipLaunchKernelGGL(nicnes_mutate_kernel<true>, dim3(512, count), dim3(256), 0, s, noise, idx, dim, sigma, vec,
                           mode, out, out_stride);
    else
        hipLaunchKernelGGL(nicnes_mutate_kernel<false>, dim3(512, count), dim3(256), 0, s, noise, idx, dim, sigma, vec,
                           mode, out, out_stride);
    return hipGetLastError();
}

// SM-PROPORTIONAL's vector (nets.py:108-112): |theta| with exact zeros (either sign) replaced by mean|theta|
__global__ __launch_bounds__(256) void nicnes_proportional_kernel(const float* theta, int64_t n, float mean_abs,
                                                                  float* out) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const float t = theta[j];
        out[j] = t == 0.f ? mean_abs : __builtin_fabsf(t);
    }
}

extern "C" hipError_t nicnes_launch_proportional(const float* theta, int64_t n, float mean_abs, float* out,
                                                 hipStream_t s) {
    hipLaunchKernelGGL(nicnes_proportional_kernel, dim3(2048), dim3(256), 0, s, theta, n, mean_abs, out);
    return hipGetLastError();
}

// exact zeros of theta (an integer count: the order of the atomic adds does not change it)
__global__ __launch_bounds__(256) void nicnes_count_zeros_kernel(const float* theta, int64_t n,
                                                                 unsigned long long* out) {
    unsigned long long c = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        c += theta[j] == 0.f ? 1ull : 0ull;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

extern "C" hipError_t nicnes_launch_count_zeros(const float* theta, int64_t n, unsigned long long* out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(nicnes_count_zeros_kernel, dim3(1024), dim3(256), 0, s, theta, n, out);
    return hipGetLastError();
}

// the sigma-scaled table the decode kernels read: out[i] = fp32(sigma * table[i]), each member's
// delta = fp32(sigma * z) (nets.py:102) then being a plain slice of it
__global__ __launch_bounds__(256) void nicnes_scale_kernel(const float* in, float* out, uint64_t n, float sigma) {
    const uint64_t n4 = n / 4;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        const f32x4 v = reinterpret_cast<const f32x4*>(in)[i];
        reinterpret_cast<f32x4*>(out)[i] = sigma * v;
    }
    const uint64_t t = 4 * n4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && t < n) out[t] = sigma * in[t];
}

extern "C" hipError_t nicnes_launch_scale(const float* in, float* out, uint64_t n, float sigma, hipStream_t s) {
    hipLaunchKernelGGL(nicnes_scale_kernel, dim3(2048), dim3(256), 0, s, in, out, n, sigma);
    return hipGetLastError();
}

__global__ void nicnes_iota_stride_kernel(uint64_t* out, int n, uint64_t stride) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint64_t)i * stride;
}

extern "C" hipError_t nicnes_launch_iota_stride(uint64_t* out, int n, uint64_t stride, hipStream_t s) {
    hipLaunchKernelGGL(nicnes_iota_stride_kernel, dim3((n + 255) / 256), dim3(256), 0, s, out, n, stride);
    return hipGetLastError();
}

#define ADAM_BLOCKS 2048
extern "C" int nicnes_adam_blocks(int64_t dim) { return (int)std::min<int64_t>((dim + 255) / 256, ADAM_BLOCKS); }

extern "C" hipError_t nicnes_launch_adam(const AdamParams* p, double* norms_out, hipStream_t s) {
    const int nb = nicnes_adam_blocks(p->dim);
    hipLaunchKernelGGL(nicnes_adam_kernel, dim3(nb), dim3(256), 0, s, *p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(nicnes_sum_partials_kernel, dim3(1), dim3(256), 0, s, p->partials, nb, norms_out);
    return hipGetLastError();
}
