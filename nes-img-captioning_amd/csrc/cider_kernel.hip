// cider_kernel.hip -- CIDEr-D fitness of every decoded candidate on gfx950.
//
// Replaces CaptPolicy.compute_ciders + CiderD.compute_score + the 'greedy' fitness
//   (/root/reference/src/captioning/policies.py:113-128,145-193, the unvendored
//    pyciderevalcap.ciderD scorer: SURVEY.md Appendix A.3; restated in oracle/cider_ref.py)
//
// Token strings are never built: a word of array_to_str() (tools/utils.py:34-40) is a token id,
// so an n-gram is packed exactly into a uint64 key  n<<56 | t0<<42 | t1<<28 | t2<<14 | t3
// (ids < 16384). One wave scores one (candidate, image) row: lane j owns n-gram slot j
// (n=1: lanes 0-15, n=2: 16-30, n=3: 31-44, n=4: 45-57), the first lane of each distinct
// n-gram carries its term frequency and tf-idf weight. Reference-side vectors are built once
// per batch (shared by every candidate) by nicnes_cook_refs_kernel. Accumulation is fp64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cider_kernel.h"

#define REF_SLOTS 64

__device__ __forceinline__ void slot_of_lane(int j, int& n, int& i) {
    if (j < 16) { n = 1; i = j; }
    else if (j < 31) { n = 2; i = j - 16; }
    else if (j < 45) { n = 3; i = j - 31; }
    else { n = 4; i = j - 45; }           // lanes 58..63: i >= 13, never valid for T = 16
}

// length of array_to_str(row): tokens up to and including the first 0
__device__ __forceinline__ int caption_len(const int32_t* row, int T) {
    int L = T;
    for (int k = T - 1; k >= 0; --k) if (row[k] == 0) L = k + 1;
    return L;
}

__device__ __forceinline__ uint64_t pack_ngram(const int32_t* row, int n, int i) {
    uint64_t key = (uint64_t)n << 56;
    for (int k = 0; k < n; ++k) key |= (uint64_t)(row[i + k] & 0x3fff) << (42 - 14 * k);
    return key;
}

__device__ __forceinline__ double df_lookup(const uint64_t* keys, const double* vals, int64_t n, uint64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < key) lo = mid + 1; else hi = mid;
    }
    return (lo < n && keys[lo] == key) ? vals[lo] : 0.0;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

struct NgramLane {
    uint64_t key;
    bool valid, first;
    int n;
    double vec;     // tf * (ref_len - log(max(1, df)))   (counts2vec)
};

// per-lane n-gram of one caption row, its tf over the row, first-occurrence flag and weight
__device__ __forceinline__ NgramLane ngram_lane(const int32_t* row, int T, int lane, const CiderTables& tb) {
    NgramLane g;
    const int L = caption_len(row, T);
    int i;
    slot_of_lane(lane, g.n, i);
    g.valid = (lane < 58) && (i + g.n <= L);
    g.key = g.valid ? pack_ngram(row, g.n, i) : 0ull;
    int tf = 0;
    bool first = g.valid;
    for (int o = 0; o < 64; ++o) {
        const uint64_t k2 = __shfl(g.key, o);
        const bool v2 = __shfl((int)g.valid, o) != 0;
        if (g.valid && v2 && k2 == g.key) {
            ++tf;
            if (o < lane) first = false;
        }
    }
    g.first = first;
    g.vec = 0.0;
    if (first) {
        const double df = df_lookup(tb.df_keys, tb.df_vals, tb.df_n, g.key);
        g.vec = (double)tf * (tb.ref_len - log(df > 1.0 ? df : 1.0));
    }
    return g;
}

// ---- per-batch reference vectors --------------------------------------------------------------
__global__ __launch_bounds__(256) void nicnes_cook_refs_kernel(const int32_t* ref_tokens, int n_refs, int T,
                                                               CiderTables tb) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= n_refs) return;
    const int32_t* row = ref_tokens + (size_t)r * T;
    const NgramLane g = ngram_lane(row, T, lane, tb);
    const uint64_t firsts = __ballot(g.first);
    const int rank = __popcll(firsts & ((1ull << lane) - 1ull));
    if (g.first) {
        tb.ref_keys[(size_t)r * REF_SLOTS + rank] = g.key;
        tb.ref_vec[(size_t)r * REF_SLOTS + rank] = g.vec;
    }
    double nrm[4];
#pragma unroll
    for (int n = 1; n <= 4; ++n) nrm[n - 1] = sqrt(wave_sum((g.first && g.n == n) ? g.vec * g.vec : 0.0));
    if (lane == 0) {
        tb.ref_count[r] = __popcll(firsts);
        const int L = caption_len(row, T);
        tb.ref_len2[r] = L > 1 ? L - 1 : 0;          // bigram count (counts2vec 'length' quirk)
#pragma unroll
        for (int n = 0; n < 4; ++n) tb.ref_norm[(size_t)r * 4 + n] = nrm[n];
    }
}

// ---- candidates: one workgroup per candidate, one wave per image row ---------------------------
__global__ __launch_bounds__(256) void nicnes_cider_kernel(const int32_t* seq, int B, int T, CiderTables tb,
                                                           const int32_t* img_ref_start, double* fitness_out) {
    __shared__ double row_score[1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cand = blockIdx.x;
    const double sigma2x2 = 2.0 * 6.0 * 6.0;
    for (int b = wave; b < B; b += 4) {
        const int32_t* row = seq + ((size_t)cand * B + b) * T;
        const NgramLane g = ngram_lane(row, T, lane, tb);
        double nh[4];
#pragma unroll
        for (int n = 1; n <= 4; ++n) nh[n - 1] = sqrt(wave_sum((g.first && g.n == n) ? g.vec * g.vec : 0.0));
        const int L = caption_len(row, T);
        const int len_h = L > 1 ? L - 1 : 0;
        double score[4] = {0.0, 0.0, 0.0, 0.0};
        const int r0 = img_ref_start[b], r1 = img_ref_start[b + 1];
        for (int r = r0; r < r1; ++r) {
            // vr[g] for this lane's n-gram (0 when the ref lacks it)
            const int cnt = tb.ref_count[r];
            double vr = 0.0;
            for (int e = 0; e < cnt; ++e) {
                const uint64_t k = tb.ref_keys[(size_t)r * REF_SLOTS + e];
                if (k == g.key) vr = tb.ref_vec[(size_t)r * REF_SLOTS + e];
            }
            const double contrib = g.first ? (g.vec < vr ? g.vec : vr) * vr : 0.0;
            const double delta = (double)(len_h - tb.ref_len2[r]);
            const double pen = exp(-(delta * delta) / sigma2x2);
#pragma unroll
            for (int n = 1; n <= 4; ++n) {
                double val = wave_sum(g.n == n ? contrib : 0.0);
                const double nr = tb.ref_norm[(size_t)r * 4 + n - 1];
                if (nh[n - 1] != 0.0 && nr != 0.0) val /= (nh[n - 1] * nr);
                score[n - 1] += val * pen;
            }
        }
        if (lane == 0) {
            double avg = (score[0] + score[1] + score[2] + score[3]) / 4.0;
            avg /= (double)(r1 - r0);
            avg *= 10.0;
            row_score[b] = avg;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int b = 0; b < B; ++b) s += row_score[b];
        fitness_out[cand] = (s / (double)B) * 100.0;        // float(cider * 100), policies.py:125
    }
}

extern "C" hipError_t nicnes_launch_cook_refs(const int32_t* ref_tokens, int n_refs, int T, const CiderTables* tb,
                                              hipStream_t stream) {
    if (n_refs <= 0) return hipSuccess;
    hipLaunchKernelGGL(nicnes_cook_refs_kernel, dim3((n_refs + 3) / 4), dim3(256), 0, stream, ref_tokens, n_refs, T, *tb);
    return hipGetLastError();
}

extern "C" hipError_t nicnes_launch_cider(const int32_t* seq, int n_cand, int B, int T, const CiderTables* tb,
                                          const int32_t* img_ref_start, double* fitness_out, hipStream_t stream) {
    if (B > 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nicnes_cider_kernel, dim3(n_cand), dim3(256), 0, stream, seq, B, T, *tb, img_ref_start, fitness_out);
    return hipGetLastError();
}
