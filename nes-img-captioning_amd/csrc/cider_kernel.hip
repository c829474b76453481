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

// lane j owns n-gram slot i = j & 15 of size n = (j >> 4) + 1: one 16-lane segment per n, so
// per-n sums are 4-step segmented reductions
__device__ __forceinline__ void slot_of_lane(int j, int& n, int& i) {
    n = (j >> 4) + 1;
    i = j & 15;
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

__device__ __host__ __forceinline__ uint64_t df_hash(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// df of an n-gram: linear probing in the hash copy of the sorted table (0 when absent)
__device__ __forceinline__ double df_lookup(const CiderTables& tb, uint64_t key) {
    uint64_t h = df_hash(key) & tb.hash_mask;
    for (uint64_t probe = 0; probe <= tb.hash_mask; ++probe) {
        const uint64_t k = tb.hash_keys[h];
        if (k == key) return tb.hash_vals[h];
        if (k == 0ull) return 0.0;
        h = (h + 1) & tb.hash_mask;
    }
    return 0.0;
}

__global__ __launch_bounds__(256) void nicnes_df_hash_build_kernel(const uint64_t* keys, const double* vals, int64_t n,
                                                                   unsigned long long* hkeys, double* hvals,
                                                                   uint64_t mask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long key = keys[i];
    uint64_t h = df_hash(key) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe) {
        const unsigned long long prev = atomicCAS(&hkeys[h], 0ull, key);
        if (prev == 0ull || prev == key) {
            hvals[h] = vals[i];
            return;
        }
        h = (h + 1) & mask;
    }
}

// sum over the lane's 16-lane segment (every lane of the segment gets it)
__device__ __forceinline__ double seg_sum(double v) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
    return v;
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

// per-lane n-gram of one caption row (L = caption_len), its tf over the row and first-occurrence flag
__device__ __forceinline__ void ngram_key(const int32_t* row, int T, int lane, int L, NgramLane& g, int& tf) {
    int i;
    slot_of_lane(lane, g.n, i);
    g.valid = i + g.n <= L;
    g.key = g.valid ? pack_ngram(row, g.n, i) : 0ull;
    tf = 0;
    bool first = g.valid;
    const int seg = lane & 48;
    for (int o = 0; o < 16; ++o) {             // equal keys have equal n: same segment
        const uint64_t k2 = __shfl(g.key, seg | o);
        if (g.valid && k2 == g.key) {           // invalid lanes hold key 0, never a valid key
            ++tf;
            if ((seg | o) < lane) first = false;
        }
    }
    g.first = first;
    g.vec = 0.0;
}

// ... and its weight
__device__ __forceinline__ NgramLane ngram_lane(const int32_t* row, int T, int lane, const CiderTables& tb) {
    NgramLane g;
    int tf;
    ngram_key(row, T, lane, caption_len(row, T), g, tf);
    if (g.first) {
        const double df = df_lookup(tb, g.key);
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
    const double nrm = sqrt(seg_sum(g.first ? g.vec * g.vec : 0.0));     // norm of this lane's n
    if ((lane & 15) == 0) tb.ref_norm[(size_t)r * 4 + (lane >> 4)] = nrm;
    if (lane == 0) {
        tb.ref_count[r] = __popcll(firsts);
        const int L = caption_len(row, T);
        tb.ref_len2[r] = L > 1 ? L - 1 : 0;          // bigram count (counts2vec 'length' quirk)
    }
}

// ---- fitness of one candidate from its per-row CIDEr-D scores (whole workgroup) ----------------
// crit 0 ('greedy'): float(cider * 100) (policies.py:125). crit 1-4 (greedy_logprob / expprob /
// linprob / avgprob, picked by Fitness.get_criterium, policies.py:50-61): the criterion over the
// per-step log-probs, rewards = per-row score as fp32 (policies.py:121,191), mask = 1 at t = 0 then
// seq[t-1] > 0; elementwise in fp32 as torch does, sum(out) / sum(mask) accumulated in fp64
// (fitness.py:43-132).
// crit 5 ('sample'): as 'greedy' over the sampled rows. crit 6 ('self_critical', compute_ciders,
// policies.py:174-184): 100 * mean of (sample score - greedy score) per row, base = the greedy rows'
// scores. crit 7 ('sc_loss'): LogFitnessCriterion (fitness.py:12-40), -lp * reward * mask with reward =
// the row's self-critical score difference (policies.py:119-123, get_criterium :50-52).
// A faulted decode (decode_fault: rows left undecoded by a hand-off or slot timeout) writes NaN instead.
__device__ void finish_fitness(const double* row_score, const int32_t* seq, const float* lp, int B, int T, int crit,
                               double* out, const double* base, int base_rpi, const int32_t* fault) {
    if (decode_fault(fault)) {
        if (threadIdx.x == 0) *out = __builtin_nan("");
        return;
    }
    if (crit == 0 || crit == 5 || crit == 6 || lp == nullptr) {
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int b = 0; b < B; ++b) s += row_score[b] - (crit == 6 && base ? base[b / base_rpi] : 0.0);
            *out = (s / (double)B) * 100.0;
        }
        return;
    }
    __shared__ double red_num[256], red_den[256];
    double num = 0.0, den = 0.0;
    const float third = (float)(1.0 / 9.0), l9 = (float)0.9542425094393249, em1 = (float)(2.718281828459045 - 1.0);
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        const float reward = (float)(row_score[b] - (base ? base[b / base_rpi] : 0.0));
        for (int t = 0; t < T; ++t) {
            if (t > 0 && seq[(size_t)b * T + t - 1] <= 0) break;   // masked from here on
            const float p = expf(lp[(size_t)b * T + t]);
            float o;
            if (crit == 7) {
                o = -lp[(size_t)b * T + t] * reward;
            } else if (crit == 2) {
                o = (expf(p) - 1.0f) / em1 * reward;
            } else if (crit == 3) {
                o = p * reward;
            } else {
                const float pfact = log10f(p + third) + l9;
                o = crit == 1 ? pfact * reward : 0.5f * reward + 0.5f * pfact * reward;
            }
            num += (double)o;
            den += 1.0;
        }
    }
    red_num[threadIdx.x] = num;
    red_den[threadIdx.x] = den;
    __syncthreads();
    if (threadIdx.x == 0) {
        double sn = 0.0, sd = 0.0;
        for (int i = 0; i < (int)blockDim.x; ++i) { sn += red_num[i]; sd += red_den[i]; }
        *out = sn / sd;
    }
}

// ---- candidates: one workgroup per candidate, one wave per image row ---------------------------
__global__ __launch_bounds__(256) void nicnes_cider_kernel(const int32_t* seq, int B, int T, CiderTables tb,
                                                           const int32_t* img_ref_start, const int32_t* member_batch,
                                                           const float* lp, int crit, double* fitness_out,
                                                           const double* base, double* scores_out, int rpi) {
    __shared__ double row_score[1024];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cand = blockIdx.x;
    img_ref_start += member_batch ? member_batch[cand >> 1] * (B / rpi) : 0;   // this member's batch (single_batch: false)
    const double sigma2x2 = 2.0 * 6.0 * 6.0;
    for (int b = wave; b < B; b += 4) {
        const int32_t* row = seq + ((size_t)cand * B + b) * T;
        const NgramLane g = ngram_lane(row, T, lane, tb);
        const double nh = sqrt(seg_sum(g.first ? g.vec * g.vec : 0.0));   // |vec_hyp[n]| for this lane's n
        const int L = caption_len(row, T);
        const int len_h = L > 1 ? L - 1 : 0;
        double score = 0.0;                                                  // score[n] of this segment
        const int r0 = img_ref_start[b / rpi], r1 = img_ref_start[b / rpi + 1];   // row b's image
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
            double val = seg_sum(contrib);
            const double nr = tb.ref_norm[(size_t)r * 4 + (lane >> 4)];
            if (nh != 0.0 && nr != 0.0) val /= (nh * nr);
            score += val * pen;
        }
        // (score[0] + score[1]) + (score[2] + score[3]) across the four segments
        score += __shfl_xor(score, 16);
        score += __shfl_xor(score, 32);
        if (lane == 0) {
            double avg = score / 4.0;
            avg /= (double)(r1 - r0);
            avg *= 10.0;
            row_score[b] = avg;
        }
    }
    __syncthreads();
    if (scores_out)
        for (int b = threadIdx.x; b < B; b += blockDim.x) scores_out[(size_t)cand * B + b] = row_score[b];
    finish_fitness(row_score, seq + (size_t)cand * B * T, lp ? lp + (size_t)cand * B * T : nullptr, B, T, crit,
                   fitness_out + cand, base ? base + (size_t)cand * (B / rpi) : nullptr, rpi, tb.fault);
}

extern "C" uint64_t nicnes_df_hash_capacity(int64_t n) {
    uint64_t c = 64;
    while (c < 2ull * (uint64_t)n) c <<= 1;
    return c;
}

extern "C" hipError_t nicnes_launch_df_hash_build(const uint64_t* keys, const double* vals, int64_t n, uint64_t* hkeys,
                                                  double* hvals, uint64_t mask, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(nicnes_df_hash_build_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, keys, vals, n,
                       (unsigned long long*)hkeys, hvals, mask);
    return hipGetLastError();
}

extern "C" hipError_t nicnes_launch_cook_refs(const int32_t* ref_tokens, int n_refs, int T, const CiderTables* tb,
                                              hipStream_t stream) {
    if (n_refs <= 0) return hipSuccess;
    hipLaunchKernelGGL(nicnes_cook_refs_kernel, dim3((n_refs + 3) / 4), dim3(256), 0, stream, ref_tokens, n_refs, T, *tb);
    return hipGetLastError();
}

extern "C" hipError_t nicnes_launch_cider(const int32_t* seq, int n_cand, int B, int T, const CiderTables* tb,
                                          const int32_t* img_ref_start, const int32_t* member_batch, const float* lp,
                                          int crit, double* fitness_out, hipStream_t stream, const double* base,
                                          double* scores_out, int rpi) {
    if (B > 1024 || rpi < 1 || B % rpi) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nicnes_cider_kernel, dim3(n_cand), dim3(256), 0, stream, seq, B, T, *tb, img_ref_start,
                       member_batch, lp, crit, fitness_out, base, scores_out, rpi);
    return hipGetLastError();
}

// ---- per-image reference n-gram tables (one wave per image, built once per batch) ------------
__global__ __launch_bounds__(64) void nicnes_img_ngram_kernel(const int32_t* img_ref_start, CiderTables tb) {
    __shared__ unsigned long long hk[IMG_CAP];
    __shared__ int hr[IMG_CAP];
    __shared__ int nrows;
    const int lane = threadIdx.x, b = blockIdx.x;
    for (int i = lane; i < IMG_CAP; i += 64) { hk[i] = 0ull; hr[i] = -1; }
    if (lane == 0) nrows = 0;
    __syncthreads();
    const int r0 = img_ref_start[b], r1 = img_ref_start[b + 1];
    for (int r = r0; r < r1 && r - r0 < IMG_MAXR; ++r) {
        const int cnt = tb.ref_count[r];
        if (lane < cnt) {
            const unsigned long long key = tb.ref_keys[(size_t)r * REF_SLOTS + lane];
            uint32_t slot = (uint32_t)df_hash(key) & (IMG_CAP - 1);
            int row = -1;
            for (int probe = 0; probe < IMG_CAP; ++probe) {
                const unsigned long long prev = atomicCAS(&hk[slot], 0ull, key);
                if (prev == 0ull) {                      // new n-gram of this image
                    row = atomicAdd(&nrows, 1);
                    hr[slot] = row;
                    break;
                }
                if (prev == key) {                       // seen in an earlier reference
                    row = hr[slot];
                    break;
                }
                slot = (slot + 1) & (IMG_CAP - 1);
            }
            if (row >= 0 && row < IMG_ROWS)
                tb.img_vr[((size_t)b * IMG_ROWS + row) * IMG_MAXR + (r - r0)] = tb.ref_vec[(size_t)r * REF_SLOTS + lane];
        }
        __syncthreads();
    }
    for (int i = lane; i < IMG_CAP; i += 64) {
        tb.img_hkey[(size_t)b * IMG_CAP + i] = hk[i];
        tb.img_hrow[(size_t)b * IMG_CAP + i] = hr[i];
    }
}

// candidates scored against the image table: one probe per distinct n-gram, then the per-reference
// weights are consecutive doubles (same arithmetic and order as nicnes_cider_kernel).
// Grid (candidate, row block of CIDER_IMG_ROWS): the probe chains are latency-bound, so each
// candidate's rows are spread over several workgroups; per-row scores go to `scores` [n_cand, B]
// and nicnes_cider_finish_kernel reduces them in row order, as the single-workgroup form did.
// Rows per workgroup: 32, or 8 when there are few candidates (64 members per GPU: 128 candidates), so that the
// launch still has >= ~2048 workgroups to hide the probe latency (the P = 64 rollouts: DESIGN §5).
#define CIDER_IMG_ROWS 32
#ifndef CIDER_PAR_PROBE
#define CIDER_PAR_PROBE 1          // the df and image-table probes of an n-gram issued together
#endif
#ifndef CIDER_WPE
#define CIDER_WPE 0                // > 0: amdgpu_waves_per_eu bound of the image kernel (register budget)
#endif
#if CIDER_WPE
#define CIDER_IMG_ATTR __attribute__((amdgpu_waves_per_eu(CIDER_WPE)))
#else
#define CIDER_IMG_ATTR
#endif
__global__ __launch_bounds__(256) CIDER_IMG_ATTR void nicnes_cider_img_kernel(const int32_t* seq, int B, int T, CiderTables tb,
                                                               const int32_t* img_ref_start, const int32_t* member_batch,
                                                               double* scores, int rpi, int rows_wg) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cand = blockIdx.x;
    const int img0 = member_batch ? member_batch[cand >> 1] * (B / rpi) : 0;   // this member's batch (single_batch: false)
    const int b_end = min(B, (int)(blockIdx.y + 1) * rows_wg);
    const double sigma2x2 = 2.0 * 6.0 * 6.0;
    for (int b = (int)blockIdx.y * rows_wg + wave; b < b_end; b += 4) {
        const int32_t* row = seq + ((size_t)cand * B + b) * T;
        const int L = caption_len(row, T);
        const int len_h = L > 1 ? L - 1 : 0;
        const int im = img0 + b / rpi;                                     // row b's image
#if CIDER_PAR_PROBE
        // the df probe and the image-table probe of the lane's n-gram both need only its key: their loads are
        // issued together (one dependent round trip less per row than df first, then the image table)
        const int rs0 = img_ref_start[im], rs1 = img_ref_start[im + 1];
        int rl2[IMG_MAXR];
        double rnm[IMG_MAXR];
#pragma unroll
        for (int u = 0; u < IMG_MAXR; ++u) {
            rl2[u] = rs0 + u < rs1 ? tb.ref_len2[rs0 + u] : 0;
            rnm[u] = rs0 + u < rs1 ? tb.ref_norm[(size_t)(rs0 + u) * 4 + (lane >> 4)] : 0.0;
        }
        NgramLane g;
        int tf;
        ngram_key(row, T, lane, L, g, tf);
        int trow = -1;
        double df = 0.0;
        if (g.first) {
            const uint64_t hs = df_hash(g.key);
            uint64_t h = hs & tb.hash_mask;
            uint32_t slot = (uint32_t)hs & (IMG_CAP - 1);
            const uint64_t* ik = tb.img_hkey + (size_t)im * IMG_CAP;
            uint64_t k1 = tb.hash_keys[h], k2 = ik[slot];
            for (uint64_t probe = 0; probe < tb.hash_mask && k1 != g.key && k1 != 0ull; ++probe) {
                h = (h + 1) & tb.hash_mask;
                k1 = tb.hash_keys[h];
            }
            for (int probe = 0; probe < IMG_CAP - 1 && k2 != g.key && k2 != 0ull; ++probe) {
                slot = (slot + 1) & (IMG_CAP - 1);
                k2 = ik[slot];
            }
            if (k1 == g.key) df = tb.hash_vals[h];
            if (k2 == g.key) trow = tb.img_hrow[(size_t)im * IMG_CAP + slot];
            g.vec = (double)tf * (tb.ref_len - log(df > 1.0 ? df : 1.0));
        }
        const double nh = sqrt(seg_sum(g.first ? g.vec * g.vec : 0.0));
#else
        const NgramLane g = ngram_lane(row, T, lane, tb);
        const double nh = sqrt(seg_sum(g.first ? g.vec * g.vec : 0.0));
        int trow = -1;
        if (g.first) {
            uint32_t slot = (uint32_t)df_hash(g.key) & (IMG_CAP - 1);
            for (int probe = 0; probe < IMG_CAP; ++probe) {
                const uint64_t k = tb.img_hkey[(size_t)im * IMG_CAP + slot];
                if (k == g.key) { trow = tb.img_hrow[(size_t)im * IMG_CAP + slot]; break; }
                if (k == 0ull) break;
                slot = (slot + 1) & (IMG_CAP - 1);
            }
        }
#endif
        const double* vrow = tb.img_vr + ((size_t)im * IMG_ROWS + (trow >= 0 ? trow : 0)) * IMG_MAXR;
        double score = 0.0;
#if CIDER_PAR_PROBE
        // (r1 - r0 <= IMG_MAXR on this path: the engine takes it only then) the image's reference terms, loaded
        // before the probes' results are waited for
        const int r0 = rs0, r1 = rs1;
#pragma unroll
        for (int u = 0; u < IMG_MAXR; ++u) {
            if (r0 + u >= r1) break;
            const double vr = trow >= 0 ? vrow[u] : 0.0;
            const double contrib = g.first ? (g.vec < vr ? g.vec : vr) * vr : 0.0;
            const double delta = (double)(len_h - rl2[u]);
            const double pen = exp(-(delta * delta) / sigma2x2);
            double val = seg_sum(contrib);
            const double nr = rnm[u];
            if (nh != 0.0 && nr != 0.0) val /= (nh * nr);
            score += val * pen;
        }
#else
        const int r0 = img_ref_start[im], r1 = img_ref_start[im + 1];
        for (int r = r0; r < r1; ++r) {
            const double vr = trow >= 0 ? vrow[r - r0] : 0.0;
            const double contrib = g.first ? (g.vec < vr ? g.vec : vr) * vr : 0.0;
            const double delta = (double)(len_h - tb.ref_len2[r]);
            const double pen = exp(-(delta * delta) / sigma2x2);
            double val = seg_sum(contrib);
            const double nr = tb.ref_norm[(size_t)r * 4 + (lane >> 4)];
            if (nh != 0.0 && nr != 0.0) val /= (nh * nr);
            score += val * pen;
        }
#endif
        score += __shfl_xor(score, 16);
        score += __shfl_xor(score, 32);
        if (lane == 0) {
            double avg = score / 4.0;
            avg /= (double)(r1 - r0);
            avg *= 10.0;
            scores[(size_t)cand * B + b] = avg;
        }
    }
}

__global__ __launch_bounds__(256) void nicnes_cider_finish_kernel(const int32_t* seq, int B, int T,
                                                                  const double* scores, const float* lp, int crit,
                                                                  double* fitness_out, const double* base, int rpi,
                                                                  const int32_t* fault) {
    const int cand = blockIdx.x;
    finish_fitness(scores + (size_t)cand * B, seq + (size_t)cand * B * T, lp ? lp + (size_t)cand * B * T : nullptr,
                   B, T, crit, fitness_out + cand, base ? base + (size_t)cand * (B / rpi) : nullptr, rpi, fault);
}

extern "C" hipError_t nicnes_launch_img_ngrams(const int32_t* img_ref_start, int B, const CiderTables* tb,
                                               hipStream_t stream) {
    hipLaunchKernelGGL(nicnes_img_ngram_kernel, dim3(B), dim3(64), 0, stream, img_ref_start, *tb);
    return hipGetLastError();
}

extern "C" hipError_t nicnes_launch_cider_img(const int32_t* seq, int n_cand, int B, int T, const CiderTables* tb,
                                              const int32_t* img_ref_start, const int32_t* member_batch, const float* lp,
                                              int crit, double* scores, double* fitness_out, hipStream_t stream,
                                              const double* base, int rpi) {
    if (B > 1024 || n_cand < 1 || rpi < 1 || B % rpi) return hipErrorInvalidValue;
    const int rows_wg = (int64_t)n_cand * ((B + CIDER_IMG_ROWS - 1) / CIDER_IMG_ROWS) >= 2048 ? CIDER_IMG_ROWS : 8;
    hipLaunchKernelGGL(nicnes_cider_img_kernel, dim3(n_cand, (B + rows_wg - 1) / rows_wg), dim3(256), 0,
                       stream, seq, B, T, *tb, img_ref_start, member_batch, scores, rpi, rows_wg);
    hipLaunchKernelGGL(nicnes_cider_finish_kernel, dim3(n_cand), dim3(256), 0, stream, seq, B, T, (const double*)scores,
                       lp, crit, fitness_out, base, rpi, tb->fault);
    return hipGetLastError();
}
