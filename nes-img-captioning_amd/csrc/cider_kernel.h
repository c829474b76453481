// Internal (non-ABI) interface of the CIDEr-D kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct CiderTables {
    const uint64_t* df_keys;   // sorted packed n-gram keys of the document-frequency table
    const double* df_vals;     // document frequency per key
    int64_t df_n;
    const uint64_t* hash_keys; // open-addressing copy of the df table (0 = empty slot; no valid key is 0)
    const double* hash_vals;
    uint64_t hash_mask;        // capacity - 1 (capacity a power of two >= 2 df_n)
    double ref_len;            // log(ref_len_raw)  (CiderScorer fixed-df mode)
    // per-reference vectors (written by nicnes_cook_refs_kernel)
    uint64_t* ref_keys;        // [n_refs, 64] distinct n-grams
    double* ref_vec;           // [n_refs, 64] tf * idf
    int32_t* ref_count;        // [n_refs]
    int32_t* ref_len2;         // [n_refs] bigram count
    double* ref_norm;          // [n_refs, 4]
    // per-image n-gram tables (written by nicnes_img_ngram_kernel): the union of the image's
    // reference n-grams, hashed to a row of per-reference tf-idf weights
    uint64_t* img_hkey;        // [images, IMG_CAP] (0 = empty)
    int32_t* img_hrow;         // [images, IMG_CAP]
    double* img_vr;            // [images, IMG_ROWS, IMG_MAXR]
    // nullable: the handle's decode counters; a coop hand-off timeout ([2]) or a sampled workgroup without a
    // logit slot ([3]) left rows undecoded, so every fitness written from then on is NaN (decode_fault)
    const int32_t* fault;
};

// the decode of this handle lost rows (sticky: the counters only grow; the engine reports it at the next host read)
__device__ __forceinline__ bool decode_fault(const int32_t* f) {
    return f != nullptr && (f[2] | f[3]) != 0;     // written by earlier launches on the stream
}
#define IMG_CAP 1024
#define IMG_ROWS 512
#define IMG_MAXR 8

extern "C" uint64_t nicnes_df_hash_capacity(int64_t n);
extern "C" hipError_t nicnes_launch_df_hash_build(const uint64_t* keys, const double* vals, int64_t n, uint64_t* hkeys,
                                                  double* hvals, uint64_t mask, hipStream_t stream);
extern "C" hipError_t nicnes_launch_cook_refs(const int32_t* ref_tokens, int n_refs, int T, const CiderTables* tb,
                                              hipStream_t stream);
extern "C" hipError_t nicnes_launch_img_ngrams(const int32_t* img_ref_start, int B, const CiderTables* tb,
                                               hipStream_t stream);
// lp (nullable) [n_cand, B, T] per-step log-probs; crit = fitness criterion (nicnes_set_fitness_mode)
// scores: scratch [n_cand, B] fp64 (per-row CIDEr-D, reduced by a second kernel)
// member_batch (nullable) [n_cand / 2]: candidate c scores against images member_batch[c / 2] * B + b.
// crit: nicnes.h NICNES_FITNESS_*. B = rows per candidate, rpi of them per image (row b scores against image
// b / rpi: the sampled modes' seq_per_img copies). base (nullable, crit 6 / 7) [n_cand, B / rpi]: the greedy
// rows' scores (one per image) the self-critical modes subtract. scores ([n_cand, B]) receives every row's
// CIDEr-D (cider_img: always, as scratch; cider: when non-null)
extern "C" hipError_t nicnes_launch_cider_img(const int32_t* seq, int n_cand, int B, int T, const CiderTables* tb,
                                              const int32_t* img_ref_start, const int32_t* member_batch, const float* lp,
                                              int crit, double* scores, double* fitness_out, hipStream_t stream,
                                              const double* base = nullptr, int rpi = 1);
extern "C" hipError_t nicnes_launch_cider(const int32_t* seq, int n_cand, int B, int T, const CiderTables* tb,
                                          const int32_t* img_ref_start, const int32_t* member_batch, const float* lp,
                                          int crit, double* fitness_out, hipStream_t stream, const double* base = nullptr,
                                          double* scores = nullptr, int rpi = 1);
