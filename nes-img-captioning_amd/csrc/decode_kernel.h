// Internal (non-ABI) launch interfaces of the engine's kernels.
#pragma once
#define SCR_SLOTS (64 + 64 + 64 + 1)   // per lane: c | h' | x of t = 0 | unfinished
#include <hip/hip_runtime.h>
#include <stdint.h>

struct DecodeParams {
    const float* theta;          // base theta, fp32 [D] (flat order: SURVEY.md Appendix A.1)
    const float* noise;          // shared Gaussian table, fp32 [noise_len]
    const uint64_t* noise_idx;   // per member slice start (multiple of 64)
    const float* fc;             // unique-image fc features [B, F]
    int32_t* seq;                // out: [members, 2, B, T] greedy tokens (masked after the first 0)
    float* lp;                   // out (nullable): [members, 2, B, T] log-prob of the greedy token (nets.py:208,241)
    float* scratch;              // nicnes_decode_scratch_floats(): lane-private c | h' | x0 | unfinished
    int32_t* stats;              // [0] = exact-pass fallbacks (atomic)
    int32_t* alive;              // [members * slabs]: 0 once every row of the workgroup finished
    float sigma;
    int32_t force_exact;         // test hook (NICNES_FORCE_EXACT=1): every step takes the exact tie pass
    int32_t B, F, V1, T;
    int64_t D;
    int64_t off_img_w, off_img_b, off_emb_w, off_log_w, off_log_b, off_i2h_w, off_i2h_b, off_h2h_w, off_h2h_b;
};

// evs (nullable): T + 4 events, recorded before the first launch and after every launch (img, step -1..T)
#define DECODE_MAX_EVENTS 64
extern "C" hipError_t nicnes_launch_decode(const DecodeParams* p, int member_count, int nslabs, hipStream_t stream,
                                           hipEvent_t* evs);
extern "C" size_t nicnes_decode_scratch_floats(int member_count, int nslabs);
