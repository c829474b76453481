// Internal (non-ABI) launch interfaces of the engine's kernels.
#pragma once
#define SCR_SLOTS (64 + 64 + 64 + 1 + 64)   // per lane: c | h' | x of t = 0 | unfinished | h' (odd parity, split path)
#define PART_FLOATS (8 * 7 * 64)             // split path: partial greedy state of one logit workgroup (8 waves x 7 x 64 lanes)
#define COOP_CTR_STRIDE 32                   // coop path: uint32 per member-slab hand-off counter (its own 128-byte line)
#include <hip/hip_runtime.h>
#include <stdint.h>

struct DecodeParams {
    const float* theta;          // base theta, fp32 [D] (flat order: SURVEY.md Appendix A.1)
    const float* noise;          // the sigma-scaled table fp32(sigma * z) [noise_len], or a mutation's delta' rows
    const uint64_t* noise_idx;   // per member slice start (multiple of 64)
    const float* fc;             // unique-image fc features [images, F]
    const int32_t* member_batch; // nullable: member k of the launch decodes images member_batch[k] * B .. + B
    int32_t* seq;                // out: [members, 2, B, T] greedy tokens (masked after the first 0)
    float* lp;                   // out (nullable): [members, 2, B, T] log-prob of the picked token (nets.py:208,225,241)
    const double* sample_u;      // nullable: sampled decode (nets.py:210-231, fused path only): the uniform of
                                 // every (member, sign, row, logit step) [members, 2, B, T]; NULL = greedy
    float* scratch;              // nicnes_decode_scratch_floats(): lane-private c | h' | x0 | unfinished | h' (odd)
    int32_t* stats;              // [0] exact-pass fallbacks (atomic), [1] sampled re-walks, [2] coop timeouts,
                                 // [3] sampled workgroups that found no free logit slot
    float* slog;                 // sampled steps kernel: slog_ns logit slots of nst * 16384 floats (> one per resident
                                 // workgroup): the logit loop stores each step's logits there, the pick reads them
    int32_t* slog_slots;         // slog_ns claim flags (0 free), zero between launches
    int32_t slog_ns;
    int32_t* alive;              // fused path: [members * slabs], 0 once every row of the workgroup finished
    int32_t* alive2;             // split path: [2][alive_stride] by step parity
    float* part;                 // split path: [members * slabs * S] x PART_FLOATS partial greedy states
    uint32_t* coop_ctr;          // coop path: [members * slabs] x 32 hand-off counters (zeroed per launch)
    int32_t coop;                // 1: the split shape (G = 4, S = 2 or 4) in one persistent launch
    int32_t coop_launch;         // coop path: 1 hipLaunchCooperativeKernel (the runtime checks the grid is resident
                                 // at once and fails the launch otherwise), 0 a plain launch of a grid the engine
                                 // bounded by the same occupancy query (the default: same residency, no launch cost)
    uint32_t test_stall_ms;      // test hook (NICNES_TEST_COOP_STALL): coop workgroup 0 starts this late, past the
                                 // partners' spin bound, so they time out (0 = off)
    int32_t no_exit;             // 1: no per-slab early exit (log-probs of a multi-slab batch, see below)
    int32_t no_mask;             // 1: feed every argmax back unmasked (forward_for_sensitivity); fused, split, coop
    int32_t force_exact;         // test hook (NICNES_FORCE_EXACT=1): every step takes the exact tie pass
    float lse_margin;            // widening of the bounded-lse interval: 2e-3 (test hook NICNES_LSE_MARGIN)
    int32_t bounded_lse;         // 1: greedy-only decode with the pair-bounded lse (needs lp == NULL)
    int32_t B, F, V1, T;         // B: rows decoded per sign and slab range
    int32_t B_img;               // images per batch in fc / the member_batch stride (= B, or the whole batch below)
    int32_t sign_off;            // 0; > 0 (the sigma = 0 rollout decoded once): sign s decodes rows s * sign_off + b,
                                 // b < B, valid while < B_img * rpi, and its rows land at s * B + b of one [2B, T] rollout
    int32_t rpi;                 // rows per image (sampled modes: the reference's seq_per_img copies): row r reads
                                 // fc row r / rpi
    int32_t G;                   // row groups per slab: 4 (128-row slabs) or 2 (64-row slabs)
    int32_t S;                   // logit workgroups per member slab (1 + G = 4: the fused step kernel)
    int32_t alive_stride;
    int64_t D;
    int64_t off_img_w, off_img_b, off_emb_w, off_log_w, off_log_b, off_i2h_w, off_i2h_b, off_h2h_w, off_h2h_b;
};

// A mutated decode on the fused greedy path (mode != 0; the kernels' second argument, so the other kernels' argument
// layout is untouched): the delta' rows in DecodeParams::noise hold only the parameters from off_log_w on (logit, i2h,
// h2h: re-read at every step); the image projection and the embedding rows (read once, and only for the tokens taken)
// form delta' = fp32(sigma z) / s (mode 1: SM-G-SUM / SM-VECTOR) or fp32(sigma z) * s (mode 2: SM-PROPORTIONAL)
// themselves, from the sigma-scaled table slice at head_idx[member] and the mutation vector
struct MutHead {
    const float* head_noise;
    const uint64_t* head_idx;
    const float* mut_vec;
    int32_t mode;
};

// launch kinds recorded next to the timing events
#define DK_IMG 0
#define DK_STEP 1        // fused step kernel (logits of t + cell of t + 1)
#define DK_STEPS 4       // fused path, every step in one launch (nicnes_decode_steps_kernel)
#define DK_CELL 2        // split path: token merge of t + cell of t + 1
#define DK_LOGIT 3       // split path: logits of t over one vocabulary range
#define DK_COOP 5        // coop path: every step of the split shape in one launch
#define DK_STEPS2 6      // fused path of 64-row slabs (G = 2, S = 1), every step in one launch

// evs (nullable): up to DECODE_MAX_EVENTS events, recorded before the first launch and after every
// launch; kinds[k] (k >= 1) is the kind of the launch that event k follows. Returns the launch count
// in *n_launch.
#define DECODE_MAX_EVENTS 64
extern "C" hipError_t nicnes_decode_init();
// workgroups of the coop kernels (min over their instantiations) and of the sampled steps kernel one CU holds at
// once (hipOccupancyMaxActiveBlocksPerMultiprocessor at their LDS): the coop grid must fit occ x CUs, the sampled
// logit slots must outnumber occ x CUs
extern "C" hipError_t nicnes_decode_occupancy(int* coop_per_cu, int* sample_per_cu);
// shifts the per-member and per-workgroup pointers of *p to member m0 (a decode of members m0.. on
// its own stream; nslabs = the launch's row slabs)
extern "C" void nicnes_decode_shift(DecodeParams* p, int m0, int nslabs, MutHead* mh);
// mh: nullable (or mode 0): no decode-formed delta'
extern "C" hipError_t nicnes_launch_decode(const DecodeParams* p, const MutHead* mh, int member_count, int nslabs,
                                           hipStream_t stream, hipEvent_t* evs, int* kinds, int* n_launch);
// zero seq_logprobs past the batch's last finishing step (rollouts = members x 2 of B rows; after a
// no_exit decode of a batch spanning several slabs)
extern "C" hipError_t nicnes_launch_lp_batch_exit(const int32_t* seq, float* lp, int rollouts, int B, int T,
                                                  hipStream_t stream);
// lane scratch for up to member_count members x row_waves 32-row waves of one sign
extern "C" size_t nicnes_decode_scratch_floats(int member_count, int row_waves_per_member);
