/*
 * nicnes.h -- C ABI of the MI355X NIC-NES population-evaluation engine (libnicnes.so).
 *
 * Plain C: status codes, raw pointers and sizes, no torch types. All array arguments are
 * DEVICE pointers on the handle's GPU unless the name ends in _host. `stream` is a
 * hipStream_t (NULL = the default stream); every call only enqueues work on it, except the
 * functions documented as synchronising. A handle is not thread-safe: one owner thread per
 * handle, one handle per GPU. Buffers passed to nicnes_set_* are borrowed (the caller keeps
 * them alive and unchanged until the handle is destroyed or the buffer is replaced); output
 * buffers are written by the enqueued work.
 *
 * Each entry point names the reference interface (rubencart/NES-img-captioning, file:line) it
 * replaces. Integration stubs for the reference side: INTEGRATION.md.
 */
#ifndef NICNES_H
#define NICNES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NICNES_OK 0
#define NICNES_ERR_INVALID 1       /* bad argument / wrong state */
#define NICNES_ERR_UNSUPPORTED 2   /* experiment option the engine does not implement */
#define NICNES_ERR_HIP 3           /* HIP runtime error (message in nicnes_last_error) */
#define NICNES_ERR_NOMEM 4
#define NICNES_ERR_FAULT 5         /* contained decode fault: NaN fitness, the optimizer step skipped (nicnes_stats) */

typedef struct nicnes_handle nicnes_handle;

/* Filled from the experiment JSON (src/algorithm/policies.py:31-41 ModelOptions,
 * src/captioning/experiment.py:27-30 vocab injection, src/algorithm/tools/utils.py:14-20 Config). */
typedef struct nicnes_config {
    int32_t vocab_size;           /* V; logits are V + 1 wide (src/captioning/nets.py:151-152) */
    int32_t input_encoding_size;  /* E (must be 128) */
    int32_t rnn_size;             /* R (must be 128) */
    int32_t fc_feat_size;         /* F (multiple of 128) */
    int32_t seq_length;           /* 16 (src/captioning/nets.py:147) */
    int32_t max_batch;            /* max unique images per batch (config.batch_size) */
    int32_t max_refs;             /* max reference captions per batch */
    int32_t max_members;          /* max population members per nicnes_evaluate call */
    uint64_t noise_len;           /* entries of the shared Gaussian table */
    uint64_t noise_seed;          /* seed of the member -> table-offset rule */
} nicnes_config;

/* flat parameter count D for a config (src/algorithm/nets.py:146-148 count_parameters) */
int64_t nicnes_param_count(const nicnes_config* cfg);
/* offsets of the 9 tensors in the flat theta (registration order) + D at [9] */
int nicnes_param_offsets(const nicnes_config* cfg, int64_t* out10_host);

int nicnes_create(const nicnes_config* cfg, int device, nicnes_handle** out);
int nicnes_destroy(nicnes_handle* h);
const char* nicnes_last_error(const nicnes_handle* h);

/* Shared noise table (borrowed), replaces the per-worker torch.normal_ draw of
 * PolicyNet.evolve, src/algorithm/nets.py:101-102. The engine keeps a sigma-scaled copy
 * fp32(sigma * table) for the decode (noise_len floats of device memory), rebuilt by the first
 * evaluation after this call or after a change of sigma; call again if the table's contents change. */
int nicnes_set_noise_table(nicnes_handle* h, const float* table, uint64_t len);

/* Current parameters (copied into the engine's fp64 master + fp32 evaluation copy), replaces
 * Policy.set_model / set_from_parameter_vector, src/algorithm/policies.py:106-147.
 * is_fp32_origin = 1 keeps the reference's fp32-theta semantics for the first Adam step. */
int nicnes_set_theta(nicnes_handle* h, const double* theta64, int is_fp32_origin, void* stream);
int nicnes_get_theta(nicnes_handle* h, double* theta64_out, float* theta32_out, void* stream);
/* Adam state in the reference layout (src/algorithm/nic_nes/optimizers.py:85-107): m, v, t */
int nicnes_set_adam_state(nicnes_handle* h, const double* m, const double* v, int64_t t, void* stream);
int nicnes_get_adam_state(nicnes_handle* h, double* m_out, double* v_out, int64_t* t_out_host, void* stream);

/* One batch (src/captioning/dataloader.py:135-203 get_batch, deduplicated to unique images):
 * fc [B, F] fp32; ref_tokens [n_refs, seq_length] int32 zero-padded label rows;
 * img_ref_start [B + 1] (refs of image b are [img_ref_start[b], img_ref_start[b+1])).
 * Builds the reference-side CIDEr-D vectors on `stream`. */
int nicnes_set_batch(nicnes_handle* h, const float* fc, int32_t B, const int32_t* ref_tokens, int32_t n_refs,
                     const int32_t* img_ref_start, void* stream);

/* Several batches at once, for per-member batches (single_batch: false in the experiment JSON: each
 * reference worker draws its own batch for every member, src/algorithm/nic_nes/nic_nes_worker.py:
 * 121-128). fc [n_batches * B, F]; batch g holds images g * B .. g * B + B - 1, whose references are
 * ranges of img_ref_start [n_batches * B + 1] as in nicnes_set_batch (= this call with n_batches 1). */
int nicnes_set_batches(nicnes_handle* h, const float* fc, int32_t n_batches, int32_t B, const int32_t* ref_tokens,
                       int32_t n_refs, const int32_t* img_ref_start, void* stream);

/* Fixed document-frequency table (CiderD(df='coco-train-idxs'), src/captioning/policies.py:72):
 * sorted packed n-gram keys (n<<56 | t0<<42 | t1<<28 | t2<<14 | t3), df counts, and
 * ref_len = log(raw ref_len) as the scorer uses it. The engine keeps its own hashed copy, built
 * here (synchronising); the caller's arrays are borrowed as for every nicnes_set_* call. */
int nicnes_set_df_table(nicnes_handle* h, const uint64_t* keys, const double* df, int64_t n, double ref_len_log);

/* Noise-table offsets of members [member_begin, member_begin + count) at `iteration`. */
int nicnes_noise_indices(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, uint64_t* out,
                         void* stream);

/* Evaluate `count` members (each an antithetic pair theta +- sigma z): greedy decode of the
 * batch + CIDEr-D fitness. Replaces NESWorker.fitness (src/algorithm/nic_nes/nic_nes_worker.py:115-161)
 * for a whole population slice. fitness_out [count, 2] fp64 = (f+, f-) per member;
 * seq_out [count, 2, B, seq_length] int32 or NULL. */
int nicnes_evaluate(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                    double* fitness_out, int32_t* seq_out, void* stream);

/* The perturbations themselves, delta_k = fp32(sigma * table[idx_k : idx_k + D]) for members
 * [member_begin, +count): out [count, D] fp32. What PolicyNet.evolve returns
 * (src/algorithm/nets.py:101-102, 118) and NESResult.evolve_noise carries to an unchanged reference
 * master (src/algorithm/nic_nes/nic_nes_worker.py:156-161); the engine's own master never needs them. */
int nicnes_noise_vectors(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                         float* out, void* stream);

/* Safe / proportional mutations (PolicyNet.evolve, src/algorithm/nets.py:96-113; Mutation enum :16-21):
 * the member's noise becomes delta' = fp32(fp32(sigma * z) / vec) with mode NICNES_MUTATION_DIVIDE
 * (SM-G-SUM: vec = the sensitivity of src/algorithm/safe_mutations.py:34-117 after its underflow
 * clamp and scaling; SM-VECTOR: the loaded vector, :27-31) or fp32(fp32(sigma * z) * vec) with
 * NICNES_MUTATION_SCALE (SM-PROPORTIONAL: vec = |theta|, zeros replaced by mean |theta|).
 * vec [D] fp32 device (copied). Every later evaluate / grad_partial / noise_vectors uses delta':
 * an evaluation materialises it per member ([max_members, D] on the device, allocated at the first
 * mutated evaluation), the weighted noise sum transforms each delta on the fly.
 * NICNES_MUTATION_PLAIN turns it off. */
#define NICNES_MUTATION_PLAIN 0
#define NICNES_MUTATION_DIVIDE 1
#define NICNES_MUTATION_SCALE 2
int nicnes_set_mutation(nicnes_handle* h, int32_t mode, const float* vec, void* stream);
/* SM-PROPORTIONAL's vector from the handle's own fp32 theta (nets.py:108-112: |theta| with exact zeros replaced
 * by mean|theta|), formed on the device: vec[j] = theta32[j] == 0 ? mean_abs : |theta32[j]|, then mode SCALE.
 * mean_abs is the caller's fp32 mean of |theta| (the reference's torch mean, whose reduction order a device sum
 * would not reproduce). Replaces a host round trip of theta through nicnes_set_mutation(SCALE, vec). */
int nicnes_set_mutation_proportional(nicnes_handle* h, float mean_abs, void* stream);
/* How many entries of the handle's fp32 theta are exactly zero (either sign): when none, SM-PROPORTIONAL's
 * mean is not used and the caller can skip computing it. Synchronises the stream. */
int nicnes_theta_zeros(nicnes_handle* h, int64_t* count_out_host, void* stream);

/* Fitness criterion (Fitness enum + get_criterium, src/captioning/policies.py:22-61, applied at
 * :119-125): GREEDY = 100 * mean CIDEr-D; the greedy_* modes weight each step's probability of the
 * greedy token by the row's CIDEr-D (src/captioning/fitness.py:43-132). The sampled modes decode with
 * FCModel._sample(greedy=False) (src/captioning/nets.py:210-231: each row draws its token from the
 * softmax with one uniform per row and step) on the fused path: SAMPLE = 100 * mean CIDEr-D of the
 * sampled rows; SELF_CRITICAL = 100 * mean of (sampled row's score - greedy row's score), the greedy
 * decode of the same member run first (compute_ciders, policies.py:145-193); SC_LOSS =
 * LogFitnessCriterion (fitness.py:12-40) of the sampled log-probs with those differences as rewards.
 * Sampled rows are not deduplicated: pass the batch with its seq_per_img copies per image (the rows
 * the reference samples independently). */
#define NICNES_FITNESS_GREEDY 0
#define NICNES_FITNESS_GREEDY_LOGPROB 1   /* AltLogFitnessCriterion */
#define NICNES_FITNESS_GREEDY_EXPPROB 2   /* ExpFitnessCriterion */
#define NICNES_FITNESS_GREEDY_LINPROB 3   /* LinFitnessCriterion */
#define NICNES_FITNESS_GREEDY_AVGPROB 4   /* AvgLogFitnessCriterion */
#define NICNES_FITNESS_SAMPLE 5           /* 'sample' */
#define NICNES_FITNESS_SELF_CRITICAL 6    /* 'self_critical' */
#define NICNES_FITNESS_SC_LOSS 7          /* 'sc_loss': LogFitnessCriterion */
int nicnes_set_fitness_mode(nicnes_handle* h, int32_t mode);

/* Rows per image of the sampled modes: each image of the batch is decoded n times (the reference's
 * seq_per_img copies, dataloader.py:175, which it samples independently), row r reading image r / n and
 * scored against its references; the rollout has B * n rows ([count, 2, B * n, seq_length] tokens). The
 * greedy modes decode one row per image (their copies are identical) and so does the self-critical
 * baseline. Default 1 (a caller may instead pass the copies as rows of the batch). */
int nicnes_set_rows_per_image(nicnes_handle* h, int32_t n);

/* Draws of the sampled modes (not a reference interface; the test hook that replays the reference's
 * numpy draws): the uniforms the next sampled evaluates use, u_host [count, 2, B, seq_length] fp64 (member,
 * sign, row, logit step), copied; n = 0 returns to the engine's own draws (a counter-based hash of the
 * noise seed, iteration, member, sign, row and step, 53-bit like RandomState.random_sample). */
int nicnes_set_sample_draws(nicnes_handle* h, const double* u_host, int64_t n);

/* nicnes_evaluate plus the per-step log-prob of each greedy token, FCModel._sample's seq_logprobs
 * (src/captioning/nets.py:191,208,241): logprob_out [count, 2, B, seq_length] fp32 or NULL. */
int nicnes_evaluate_lp(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                       double* fitness_out, int32_t* seq_out, float* logprob_out, void* stream);

/* nicnes_evaluate_lp where member member_begin + k decodes and is scored on batch
 * member_batch_host[k] (a HOST array of count entries in [0, n_batches), copied before return) of
 * the batches set by nicnes_set_batches. NULL = every member on batch 0 (only with one batch held).
 * Greedy decodes without log-prob output may bound lse from an exp-sum over pair maxima instead of
 * summing every exp (same tokens; rows the bound leaves undecided take the exact pass). The engine
 * switches to the exact sum for the next 32 such decodes when a bounded decode needed >= 2 exact
 * passes (peaked logits of trained models); env NICNES_BOUNDED_LSE=0 / 1 forces never / always. */
int nicnes_evaluate_batches(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                            const int32_t* member_batch_host, double* fitness_out, int32_t* seq_out, float* logprob_out,
                            void* stream);

/* CaptPolicy.rollout of theta itself (src/captioning/policies.py:86-128, called for the eval result
 * of nic_nes_worker.py:65-70 with the unperturbed parameters): fitness_out[0] = the fitness of the
 * batch (the one held, or batch `batch` of nicnes_set_batches), decoded ONCE. At sigma = 0 both
 * antithetic signs are theta, so sign + decodes the first ceil(B/2) images and sign - the rest and
 * the halves are scored as one rollout: seq_out [B, seq_length] int32 and logprob_out [B, seq_length]
 * (both nullable, rows 0..B-1 in batch order) and the fitness equal nicnes_evaluate_lp's sign-+
 * row of a sigma = 0 member bit for bit, at half its decode work. The sampled fitness modes draw from
 * the stream of `iteration` reserved for eval rollouts (member index 2^32 - 1 in the draw hash), so each
 * eval rollout draws afresh, as the reference's worker RNG does, and never shares an evolve member's
 * draws. */
int nicnes_evaluate_theta(nicnes_handle* h, int32_t batch, uint64_t iteration, double* fitness_out, int32_t* seq_out,
                          float* logprob_out, void* stream);

/* Centred ranks + antithetic weights over the WHOLE population, replaces
 * NESMaster.compute_centered_ranks and the weights line of gradient_estimate
 * (src/algorithm/nic_nes/nic_nes_master.py:170-205). fitness [P, 2] fp64 -> cr [P, 2] (or NULL),
 * w [P] fp32. */
int nicnes_rank_weights(nicnes_handle* h, const double* fitness, int32_t P, double* cr_out, float* w_out, void* stream);

/* gsum = sum over members [member_begin, +count) of w[i] * delta_i (fp32 result of an fp64 sum);
 * replaces batched_weighted_sum (nic_nes_master.py:207-221) without materialising delta.
 * `w` points at the weights of member_begin. Multi-GPU: all-reduce gsum between the call
 * and nicnes_adam_step. */
int nicnes_grad_partial(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, const float* w,
                        float sigma, float* gsum_out, void* stream);
/* The same sum on parameters [j0, j1) only (j0 a multiple of 64): gsum_out[j0 .. j1) written. Lets a
 * multi-GPU caller all-reduce one range while the next is summed (not a reference interface). */
int nicnes_grad_partial_range(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, const float* w,
                              float sigma, int64_t j0, int64_t j1, float* gsum_out, void* stream);

/* g = gsum / (2P); globalg = -g + l2coeff * theta; Adam step on the engine's theta
 * (nic_nes_master.py:126-137, optimizers.py:15-22,78-83). With ratio_out_host set it is
 * synchronising and returns the update ratio |step| / |theta_old| there; with NULL it only
 * enqueues, and nicnes_last_ratio reads the ratio later (so an iteration loop need not idle
 * the GPU once per step). */
int nicnes_adam_step(nicnes_handle* h, const float* gsum, int32_t P, double l2coeff, double stepsize, double beta1,
                     double beta2, double epsilon, double* ratio_out_host, void* stream);

/* The update ratio of the newest optimizer step (synchronising on `stream`). */
int nicnes_last_ratio(nicnes_handle* h, double* ratio_out_host, void* stream);

/* SGD with momentum in the same fused form (src/algorithm/nic_nes/optimizers.py:38-47). */
int nicnes_sgd_step(nicnes_handle* h, const float* gsum, int32_t P, double l2coeff, double stepsize, double momentum,
                    double* ratio_out_host, void* stream);

/* Optimizer.update(globalg) (optimizers.py:15-22) with a caller-provided globalg [D] widened to
 * fp64; globalg_fp32 = 1 when the caller's array was fp32 (numpy then keeps (1 - b) * globalg in
 * fp32). kind 0 = Adam (beta1, beta2, epsilon), 1 = SGD (beta1 = momentum). Synchronising (ratio). */
int nicnes_optimizer_update(nicnes_handle* h, int kind, const double* globalg, int globalg_fp32, double stepsize,
                            double beta1, double beta2, double epsilon, double* ratio_out_host, void* stream);

/* Multi-GPU data plane: one handle per GPU, one rank per handle. The reference
 * has no collective -- its master gathers every worker's 11.46 MB noise vector over redis and sums
 * them in gradient_estimate (src/dist.py:90-93,199-201, src/algorithm/nic_nes/nic_nes_master.py:
 * 92-123,170-182); the engine exchanges the (P, 2) fitness and one D-float noise sum over RCCL.
 * nicnes_comm_unique_id: rank 0 makes the 128-byte id and sends it to the other ranks out of band;
 * nicnes_comm_init: every rank joins (collective, blocking); nicnes_comm_attach borrows an
 * ncclComm_t the caller already owns (e.g. torch.distributed's); nicnes_comm_destroy releases.
 * nicnes_comm_count: the rank count and this rank's index as RCCL itself reports them
 * (ncclCommCount / ncclCommUserRank on the bound communicator; 1 and 0 with none bound) -- what a
 * multi-GPU bench line records to prove the collective saw N ranks (the reference's counterpart is
 * the number of live worker processes, src/main.py:144-153). */
#define NICNES_COMM_ID_BYTES 128
int nicnes_comm_unique_id(uint8_t* id_out_host);
int nicnes_comm_init(nicnes_handle* h, int32_t nranks, int32_t rank, const uint8_t* id_host);
int nicnes_comm_attach(nicnes_handle* h, void* nccl_comm);
int nicnes_comm_destroy(nicnes_handle* h);
int nicnes_comm_count(nicnes_handle* h, int32_t* nranks_out_host, int32_t* rank_out_host);
/* fit_all [P_local * nranks, 2] fp64 <- every rank's fit_local [P_local, 2], in rank order, so every
 * rank then ranks the whole population identically (compute_centered_ranks needs all 2P values). */
int nicnes_allgather_fitness(nicnes_handle* h, const double* fit_local, int32_t P_local, double* fit_all, void* stream);
/* gsum [D] fp32 summed in place over the ranks: the shards' nicnes_grad_partial results become the
 * whole population's noise sum before nicnes_adam_step (batched_weighted_sum, nic_nes_master.py:207-221). */
int nicnes_allreduce_grad(nicnes_handle* h, float* gsum, void* stream);

/* diagnostics since creation (synchronising): [0] = exact-pass fallbacks of the greedy tie rule,
 * [1] = sampled picks whose crossing stage's own sums stopped short of the threshold by rounding (its last id),
 * [2] = coop-path hand-off timeouts, [3] = sampled workgroups that found no free logit slot.
 * Decode faults ([2] or [3] nonzero: rows left undecoded) are sticky and contained on the device, in the
 * iteration that hit them, without a host wait: every fitness written from then on is NaN, nicnes_grad_partial
 * writes NaN everywhere (so an all-reduce carries the fault to every rank), and an optimizer step on this handle,
 * or on a noise sum whose first entry is NaN, leaves theta, m and v untouched. The error (NICNES_ERR_FAULT) is
 * returned by the next evaluate that finds the counters read back, and by the ratio read of the skipped step
 * (nicnes_adam_step / nicnes_sgd_step with ratio_out_host, nicnes_last_ratio); a skipped step is known by
 * the Adam kernel's own skip flag, so the NaN ratio of an applied step (0/0) is returned as a ratio, not an
 * error. The handle stays faulted until nicnes_clear_faults, or destroy it (the reference's worker process
 * dies and is restarted, main.py:107-141). */
int nicnes_stats(nicnes_handle* h, int64_t* out4_host);

/* Clear a contained decode fault (synchronising on the device): out2_host (nullable) receives the fault
 * counters [2], [3] of nicnes_stats before they are zeroed; the logit-slot claim flags are reset. theta, m
 * and v are those from before the faulted iteration (its step was skipped), so a caller can re-run that
 * iteration on the same handle (nicnes.master.EngineMaster.run does, once). Not a reference interface: the
 * reference's recovery is a fresh worker process (main.py:107-141). */
int nicnes_clear_faults(nicnes_handle* h, int64_t* out2_host);

/* Kernel timing with HIP events recorded on the launch stream around the decode and CIDEr-D
 * launches of nicnes_evaluate (off by default). nicnes_kernel_times synchronises on the events
 * and returns the last call's [0] = decode ms, [1] = CIDEr-D ms. */
int nicnes_set_timing(nicnes_handle* h, int on);
int nicnes_kernel_times(nicnes_handle* h, float* out2_host);

/* Per-kernel split of the last timed decode (events between its launches), in ms: [0] img-embed
 * kernel, [1] the two cell-only launches (t = -1, 0; one-launch-per-step builds only), [2] fused
 * path: the steps kernel (every step t = -1..T in one launch; or the per-step launches summed),
 * [3] its launch count, [4] split-path logit launches summed, [5] their count, [6] split-path cell
 * launches summed (token merge + next cell, t = -1..T), [7] their count. The coop path's one launch
 * counts as [2] / [3]. Synchronising. */
int nicnes_decode_phase_times(nicnes_handle* h, float* out8_host);

/* Decode launch shape. Not a reference interface: the reference decodes one member per CPU process
 * (src/algorithm/nic_nes/nic_nes_worker.py:142-154); the engine spreads a member over S workgroups
 * when members x slabs cannot fill the GPU. S = 0 / G = 0 pick automatically (S from the CU count,
 * G = 2 -- 64-row slabs -- when B pads to fewer rows that way, e.g. mscoco_nes.json batch_size 64).
 * G = 4 with S = 1 is the fused path (one launch for every step). Tokens do not depend on the shape. */
int nicnes_set_decode_split(nicnes_handle* h, int32_t S, int32_t G);
/* the shape an evaluate of `count` members of a B-image batch would use: [0] G, [1] slabs, [2] S */
int nicnes_decode_shape(nicnes_handle* h, int32_t B, int32_t count, int32_t* out3_host);
/* Decode streams (not a reference interface): the evaluate's members split evenly over n streams, the
 * caller's and n - 1 engine streams joined back into the caller's before the CIDEr-D launch, so that one
 * part's launches fill the CUs the others' launch gaps leave idle. n = 0 picks automatically (2 on the
 * split path, 1 on the fused path), 1..4 forces; env NICNES_DECODE_STREAMS sets the initial value. A
 * multi-stream decode records no per-launch events (nicnes_decode_phase_times reports zeros).
 * Tokens do not depend on n. */
int nicnes_set_decode_streams(nicnes_handle* h, int32_t n);
/* Coop decode (not a reference interface): when the split shape has 128-row slabs, S = 2 or 4 and every
 * workgroup fits on the GPU at once (S x members x slabs <= the kernel's occupancy x CUs, from
 * hipOccupancyMaxActiveBlocksPerMultiprocessor: 64 or 128 members per GPU at B = 128), the whole decode runs
 * as one persistent launch (env NICNES_COOP_LAUNCH=1: a cooperative launch, whose runtime check refuses a grid
 * that cannot be resident at once; 0.4 % slower per iteration at P = 64) whose S workgroups per
 * member slab hand the partial greedy states and h' to each other (mode 1, the default; env
 * NICNES_DECODE_COOP=0/1 sets the initial value), instead of two launches per step (mode 0). Tokens do not
 * depend on it. A partner missing for 0.5 s is a decode fault (nicnes_stats). */
int nicnes_set_decode_coop(nicnes_handle* h, int32_t mode);

/* SM-G-SUM sensitivity of the current theta on the first `rows` images of the batch held (batch 0):
 * replaces Sensitivity.calc_sensitivity / _calc_sum_sensitivity (src/algorithm/safe_mutations.py:34-117)
 * on CaptionModel.forward_for_sensitivity (src/captioning/nets.py:22-70; length 5, groups of 100).
 * out (device, D floats) = sqrt(sum_k J[k, :]^2) / rows, clamped to >= underflow and divided by it
 * (safe_mutations.py:63-65; underflow <= 0: the raw vector). The greedy tokens come from the engine's
 * bit-exact decode; the K = V1 / 100 + 1 backward passes run batched on the GPU, so the vector agrees
 * with the reference's to fp32 rounding (a stated tolerance), not bit for bit. Asynchronous on stream. */
int nicnes_sum_sensitivity(nicnes_handle* h, int32_t rows, float underflow, float* out_dev, void* stream);
/* the decode path an evaluate of `count` members of a B-image batch would take: 0 fused (one launch,
 * one workgroup per member slab), 1 split (two launches per step), 2 coop (the split shape in one launch) */
int nicnes_decode_path(nicnes_handle* h, int32_t B, int32_t count, int32_t* out_host);
/* the log-sum-exp mode of the last greedy decode enqueued: 1 the pair-bounded lse (greedy-only decodes while the
 * engine's adaptive policy allows it), 0 the exact exp-sum (log-probs written, NICNES_BOUNDED_LSE=0, or the policy's
 * exact stretch after a bounded decode needed exact passes). Measurement bookkeeping for bench.py (which kernel
 * instantiation a line's PMC counters belong to); no reference counterpart. */
int nicnes_last_decode_lse(nicnes_handle* h, int32_t* bounded_host);

#ifdef __cplusplus
}
#endif

#endif /* NICNES_H */
