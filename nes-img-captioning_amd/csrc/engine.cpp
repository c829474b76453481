// engine.cpp -- the C ABI of libnicnes (include/nicnes.h): handle state, validation, launches.
//
// Host-side orchestration only; the arithmetic lives in decode_kernel.hip, cider_kernel.hip and
// update_kernels.hip. Nothing here allocates or synchronises inside nicnes_evaluate /
// nicnes_grad_partial / nicnes_rank_weights, so a caller may capture them in a hipGraph.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include <rccl/rccl.h>

#include "../../include/nicnes.h"
#include "cider_kernel.h"
#include "decode_kernel.h"
#include "update_kernels.h"
#include "sensitivity.h"

#define MB_RING 4   // pinned staging slots of the member -> batch map (nicnes_evaluate_batches)

struct nicnes_handle {
    nicnes_config cfg;
    int device = 0;
    std::string err;
    int64_t off[10];
    int64_t D = 0;
    int32_t V1 = 0;

    const float* noise = nullptr;
    uint64_t noise_len = 0;

    double* theta64 = nullptr;
    float* theta32 = nullptr;
    double* m = nullptr;
    double* v = nullptr;
    int64_t t = 0;
    int theta_is_fp32 = 0;
    bool theta_set = false;

    const float* fc = nullptr;
    int32_t B = 0;                    // rows (images) decoded per member
    int32_t n_batches = 1;            // batches held (single_batch: false holds several)
    int32_t n_img = 0;                // images held = n_batches * B
    int32_t img_cap = 0;              // per-image CIDEr-D table capacity
    int32_t* mbatch = nullptr;        // [max_members] member -> batch map of the current evaluate
    // the caller's host map is staged in a ring of pinned buffers (each reused only after its copy has
    // run, told by its event), so an evaluate with a map never waits for the queued GPU work
    int32_t* mb_pin[MB_RING] = {};
    hipEvent_t mb_ev[MB_RING] = {};
    bool mb_used[MB_RING] = {};
    int mb_next = 0;
    int32_t n_refs = 0;
    const int32_t* img_ref_start = nullptr;
    bool batch_set = false;

    const uint64_t* df_keys = nullptr;
    const double* df_vals = nullptr;
    int64_t df_n = 0;
    uint64_t* hash_keys = nullptr;   // engine-owned open-addressing copy of the df table
    double* hash_vals = nullptr;
    uint64_t hash_mask = 0;
    double ref_len = 0.0;
    bool df_set = false;

    uint64_t* img_hkey = nullptr;     // per-image reference n-gram tables (CIDEr-D)
    int32_t* img_hrow = nullptr;
    double* img_vr = nullptr;
    bool img_tables = false;          // every image has <= IMG_MAXR references
    uint64_t* ref_keys = nullptr;
    double* ref_vec = nullptr;
    int32_t* ref_count = nullptr;
    int32_t* ref_len2 = nullptr;
    double* ref_norm = nullptr;

    uint64_t* nidx = nullptr;
    int32_t* seq = nullptr;
    float* lp = nullptr;              // per-step log-probs for the greedy_* criteria
    double* row_scores = nullptr;     // per-row CIDEr-D of the image-table scorer [2 * max_members, max_batch]
    int fitness_mode = 0;             // nicnes_set_fitness_mode (0 = 'greedy')
    double* su = nullptr;             // sampled modes: the draws of a decode [count, 2, B, T]
    double* base_scores = nullptr;    // self-critical modes: the greedy rows' CIDEr-D [2 count, B]
    int64_t su_cap = 0, base_cap = 0; // ... their capacities (doubles)
    float* slog = nullptr;            // sampled modes: logit slots of the steps kernel (one per resident workgroup + spare)
    int32_t* slog_slots = nullptr;    // ... their claim flags (zero between launches)
    int slog_ns = 0;
    std::vector<double> su_host;      // nicnes_set_sample_draws (test hook): draws to use instead of the engine's
    int rpi = 1;                      // nicnes_set_rows_per_image: rows the sampled modes decode per image
    float* dscratch = nullptr;
    unsigned long long* zcount = nullptr; // nicnes_theta_zeros: the count of exact zeros of theta32
    int32_t* stats = nullptr;
    int32_t* alive = nullptr;         // per decode workgroup: rows left unfinished (fused [stride], split [2][stride])
    int32_t alive_stride = 0;         // max decode workgroups (members x 64-row slabs)
    float* part = nullptr;            // split decode: partial greedy states
    float* noise_sc = nullptr;        // fp32(sc_sigma * table): what the decode kernels read (no multiply per use)
    float sc_sigma = 0.f;
    bool sc_valid = false;
    int mut_mode = 0;                 // nicnes_set_mutation: 0 plain, 1 divide, 2 multiply
    bool mut_full = false;            // NICNES_MUT_FULL=1: materialise every parameter's delta' (no decode-formed head)
    float* mut_vec = nullptr;         // [D] sensitivity (mode 1) or |theta| scale (mode 2)
    float* dbuf = nullptr;            // [max_members, Dp] the members' mutated deltas (mode != 0)
    uint64_t* didx = nullptr;         // [max_members] k * Dp: row offsets of dbuf
    int64_t Dp = 0;
    uint64_t* rank_key = nullptr;     // rank sort scratch (grown to the largest population ranked)
    uint32_t* rank_idx = nullptr;
    size_t rank_cap = 0;
    int64_t part_cap = 0;             // in logit workgroups (members x slabs x S)
    int n_cu = 256;
    int dec_S = 0, dec_G = 0;         // nicnes_set_decode_split (0 = automatic)
    // the decode's members in n parts on n streams (nicnes_set_decode_streams, NICNES_DECODE_STREAMS;
    // 0 = automatic: 2 on the split path, 1 on the fused path): one part's launches fill the CUs the
    // others' launch gaps and tails leave idle
    int dec_streams = 0;
    int coop_mode = 1;                // nicnes_set_decode_coop: 0 never, 1 the split shape in one launch when it fits
    int coop_occ = 1;                 // coop kernel workgroups resident per CU (occupancy API): the grid bound
    int sample_occ = 1;               // sampled steps kernel workgroups resident per CU: the logit slots needed
    // NICNES_COOP_LAUNCH=1: hipLaunchCooperativeKernel for the coop kernel. The default plain launch gets the same
    // residency from the same occupancy-bounded grid (coop_fits; MI355X_MICROARCH.md: the cooperative launch adds
    // only the runtime's check of that bound) and costs 0.4 % less per iteration at P = 64 (r04 A/B)
    int coop_launch = 0;
    uint32_t test_stall_ms = 0;       // test hook NICNES_TEST_COOP_STALL (ms): coop workgroup 0 starts late
    int test_stall_left = -1;         // ... on the first NICNES_TEST_COOP_STALL_LAUNCHES coop launches only (-1: all)
    int test_slots = 0;               // test hook NICNES_TEST_SLOTS: this many sampled logit slots (0 = enough)
    uint32_t* coop_ctr = nullptr;     // [max_members * slabs * COOP_CTR_STRIDE] coop hand-off counters
    SensWork* sens = nullptr;         // SM-G-SUM sensitivity work buffers (nicnes_sum_sensitivity)
    float* zero_noise = nullptr;      // [D] zeros + one zero index: the sigma = 0 decode of the sensitivity
    uint64_t* zero_idx = nullptr;
    int32_t* sens_tok = nullptr;      // [2 * max_batch * 4] its greedy tokens
    hipStream_t sx[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_fork = nullptr;
    hipEvent_t ev_join[3] = {nullptr, nullptr, nullptr};
    double* partials = nullptr;
    double* norms = nullptr;

    ncclComm_t comm = nullptr;        // population shards over ranks (nicnes_comm_init / _attach)
    bool comm_owned = false;
    int comm_nranks = 1;

    bool timing = false;
    int force_exact = 0;      // test hook: exact tie pass on every step (NICNES_FORCE_EXACT=1)
    float lse_margin = 2e-3f; // bounded-lse margin; test hook NICNES_LSE_MARGIN widens it (more undecided rows)
    // bounded-lse policy: greedy-only decodes use the pair-bounded lse unless the previous bounded decode
    // sent rows to the exact pass (peaked, trained-model logits put lse near binade edges); then the
    // next exact_span decodes sum the exp exactly. The fallback counter is read back asynchronously.
    int bounded_mode = 2;     // NICNES_BOUNDED_LSE: 0 never, 1 always, 2 adaptive
    int exact_left = 0;
    int last_bounded = 0;
    int last_decode_bounded = 0;      // nicnes_last_decode_lse: the lse mode of the last decode enqueued
    int32_t fb_seen = 0;
    int32_t* stats_host = nullptr;
    hipEvent_t stats_ev = nullptr;
    bool stats_pending = false;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    hipEvent_t dev[DECODE_MAX_EVENTS] = {};   // between the decode's launches (phase split)
    int dev_kind[DECODE_MAX_EVENTS] = {};     // kind of the launch each event follows (DK_*)
    int n_dev = 0;                            // events recorded by the last timed decode
    bool multi_stream = false;                // the last decode ran on several streams
    bool last_nes_form = true;                // the newest optimizer step took the noise sum (not a globalg)
    // a skipped step (the Adam kernel's skip flag) leaves theta, m, v untouched; the host state it advanced
    // (t, theta_is_fp32) is rolled back once the flag is seen, so a re-run of the iteration steps as the first try would
    bool step_pending_check = false;
    int64_t t_prev = 0;
    int theta_fp32_prev = 0;
};

namespace {

int fail(nicnes_handle* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

#define HIPC(h, expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((h), NICNES_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

void layout(const nicnes_config* c, int64_t* off) {
    const int64_t V1 = (int64_t)c->vocab_size + 1, E = c->input_encoding_size, R = c->rnn_size,
                  F = c->fc_feat_size;
    int64_t o = 0;
    off[0] = o; o += E * F;        // img_embed.weight
    off[1] = o; o += E;            // img_embed.bias
    off[2] = o; o += V1 * E;       // embed.weight
    off[3] = o; o += V1 * R;       // logit.weight
    off[4] = o; o += V1;           // logit.bias
    off[5] = o; o += 5 * R * E;    // core.i2h.weight
    off[6] = o; o += 5 * R;        // core.i2h.bias
    off[7] = o; o += 5 * R * R;    // core.h2h.weight
    off[8] = o; o += 5 * R;        // core.h2h.bias
    off[9] = o;
}

__global__ void f64_to_f32_kernel(const double* in, float* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)in[i];
}

// decode shape: G row groups per slab (4: 128-row slabs; 2: 64-row slabs when that pads fewer rows,
// e.g. mscoco_nes.json's batch_size 64), and S logit workgroups per member slab
int auto_G(int B) { return (B + 63) / 64 * 64 < (B + 127) / 128 * 128 ? 2 : 4; }
int nslabs_of(int B, int G) { return (B + 32 * G - 1) / (32 * G); }

// S minimising the makespan ceil(n_wg * S / n_cu) * (1/S + per-workgroup overhead); the split path
// (two launches per step) is charged 2 % over the fused step kernel
int auto_split(int64_t n_wg, int n_cu, int G) {
    int best = 1;
    double bc = 1e300;
    for (int S = 1; S <= 16; S *= 2) {
        const double rounds = std::ceil((double)n_wg * S / n_cu);
        const double cost = rounds * (1.0 / S + 0.03) * ((G == 4 && S > 1) ? 1.02 : 1.0);
        if (cost < bc - 1e-12) {
            bc = cost;
            best = S;
        }
    }
    return best;
}

// logit workgroups the automatic rule can ask for, up to max_members x the widest slab count
int64_t auto_part_cap(int max_members, int max_batch, int n_cu) {
    int64_t cap = 1;
    for (int G = 2; G <= 4; G += 2) {
        const int ns = nslabs_of(max_batch, G);
        for (int64_t n = 1; n <= (int64_t)max_members * ns; ++n)
            cap = std::max(cap, n * auto_split(n, n_cu, G));
    }
    return cap;
}

template <class T>
int dalloc(nicnes_handle* h, T** p, size_t n) {
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e != hipSuccess) return fail(h, NICNES_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return NICNES_OK;
}

void decode_shape(const nicnes_handle* h, int B, int count, int* G, int* nslabs, int* S) {
    *G = h->dec_G ? h->dec_G : auto_G(B);
    *nslabs = nslabs_of(B, *G);
    *S = h->dec_S ? h->dec_S : auto_split((int64_t)count * *nslabs, h->n_cu, *G);
}

// The coop path (the split shape in one persistent launch, nicnes_decode_coop_kernel): 128-row slabs, 2 or
// 4 logit ranges per member slab, and every workgroup of the launch resident at once (one per CU).
bool coop_fits(const nicnes_handle* h, int G, int nslabs, int S, int count) {
    // (nst >= S: coop_step assumes every logit range non-empty; the split path handles empty ranges)
    return h->coop_mode && G == 4 && (S == 2 || S == 4) && (h->V1 + 63) / 64 >= S &&
           (int64_t)count * nslabs * S <= (int64_t)h->coop_occ * h->n_cu;
}

// Buffers sized by the reference count: the cooked reference n-gram vectors (CIDEr-D).
int alloc_refs(nicnes_handle* h, int max_refs) {
    void* old[] = {h->ref_keys, h->ref_vec, h->ref_count, h->ref_len2, h->ref_norm};
    for (void* q : old)
        if (q) (void)hipFree(q);
    h->ref_keys = nullptr; h->ref_vec = nullptr; h->ref_count = nullptr; h->ref_len2 = nullptr; h->ref_norm = nullptr;
    const size_t MR = (size_t)max_refs;
    int rc = dalloc(h, &h->ref_keys, MR * 64);
    if (!rc) rc = dalloc(h, &h->ref_vec, MR * 64);
    if (!rc) rc = dalloc(h, &h->ref_count, MR);
    if (!rc) rc = dalloc(h, &h->ref_len2, MR);
    if (!rc) rc = dalloc(h, &h->ref_norm, MR * 4);
    if (!rc) h->cfg.max_refs = max_refs;
    return rc;
}

// Buffers sized by the batch: per-image n-gram tables, tokens / log-probs / row scores of a launch,
// decode lane scratch, alive flags and partial states.
int alloc_batch(nicnes_handle* h, int max_batch) {
    void* old[] = {h->seq, h->lp, h->row_scores, h->dscratch, h->alive, h->part};
    for (void* q : old)
        if (q) (void)hipFree(q);
    h->seq = nullptr; h->lp = nullptr; h->row_scores = nullptr; h->dscratch = nullptr; h->alive = nullptr;
    h->part = nullptr;
    if (h->coop_ctr) (void)hipFree(h->coop_ctr);
    h->coop_ctr = nullptr;
    const size_t MM = (size_t)h->cfg.max_members, MB = (size_t)max_batch, T = (size_t)h->cfg.seq_length;
    // lane scratch: 2G row waves per slab, the larger of the two slab layouts
    const int rw = std::max(8 * nslabs_of((int)MB, 4), 4 * nslabs_of((int)MB, 2));
    h->alive_stride = (int32_t)(MM * (size_t)nslabs_of((int)MB, 2));
    const int ns = std::max(nslabs_of((int)MB, 2), nslabs_of((int)MB, 4));
    h->part_cap = std::max(auto_part_cap((int)MM, (int)MB, h->n_cu), (int64_t)MM * ns * std::max(h->dec_S, 1));
    int rc = dalloc(h, &h->seq, MM * 2 * MB * T);
    if (!rc) rc = dalloc(h, &h->lp, MM * 2 * MB * T);
    if (!rc) rc = dalloc(h, &h->row_scores, MM * 2 * MB);
    if (!rc) rc = dalloc(h, &h->dscratch, nicnes_decode_scratch_floats((int)MM, rw));
    if (!rc) rc = dalloc(h, &h->coop_ctr, MM * (size_t)ns * COOP_CTR_STRIDE);
    if (!rc) rc = dalloc(h, &h->alive, 3 * (size_t)h->alive_stride);
    if (!rc) rc = dalloc(h, &h->part, (size_t)h->part_cap * PART_FLOATS);
    if (!rc) h->cfg.max_batch = max_batch;
    return rc;
}

// Per-image CIDEr-D n-gram tables for every image held (all batches of a per-member-batch evaluate).
int alloc_images(nicnes_handle* h, int n_img) {
    void* old[] = {h->img_hkey, h->img_hrow, h->img_vr};
    for (void* q : old)
        if (q) (void)hipFree(q);
    h->img_hkey = nullptr; h->img_hrow = nullptr; h->img_vr = nullptr;
    const size_t N = (size_t)n_img;
    int rc = dalloc(h, &h->img_hkey, N * IMG_CAP);
    if (!rc) rc = dalloc(h, &h->img_hrow, N * IMG_CAP);
    if (!rc) rc = dalloc(h, &h->img_vr, N * IMG_ROWS * IMG_MAXR);
    if (!rc) h->img_cap = n_img;
    return rc;
}

}  // namespace

extern "C" {

int64_t nicnes_param_count(const nicnes_config* cfg) {
    if (!cfg) return -1;
    int64_t off[10];
    layout(cfg, off);
    return off[9];
}

int nicnes_param_offsets(const nicnes_config* cfg, int64_t* out10_host) {
    if (!cfg || !out10_host) return NICNES_ERR_INVALID;
    layout(cfg, out10_host);
    return NICNES_OK;
}

int nicnes_create(const nicnes_config* cfg, int device, nicnes_handle** out) {
    if (!cfg || !out) return NICNES_ERR_INVALID;
    *out = nullptr;
    const int V1 = cfg->vocab_size + 1;
    if (cfg->input_encoding_size != 128 || cfg->rnn_size != 128) return NICNES_ERR_UNSUPPORTED;
    if (cfg->fc_feat_size <= 0 || cfg->fc_feat_size % 128 != 0) return NICNES_ERR_UNSUPPORTED;
    if (V1 % 4 != 0 || V1 < 8 || V1 > 16384) return NICNES_ERR_UNSUPPORTED;
    if (cfg->seq_length < 1 || cfg->seq_length > 16) return NICNES_ERR_UNSUPPORTED;
    if (cfg->max_batch < 1 || cfg->max_batch > 1024 || cfg->max_members < 1 || cfg->max_refs < 1)
        return NICNES_ERR_INVALID;
    nicnes_handle* h = new nicnes_handle();
    h->cfg = *cfg;
    h->device = device;
    h->V1 = V1;
    layout(cfg, h->off);
    h->D = h->off[9];
    if (h->D * 4 >= (int64_t)1 << 32) {
        delete h;
        return NICNES_ERR_UNSUPPORTED;
    }
    if (cfg->noise_len < (uint64_t)h->D) {
        delete h;
        return NICNES_ERR_INVALID;
    }
    if (hipSetDevice(device) != hipSuccess) {
        delete h;
        return NICNES_ERR_HIP;
    }
    const size_t D = (size_t)h->D, MM = (size_t)cfg->max_members;
    int rc = NICNES_OK;
    if (!rc) rc = dalloc(h, &h->theta64, D);
    if (!rc) rc = dalloc(h, &h->theta32, D);
    if (!rc) rc = dalloc(h, &h->m, D);
    if (!rc) rc = dalloc(h, &h->v, D);
    if (!rc) rc = dalloc(h, &h->nidx, MM);
    {
        const char* fe = getenv("NICNES_FORCE_EXACT");
        h->force_exact = (fe && fe[0] == '1') ? 1 : 0;
        const char* lm = getenv("NICNES_LSE_MARGIN");
        if (lm && lm[0]) h->lse_margin = (float)atof(lm);
        const char* mf = getenv("NICNES_MUT_FULL");
        h->mut_full = mf && mf[0] == '1';
        const char* bl = getenv("NICNES_BOUNDED_LSE");
        if (bl && (bl[0] == '0' || bl[0] == '1')) h->bounded_mode = bl[0] - '0';
        const char* ds = getenv("NICNES_DECODE_STREAMS");
        if (ds && ds[0] >= '1' && ds[0] <= '4' && ds[1] == 0) h->dec_streams = ds[0] - '0';
        const char* dc = getenv("NICNES_DECODE_COOP");
        if (dc && (dc[0] == '0' || dc[0] == '1') && dc[1] == 0) h->coop_mode = dc[0] - '0';
        const char* cl = getenv("NICNES_COOP_LAUNCH");
        if (cl && (cl[0] == '0' || cl[0] == '1') && cl[1] == 0) h->coop_launch = cl[0] - '0';
        const char* st = getenv("NICNES_TEST_COOP_STALL");
        if (st && st[0]) h->test_stall_ms = (uint32_t)atoi(st);
        const char* sl = getenv("NICNES_TEST_COOP_STALL_LAUNCHES");
        if (sl && sl[0]) h->test_stall_left = atoi(sl);
        const char* ts = getenv("NICNES_TEST_SLOTS");
        if (ts && ts[0]) h->test_slots = atoi(ts);
    }
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
            h->n_cu = ncu;
    }
    if (!rc && nicnes_decode_init() != hipSuccess) rc = fail(h, NICNES_ERR_HIP, "nicnes_decode_init");
    if (!rc && (nicnes_decode_occupancy(&h->coop_occ, &h->sample_occ) != hipSuccess || h->coop_occ < 1 ||
                h->sample_occ < 1))
        rc = fail(h, NICNES_ERR_HIP, "nicnes_decode_occupancy");
    if (!rc) rc = dalloc(h, &h->stats, 4);
    if (!rc && hipHostMalloc((void**)&h->stats_host, 4 * sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
        rc = fail(h, NICNES_ERR_HIP, "hipHostMalloc");
    if (!rc && hipEventCreateWithFlags(&h->stats_ev, hipEventDisableTiming) != hipSuccess)
        rc = fail(h, NICNES_ERR_HIP, "hipEventCreate");
    if (!rc) rc = dalloc(h, &h->partials, 2 * (size_t)nicnes_adam_blocks(h->D));
    if (!rc) rc = dalloc(h, &h->norms, 3);       // |step|^2, |theta|^2, the skip flag
    if (!rc) {
        h->rank_cap = nicnes_rank_scratch_pairs(2 * cfg->max_members);
        rc = dalloc(h, &h->rank_key, h->rank_cap);
        if (!rc) rc = dalloc(h, &h->rank_idx, h->rank_cap);
    }
    if (!rc) rc = alloc_refs(h, cfg->max_refs);
    if (!rc) rc = alloc_batch(h, cfg->max_batch);
    if (!rc) rc = alloc_images(h, cfg->max_batch);
    if (!rc) rc = dalloc(h, &h->mbatch, (size_t)cfg->max_members);
    for (int i = 0; i < MB_RING && !rc; ++i) {
        if (hipHostMalloc((void**)&h->mb_pin[i], (size_t)cfg->max_members * sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
            rc = fail(h, NICNES_ERR_HIP, "hipHostMalloc");
        else if (hipEventCreateWithFlags(&h->mb_ev[i], hipEventDisableTiming) != hipSuccess)
            rc = fail(h, NICNES_ERR_HIP, "hipEventCreate");
    }
    if (rc) {
        nicnes_destroy(h);
        return rc;
    }
    (void)hipMemset(h->m, 0, D * sizeof(double));
    (void)hipMemset(h->v, 0, D * sizeof(double));
    (void)hipMemset(h->stats, 0, 4 * sizeof(int32_t));
    if (hipDeviceSynchronize() != hipSuccess) {
        nicnes_destroy(h);
        return NICNES_ERR_HIP;
    }
    *out = h;
    return NICNES_OK;
}

int nicnes_destroy(nicnes_handle* h) {
    if (!h) return NICNES_OK;
    (void)hipSetDevice(h->device);
    if (h->comm && h->comm_owned) (void)ncclCommDestroy(h->comm);
    void* bufs[] = {h->theta64, h->theta32, h->m, h->v, h->ref_keys, h->ref_vec, h->ref_count, h->ref_len2,
                    h->ref_norm, h->nidx, h->seq, h->lp, h->row_scores, h->dscratch, h->stats, h->partials, h->norms,
                    h->hash_keys, h->hash_vals, h->img_hkey, h->img_hrow, h->img_vr, h->alive, h->part,
                    h->rank_key, h->rank_idx, h->mbatch, h->mut_vec, h->dbuf, h->didx, h->noise_sc, h->coop_ctr,
                    h->zero_noise, h->zero_idx, h->sens_tok, h->su, h->base_scores, h->slog, h->slog_slots, h->zcount};
    if (h->sens) nicnes_sens_destroy(h->sens);
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (h->stats_pending) (void)hipEventSynchronize(h->stats_ev);
    if (h->stats_host) (void)hipHostFree(h->stats_host);
    if (h->stats_ev) (void)hipEventDestroy(h->stats_ev);
    for (int i = 0; i < MB_RING; ++i) {
        if (h->mb_ev[i]) {
            (void)hipEventSynchronize(h->mb_ev[i]);
            (void)hipEventDestroy(h->mb_ev[i]);
        }
        if (h->mb_pin[i]) (void)hipHostFree(h->mb_pin[i]);
    }
    for (hipEvent_t e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : h->dev)
        if (e) (void)hipEventDestroy(e);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    for (int i = 0; i < 3; ++i) {
        if (h->ev_join[i]) (void)hipEventDestroy(h->ev_join[i]);
        if (h->sx[i]) {
            (void)hipStreamSynchronize(h->sx[i]);
            (void)hipStreamDestroy(h->sx[i]);
        }
    }
    delete h;
    return NICNES_OK;
}

const char* nicnes_last_error(const nicnes_handle* h) { return h ? h->err.c_str() : "null handle"; }

int nicnes_set_noise_table(nicnes_handle* h, const float* table, uint64_t len) {
    if (!h || !table) return NICNES_ERR_INVALID;
    if (len != h->cfg.noise_len) return fail(h, NICNES_ERR_INVALID, "noise table length != config.noise_len");
    if (((uintptr_t)table & 15u) != 0) return fail(h, NICNES_ERR_INVALID, "noise table must be 16-byte aligned");
    h->noise = table;
    h->noise_len = len;
    h->sc_valid = false;          // the sigma-scaled copy is rebuilt at the next evaluation
    return NICNES_OK;
}

int nicnes_set_theta(nicnes_handle* h, const double* theta64, int is_fp32_origin, void* stream) {
    if (!h || !theta64) return NICNES_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, hipMemcpyAsync(h->theta64, theta64, (size_t)h->D * sizeof(double), hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(f64_to_f32_kernel, dim3((unsigned)((h->D + 255) / 256)), dim3(256), 0, s, h->theta64,
                       h->theta32, h->D);
    HIPC(h, hipGetLastError());
    h->theta_is_fp32 = is_fp32_origin ? 1 : 0;
    h->step_pending_check = false;
    h->theta_set = true;
    return NICNES_OK;
}

int nicnes_get_theta(nicnes_handle* h, double* theta64_out, float* theta32_out, void* stream) {
    if (!h || !h->theta_set) return NICNES_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    if (theta64_out)
        HIPC(h, hipMemcpyAsync(theta64_out, h->theta64, (size_t)h->D * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (theta32_out)
        HIPC(h, hipMemcpyAsync(theta32_out, h->theta32, (size_t)h->D * sizeof(float), hipMemcpyDeviceToDevice, s));
    return NICNES_OK;
}

int nicnes_set_adam_state(nicnes_handle* h, const double* m, const double* v, int64_t t, void* stream) {
    if (!h || !m || !v || t < 0) return NICNES_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, hipMemcpyAsync(h->m, m, (size_t)h->D * sizeof(double), hipMemcpyDeviceToDevice, s));
    HIPC(h, hipMemcpyAsync(h->v, v, (size_t)h->D * sizeof(double), hipMemcpyDeviceToDevice, s));
    h->t = t;
    h->step_pending_check = false;
    return NICNES_OK;
}

int nicnes_get_adam_state(nicnes_handle* h, double* m_out, double* v_out, int64_t* t_out_host, void* stream) {
    if (!h) return NICNES_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    if (m_out) HIPC(h, hipMemcpyAsync(m_out, h->m, (size_t)h->D * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (v_out) HIPC(h, hipMemcpyAsync(v_out, h->v, (size_t)h->D * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (t_out_host) *t_out_host = h->t;
    return NICNES_OK;
}

static CiderTables tables_of(nicnes_handle* h) {
    CiderTables tb;
    tb.df_keys = h->df_keys;
    tb.df_vals = h->df_vals;
    tb.df_n = h->df_n;
    tb.hash_keys = h->hash_keys;
    tb.hash_vals = h->hash_vals;
    tb.hash_mask = h->hash_mask;
    tb.ref_len = h->ref_len;
    tb.ref_keys = h->ref_keys;
    tb.ref_vec = h->ref_vec;
    tb.ref_count = h->ref_count;
    tb.ref_len2 = h->ref_len2;
    tb.ref_norm = h->ref_norm;
    tb.img_hkey = h->img_hkey;
    tb.img_hrow = h->img_hrow;
    tb.img_vr = h->img_vr;
    tb.fault = h->stats;
    return tb;
}

int nicnes_set_df_table(nicnes_handle* h, const uint64_t* keys, const double* df, int64_t n, double ref_len_log) {
    if (!h || n < 0 || (n > 0 && (!keys || !df))) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    if (h->hash_keys) (void)hipFree(h->hash_keys);
    if (h->hash_vals) (void)hipFree(h->hash_vals);
    h->hash_keys = nullptr;
    h->hash_vals = nullptr;
    const uint64_t cap = nicnes_df_hash_capacity(n);
    int rc = dalloc(h, &h->hash_keys, cap);
    if (rc) return rc;
    rc = dalloc(h, &h->hash_vals, cap);
    if (rc) return rc;
    HIPC(h, hipMemset(h->hash_keys, 0, cap * sizeof(uint64_t)));
    HIPC(h, nicnes_launch_df_hash_build(keys, df, n, h->hash_keys, h->hash_vals, cap - 1, nullptr));
    HIPC(h, hipDeviceSynchronize());
    h->hash_mask = cap - 1;
    h->df_keys = keys;
    h->df_vals = df;
    h->df_n = n;
    h->ref_len = ref_len_log;
    h->df_set = true;
    h->batch_set = false;   // reference vectors depend on the df table: set the batch again
    return NICNES_OK;
}

int nicnes_set_batches(nicnes_handle* h, const float* fc, int32_t n_batches, int32_t B, const int32_t* ref_tokens,
                       int32_t n_refs, const int32_t* img_ref_start, void* stream) {
    if (!h || !fc || !ref_tokens || !img_ref_start) return NICNES_ERR_INVALID;
    if (B < 1 || B > 1024) return fail(h, NICNES_ERR_INVALID, "B out of [1, 1024]");
    if (n_batches < 1 || (int64_t)n_batches * B > (1 << 20)) return fail(h, NICNES_ERR_INVALID, "n_batches out of range");
    const int n_img = n_batches * B;
    if (n_refs < n_img) return fail(h, NICNES_ERR_INVALID, "n_refs < images");
    if (!h->df_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_df_table first");
    if (((uintptr_t)fc & 15u) != 0) return fail(h, NICNES_ERR_INVALID, "fc must be 16-byte aligned");
    HIPC(h, hipSetDevice(h->device));
    // a batch-size curriculum (bs_multiplier, tools/iteration.py:149-153) or more batches can outgrow
    // the sizes the handle was created with: re-create those buffers (outside every evaluate, so no
    // launch in flight uses them once the device is idle)
    if (B > h->cfg.max_batch || n_refs > h->cfg.max_refs || n_img > h->img_cap) {
        HIPC(h, hipDeviceSynchronize());
        int rc = NICNES_OK;
        if (n_refs > h->cfg.max_refs) rc = alloc_refs(h, std::max(n_refs, 2 * h->cfg.max_refs));
        if (!rc && B > h->cfg.max_batch) rc = alloc_batch(h, B);
        if (!rc && n_img > h->img_cap) rc = alloc_images(h, n_img);
        if (rc) {
            h->batch_set = false;
            return rc;
        }
    }
    // reference ranges: CiderD asserts every image has references (len(ref) > 0, upstream
    // cider_scorer); ranges must tile [0, n_refs)
    std::vector<int32_t> st((size_t)n_img + 1);
    HIPC(h, hipMemcpyAsync(st.data(), img_ref_start, st.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
    HIPC(h, hipStreamSynchronize((hipStream_t)stream));
    int maxr = 0;
    bool ok = st[0] == 0 && st[n_img] == n_refs;
    for (int b = 0; b < n_img && ok; ++b) {
        ok = st[b + 1] > st[b];
        maxr = std::max(maxr, st[b + 1] - st[b]);
    }
    if (!ok) {
        h->batch_set = false;
        return fail(h, NICNES_ERR_INVALID, "img_ref_start must start at 0, end at n_refs and give every image >= 1 reference");
    }
    h->fc = fc;
    h->B = B;
    h->n_batches = n_batches;
    h->n_img = n_img;
    h->n_refs = n_refs;
    h->img_ref_start = img_ref_start;
    CiderTables tb = tables_of(h);
    HIPC(h, nicnes_launch_cook_refs(ref_tokens, n_refs, h->cfg.seq_length, &tb, (hipStream_t)stream));
    // per-image n-gram tables when every image has at most IMG_MAXR references (else the
    // per-reference scan kernel scores the candidates)
    h->img_tables = maxr <= IMG_MAXR;
    if (h->img_tables) {
        HIPC(h, hipMemsetAsync(h->img_vr, 0, (size_t)n_img * IMG_ROWS * IMG_MAXR * sizeof(double), (hipStream_t)stream));
        HIPC(h, nicnes_launch_img_ngrams(img_ref_start, n_img, &tb, (hipStream_t)stream));
    }
    h->batch_set = true;
    return NICNES_OK;
}

int nicnes_set_batch(nicnes_handle* h, const float* fc, int32_t B, const int32_t* ref_tokens, int32_t n_refs,
                     const int32_t* img_ref_start, void* stream) {
    return nicnes_set_batches(h, fc, 1, B, ref_tokens, n_refs, img_ref_start, stream);
}

int nicnes_noise_indices(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, uint64_t* out,
                         void* stream) {
    if (!h || !out || member_begin < 0 || count < 0) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, nicnes_launch_noise_index(h->cfg.noise_seed, iteration, (uint64_t)member_begin, count, h->cfg.noise_len,
                                      (uint64_t)h->D, out, (hipStream_t)stream));
    return NICNES_OK;
}

int nicnes_noise_vectors(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                         float* out, void* stream) {
    if (!h || !out || member_begin < 0 || count < 1) return NICNES_ERR_INVALID;
    if (count > h->cfg.max_members) return fail(h, NICNES_ERR_INVALID, "count > max_members");
    if (!h->noise) return fail(h, NICNES_ERR_INVALID, "nicnes_set_noise_table first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, nicnes_launch_noise_index(h->cfg.noise_seed, iteration, (uint64_t)member_begin, count, h->cfg.noise_len,
                                      (uint64_t)h->D, h->nidx, s));
    if (h->mut_mode)
        HIPC(h, nicnes_launch_mutate(h->noise, h->nidx, count, h->D, sigma, h->mut_vec, h->mut_mode, out, h->D, s));
    else
        HIPC(h, nicnes_launch_noise_vectors(h->noise, h->nidx, count, h->D, sigma, out, s));
    return NICNES_OK;
}

int nicnes_set_mutation(nicnes_handle* h, int32_t mode, const float* vec, void* stream) {
    if (!h || mode < 0 || mode > 2 || (mode && !vec)) return NICNES_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    if (mode && !h->mut_vec) {       // first use: the [D] vector
        HIPC(h, hipDeviceSynchronize());
        int rc = dalloc(h, &h->mut_vec, (size_t)h->D);
        if (rc) return rc;
    }
    if (mode) HIPC(h, hipMemcpyAsync(h->mut_vec, vec, (size_t)h->D * sizeof(float), hipMemcpyDeviceToDevice, s));
    h->mut_mode = mode;
    return NICNES_OK;
}

int nicnes_set_mutation_proportional(nicnes_handle* h, float mean_abs, void* stream) {
    if (!h || !(mean_abs >= 0.f)) return NICNES_ERR_INVALID;
    if (!h->theta_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_theta first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    if (!h->mut_vec) {               // first use: the [D] vector
        HIPC(h, hipDeviceSynchronize());
        int rc = dalloc(h, &h->mut_vec, (size_t)h->D);
        if (rc) return rc;
    }
    HIPC(h, nicnes_launch_proportional(h->theta32, h->D, mean_abs, h->mut_vec, s));
    h->mut_mode = 2;
    return NICNES_OK;
}

int nicnes_theta_zeros(nicnes_handle* h, int64_t* count_out_host, void* stream) {
    if (!h || !count_out_host) return NICNES_ERR_INVALID;
    if (!h->theta_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_theta first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    if (!h->zcount) {
        HIPC(h, hipDeviceSynchronize());
        int rc = dalloc(h, &h->zcount, 1);
        if (rc) return rc;
    }
    unsigned long long* d = h->zcount;
    HIPC(h, nicnes_launch_count_zeros(h->theta32, h->D, d, s));
    unsigned long long c = 0;
    HIPC(h, hipMemcpyAsync(&c, d, sizeof c, hipMemcpyDeviceToHost, s));
    HIPC(h, hipStreamSynchronize(s));
    *count_out_host = (int64_t)c;
    return NICNES_OK;
}

int nicnes_set_rows_per_image(nicnes_handle* h, int32_t n) {
    if (!h || n < 1 || n > 64) return NICNES_ERR_INVALID;
    h->rpi = n;
    return NICNES_OK;
}

int nicnes_set_sample_draws(nicnes_handle* h, const double* u_host, int64_t n) {
    if (!h || n < 0 || (n > 0 && !u_host)) return NICNES_ERR_INVALID;
    h->su_host.assign(u_host, u_host + n);
    return NICNES_OK;
}

int nicnes_set_fitness_mode(nicnes_handle* h, int32_t mode) {
    if (!h) return NICNES_ERR_INVALID;
    if (mode < NICNES_FITNESS_GREEDY || mode > NICNES_FITNESS_SC_LOSS)
        return fail(h, NICNES_ERR_UNSUPPORTED, "fitness mode: the engine implements greedy, greedy_{log,exp,lin,avg}prob, "
                                               "sample, self_critical and sc_loss");
    h->fitness_mode = mode;
    return NICNES_OK;
}

// [D] zeros + one zero slice index: theta itself as a "member" (the sigma = 0 decodes)
static int ensure_zero_noise(nicnes_handle* h) {
    if (h->zero_noise) return NICNES_OK;
    HIPC(h, hipDeviceSynchronize());
    int rc = dalloc(h, &h->zero_noise, (size_t)h->D);
    if (!rc) rc = dalloc(h, &h->zero_idx, 1);
    if (rc) return rc;
    HIPC(h, hipMemset(h->zero_noise, 0, (size_t)h->D * sizeof(float)));
    HIPC(h, hipMemset(h->zero_idx, 0, sizeof(uint64_t)));
    return NICNES_OK;
}

int nicnes_evaluate(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                    double* fitness_out, int32_t* seq_out, void* stream) {
    return nicnes_evaluate_lp(h, iteration, member_begin, count, sigma, fitness_out, seq_out, nullptr, stream);
}

int nicnes_evaluate_lp(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                       double* fitness_out, int32_t* seq_out, float* logprob_out, void* stream) {
    return nicnes_evaluate_batches(h, iteration, member_begin, count, sigma, nullptr, fitness_out, seq_out, logprob_out,
                                   stream);
}

// eval_theta: the sigma = 0 rollout of theta itself (count 1), decoded ONCE: sign + takes the first half of the
// batch's images and sign - the second (at sigma = 0 both signs are theta, so the halves are one decode of the
// batch), scored as one rollout of B rows
// scores_out (nullable, [n_cand, B]): every rollout row's CIDEr-D (the self-critical modes' greedy baseline)
static int evaluate_impl(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                         const int32_t* member_batch_host, double* fitness_out, int32_t* seq_out, float* logprob_out,
                         void* stream, bool eval_theta, double* scores_out = nullptr) {
    if (!h || !fitness_out || member_begin < 0) return NICNES_ERR_INVALID;
    const int mode = h->fitness_mode;
    const bool sampled = mode >= NICNES_FITNESS_SAMPLE;
    const bool self_critical = mode == NICNES_FITNESS_SELF_CRITICAL || mode == NICNES_FITNESS_SC_LOSS;
    if (self_critical && !scores_out) {
        // the greedy decode of the same rollouts first (compute_ciders, policies.py:174-180): its row scores
        // are the baseline the sampled rows' scores are reduced by
        const int64_t need = (int64_t)2 * h->cfg.max_members * h->cfg.max_batch;
        if (need > h->base_cap) {
            HIPC(h, hipDeviceSynchronize());
            if (h->base_scores) HIPC(h, hipFree(h->base_scores));
            h->base_scores = nullptr;
            h->base_cap = 0;
            int rc = dalloc(h, &h->base_scores, (size_t)need);
            if (rc) return rc;
            h->base_cap = need;
        }
        h->fitness_mode = NICNES_FITNESS_GREEDY;
        const int rc = evaluate_impl(h, iteration, member_begin, count, sigma, member_batch_host, fitness_out, nullptr,
                                     nullptr, stream, eval_theta, h->base_scores);
        h->fitness_mode = mode;
        if (rc) return rc;
    }
    if (count < 1 || count > h->cfg.max_members) return fail(h, NICNES_ERR_INVALID, "count out of [1, max_members]");
    if (!h->noise) return fail(h, NICNES_ERR_INVALID, "nicnes_set_noise_table first");
    if (!h->theta_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_theta first");
    if (!h->batch_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_batch first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    // rollout rows: the images, or rpi copies of each in the sampled modes (the reference's seq_per_img rows);
    // the row buffers grow before anything below takes their addresses
    const int rpi = sampled ? h->rpi : 1;
    const int rows_total = h->B * rpi;
    if (rows_total > h->cfg.max_batch) {
        HIPC(h, hipDeviceSynchronize());
        int rc = alloc_batch(h, rows_total);
        if (rc) return rc;
    }
    const int32_t* mb = nullptr;
    if (member_batch_host) {
        for (int k = 0; k < count; ++k)
            if (member_batch_host[k] < 0 || member_batch_host[k] >= h->n_batches)
                return fail(h, NICNES_ERR_INVALID, "member_batch entry outside [0, n_batches)");
        // the caller's array may go away on return: copied to a pinned ring slot whose previous copy has run
        const int slot = h->mb_next;
        h->mb_next = (slot + 1) % MB_RING;
        if (h->mb_used[slot]) HIPC(h, hipEventSynchronize(h->mb_ev[slot]));
        std::memcpy(h->mb_pin[slot], member_batch_host, (size_t)count * sizeof(int32_t));
        HIPC(h, hipMemcpyAsync(h->mbatch, h->mb_pin[slot], (size_t)count * sizeof(int32_t), hipMemcpyHostToDevice, s));
        HIPC(h, hipEventRecord(h->mb_ev[slot], s));
        h->mb_used[slot] = true;
        mb = h->mbatch;
    } else if (h->n_batches != 1) {
        return fail(h, NICNES_ERR_INVALID, "several batches are held: pass member_batch (nicnes_evaluate_batches)");
    }
    DecodeParams p;
    p.theta = h->theta32;
    p.noise = h->noise;
    p.noise_idx = h->nidx;
    if (eval_theta) {       // theta itself: a zero slice (the sigma-scaled table is left as it is)
        int rc = ensure_zero_noise(h);
        if (rc) return rc;
        p.noise = h->zero_noise;
        p.noise_idx = h->zero_idx;
    } else {
        HIPC(h, nicnes_launch_noise_index(h->cfg.noise_seed, iteration, (uint64_t)member_begin, count, h->cfg.noise_len,
                                          (uint64_t)h->D, h->nidx, s));
    }
    if (eval_theta) {
    } else if (h->mut_mode && !h->dbuf) {   // first mutated evaluation: [max_members, Dp] delta' rows
        HIPC(h, hipDeviceSynchronize());
        h->Dp = (h->D + 63) / 64 * 64;
        int rc = dalloc(h, &h->dbuf, (size_t)h->cfg.max_members * (size_t)h->Dp);
        if (!rc) rc = dalloc(h, &h->didx, (size_t)h->cfg.max_members);
        if (rc) return rc;
        HIPC(h, nicnes_launch_iota_stride(h->didx, h->cfg.max_members, (uint64_t)h->Dp, s));
    }
    if (!eval_theta) {      // fp32(sigma * z), the table scaled once per sigma: the plain decode's noise, and the
        if (!h->noise_sc) { // sigma z a mutated fused decode forms the head parameters' delta' from (below)
            HIPC(h, hipDeviceSynchronize());
            int rc = dalloc(h, &h->noise_sc, (size_t)h->cfg.noise_len);
            if (rc) return rc;
        }
        if (!h->sc_valid || __builtin_bit_cast(uint32_t, h->sc_sigma) != __builtin_bit_cast(uint32_t, sigma)) {
            HIPC(h, nicnes_launch_scale(h->noise, h->noise_sc, h->cfg.noise_len, sigma, s));
            h->sc_sigma = sigma;
            h->sc_valid = true;
        }
    }
    if (eval_theta) {
    } else if (h->mut_mode) {      // safe / proportional mutations: the decode reads the members' delta' rows
        p.noise = h->dbuf;         // (materialised below, once the decode path is known)
        p.noise_idx = h->didx;
    } else {
        p.noise = h->noise_sc;
    }
    MutHead mh{nullptr, nullptr, nullptr, 0};
    p.fc = h->fc;
    p.member_batch = mb;
    p.seq = seq_out ? seq_out : h->seq;
    const bool crit_lp = (mode >= NICNES_FITNESS_GREEDY_LOGPROB && mode <= NICNES_FITNESS_GREEDY_AVGPROB) ||
                         mode == NICNES_FITNESS_SC_LOSS;                // the criterion needs seq_logprobs
    p.lp = logprob_out ? logprob_out : (crit_lp ? h->lp : nullptr);
    p.sample_u = nullptr;
    p.slog = nullptr;
    p.slog_slots = nullptr;
    p.slog_ns = 0;
    p.scratch = h->dscratch;
    p.stats = h->stats;
    p.alive = h->alive;
    p.force_exact = h->force_exact;
    p.lse_margin = h->lse_margin;
    if (h->stats_pending && hipEventQuery(h->stats_ev) == hipSuccess) {   // the last decode's fallbacks
        const int32_t fb = h->stats_host[0];
        if (h->stats_host[2] != 0)
            return fail(h, NICNES_ERR_FAULT, "coop decode: a workgroup's partners never arrived (hand-off timeout)");
        if (h->stats_host[3] != 0)
            return fail(h, NICNES_ERR_FAULT, "sampled decode: a workgroup found no free logit slot");
        if (h->last_bounded && fb - h->fb_seen >= 2) h->exact_left = 32;
        h->fb_seen = fb;
        h->stats_pending = false;
    }
    bool bounded = h->bounded_mode == 1 || (h->bounded_mode == 2 && h->exact_left == 0);
    if (h->bounded_mode == 2 && h->exact_left > 0 && !p.lp) --h->exact_left;
    p.bounded_lse = bounded ? 1 : 0;
    h->last_decode_bounded = (bounded && !p.lp) ? 1 : 0;
    // rows per sign: all of the rollout's rows, or the first half (eval_theta; sign - takes rows half + b)
    const int rows = eval_theta ? (rows_total + 1) / 2 : rows_total;
    int G = 0, nslabs = 0, S = 0;
    decode_shape(h, rows, count, &G, &nslabs, &S);
    if (sampled) {          // the sampled pick runs on the fused path (128-row slabs, one workgroup per slab)
        G = 4;
        S = 1;
        nslabs = nslabs_of(rows, 4);
        const int64_t need = (int64_t)count * 2 * rows * h->cfg.seq_length;
        if (need > h->su_cap) {
            HIPC(h, hipDeviceSynchronize());
            if (h->su) HIPC(h, hipFree(h->su));
            h->su = nullptr;
            h->su_cap = 0;
            int rc = dalloc(h, &h->su, (size_t)need);
            if (rc) return rc;
            h->su_cap = need;
        }
        if (!h->su_host.empty()) {
            if ((int64_t)h->su_host.size() != need)
                return fail(h, NICNES_ERR_INVALID, "nicnes_set_sample_draws: count x 2 x B x seq_length draws needed");
            HIPC(h, hipMemcpyAsync(h->su, h->su_host.data(), (size_t)need * sizeof(double), hipMemcpyHostToDevice, s));
        } else {
            // eval rollouts (eval_theta) draw from a member index no population reaches
            HIPC(h, nicnes_launch_sample_draws(h->cfg.noise_seed, iteration,
                                               eval_theta ? (uint64_t)0xffffffffu : (uint64_t)member_begin, count, rows,
                                               h->cfg.seq_length, h->su, s));
        }
        p.sample_u = h->su;
        if (!h->slog) {
            // a slot per resident workgroup (one per CU: the steps kernel's LDS) plus spares, each holding one
            // step's logits and stage sums of a workgroup's 2 x 128 rows (nst stages of 72 KiB)
            const int ns = h->test_slots > 0 ? h->test_slots : h->sample_occ * h->n_cu + 16;
            // 72 KiB per stage + 8 KiB per block of 8 stages (decode_kernel.hip, SLOG_*)
            const int nst = (h->V1 + 63) / 64;
            const size_t per = (size_t)nst * 18432 + (size_t)((nst + 7) / 8) * 2048;
            HIPC(h, hipDeviceSynchronize());
            int rc = dalloc(h, &h->slog, per * ns);
            if (!rc) rc = dalloc(h, &h->slog_slots, (size_t)ns);
            if (rc) return rc;
            HIPC(h, hipMemset(h->slog_slots, 0, ns * sizeof(int32_t)));
            h->slog_ns = ns;
        }
        p.slog = h->slog;
        p.slog_slots = h->slog_slots;
        p.slog_ns = h->slog_ns;
    }
    if ((int64_t)count * nslabs * S > h->part_cap)
        return fail(h, NICNES_ERR_INVALID, "decode split beyond the partial-state buffer (nicnes_set_decode_split)");
    p.G = G;
    p.S = S;
    p.part = h->part;
    p.coop = !sampled && coop_fits(h, G, nslabs, S, count) ? 1 : 0;
    p.coop_launch = h->coop_launch;
    if (!eval_theta && h->mut_mode) {
        // the members' delta' rows. On the fused greedy path only the parameters from off_log_w on (logit, i2h, h2h,
        // which every step re-reads) are materialised; the decode forms the image projection's and the embedding
        // rows' delta' itself from sigma z and the vector (DecodeParams::mut_head): 5.6 of the 11.5 MB per member
        const bool head = !sampled && !p.coop && G == 4 && S == 1 && !h->mut_full;
        const int64_t j0 = head ? h->off[3] : 0;
        HIPC(h, nicnes_launch_mutate(h->noise + j0, h->nidx, count, h->D - j0, sigma, h->mut_vec + j0, h->mut_mode,
                                     h->dbuf + j0, h->Dp, s));
        if (head) mh = MutHead{h->noise_sc, h->nidx, h->mut_vec, h->mut_mode};
    }
    p.test_stall_ms = h->test_stall_left != 0 ? h->test_stall_ms : 0;
    if (p.coop && h->test_stall_ms && h->test_stall_left > 0) --h->test_stall_left;
    // log-probs of a batch spread over several slabs: every slab runs to T, then the steps after the
    // batch's last finishing step are zeroed (nicnes_lp_batch_exit), as FCModel._sample leaves them
    p.no_exit = (p.lp && nslabs > 1) ? 1 : 0;
    p.no_mask = 0;
    p.coop_ctr = h->coop_ctr;
    p.alive2 = h->alive + h->alive_stride;
    p.alive_stride = h->alive_stride;
    p.B = rows;
    p.B_img = h->B;
    p.rpi = rpi;
    p.sign_off = eval_theta ? rows : 0;
    p.F = h->cfg.fc_feat_size;
    p.V1 = h->V1;
    p.T = h->cfg.seq_length;
    p.D = h->D;
    p.off_img_w = h->off[0];
    p.off_img_b = h->off[1];
    p.off_emb_w = h->off[2];
    p.off_log_w = h->off[3];
    p.off_log_b = h->off[4];
    p.off_i2h_w = h->off[5];
    p.off_i2h_b = h->off[6];
    p.off_h2h_w = h->off[7];
    p.off_h2h_b = h->off[8];
    // rows a member never writes (all finished early) must read as 0 (nets.py:188 zeros). eval_theta's output is
    // the one rollout of rows_total rows (with an odd count sign - has one row fewer than sign +)
    const size_t out_rows = eval_theta ? (size_t)rows_total : (size_t)count * 2 * rows;
    HIPC(h, hipMemsetAsync(p.seq, 0, out_rows * h->cfg.seq_length * sizeof(int32_t), s));
    if (p.lp) HIPC(h, hipMemsetAsync(p.lp, 0, out_rows * h->cfg.seq_length * sizeof(float), s));
    if (h->timing) HIPC(h, hipEventRecord(h->ev[0], s));
    int n_ev = 0;
    // the coop launch needs all its workgroups resident: never split over streams
    const int nstr = p.coop ? 1 : std::min(count, h->dec_streams ? h->dec_streams : (S == 1 ? 1 : 2));
    if (nstr > 1) {
        // members split evenly over the caller's stream and nstr - 1 engine streams; the parts share
        // nothing but the fallback counter (an atomic). No per-launch events: the launches overlap
        if (!h->ev_fork) HIPC(h, hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
        for (int i = 0; i < nstr - 1; ++i)
            if (!h->sx[i]) {
                HIPC(h, hipStreamCreateWithFlags(&h->sx[i], hipStreamNonBlocking));
                HIPC(h, hipEventCreateWithFlags(&h->ev_join[i], hipEventDisableTiming));
            }
        HIPC(h, hipEventRecord(h->ev_fork, s));
        for (int i = 0; i < nstr; ++i) {
            const int a = (int)((int64_t)count * i / nstr), b = (int)((int64_t)count * (i + 1) / nstr);
            DecodeParams pi = p;
            MutHead mi = mh;
            nicnes_decode_shift(&pi, a, nslabs, &mi);
            hipStream_t si = i == 0 ? s : h->sx[i - 1];
            if (i > 0) HIPC(h, hipStreamWaitEvent(si, h->ev_fork, 0));
            HIPC(h, nicnes_launch_decode(&pi, &mi, b - a, nslabs, si, nullptr, nullptr, nullptr));
        }
        for (int i = 0; i < nstr - 1; ++i) {
            HIPC(h, hipEventRecord(h->ev_join[i], h->sx[i]));
            HIPC(h, hipStreamWaitEvent(s, h->ev_join[i], 0));
        }
    } else {
        HIPC(h, nicnes_launch_decode(&p, &mh, count, nslabs, s, h->timing ? h->dev : nullptr, h->dev_kind, &n_ev));
    }
    h->n_dev = h->timing ? n_ev : 0;
    h->multi_stream = nstr > 1;
    if (p.no_exit)      // eval_theta: the two halves are one rollout
        HIPC(h, nicnes_launch_lp_batch_exit(p.seq, p.lp, eval_theta ? 1 : 2 * count, rows_total, h->cfg.seq_length, s));
    if (h->timing) HIPC(h, hipEventRecord(h->ev[1], s));
    if (!h->stats_pending) {          // read the fallback counter back without a host wait
        HIPC(h, hipMemcpyAsync(h->stats_host, h->stats, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        HIPC(h, hipEventRecord(h->stats_ev, s));
        h->stats_pending = true;
        h->last_bounded = bounded && !p.lp;
    }
    CiderTables tb = tables_of(h);
    const int n_cand = eval_theta ? 1 : 2 * count;      // eval_theta: rows s * half + b = image s * half + b
    const double* base = self_critical ? h->base_scores : nullptr;
    if (h->img_tables) {
        HIPC(h, nicnes_launch_cider_img(p.seq, n_cand, rows_total, h->cfg.seq_length, &tb, h->img_ref_start, mb, p.lp,
                                         h->fitness_mode, h->row_scores, fitness_out, s, base, rpi));
        if (scores_out)
            HIPC(h, hipMemcpyAsync(scores_out, h->row_scores, (size_t)n_cand * rows_total * sizeof(double),
                                   hipMemcpyDeviceToDevice, s));
    } else {
        HIPC(h, nicnes_launch_cider(p.seq, n_cand, rows_total, h->cfg.seq_length, &tb, h->img_ref_start, mb, p.lp,
                                    h->fitness_mode, fitness_out, s, base, scores_out, rpi));
    }
    if (h->timing) HIPC(h, hipEventRecord(h->ev[2], s));
    return NICNES_OK;
}

int nicnes_evaluate_batches(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, float sigma,
                            const int32_t* member_batch_host, double* fitness_out, int32_t* seq_out, float* logprob_out,
                            void* stream) {
    return evaluate_impl(h, iteration, member_begin, count, sigma, member_batch_host, fitness_out, seq_out, logprob_out,
                         stream, false);
}

int nicnes_evaluate_theta(nicnes_handle* h, int32_t batch, uint64_t iteration, double* fitness_out, int32_t* seq_out,
                          float* logprob_out, void* stream) {
    if (!h) return NICNES_ERR_INVALID;
    if (batch < 0 || (h->batch_set && batch >= h->n_batches)) return fail(h, NICNES_ERR_INVALID, "batch outside [0, n_batches)");
    const int32_t mb = batch;
    return evaluate_impl(h, iteration, 0, 1, 0.f, h->n_batches > 1 ? &mb : nullptr, fitness_out, seq_out, logprob_out,
                         stream, true);
}

int nicnes_sum_sensitivity(nicnes_handle* h, int32_t rows, float underflow, float* out, void* stream) {
    if (!h || !out || rows < 1) return NICNES_ERR_INVALID;
    if (!h->theta_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_theta first");
    if (!h->batch_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_batch first");
    if (rows > h->B) return fail(h, NICNES_ERR_INVALID, "rows beyond the batch held");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    const int L = 5, split = 100;                                  // forward_for_sensitivity defaults (nets.py:22)
    if (!h->sens_tok) {
        HIPC(h, hipDeviceSynchronize());
        int rc = dalloc(h, &h->sens_tok, (size_t)2 * h->cfg.max_batch * (L - 1));
        if (rc) return rc;
        h->sens = nicnes_sens_create();
    }
    SensParams sp;
    sp.theta = h->theta32;
    sp.fc = h->fc;
    sp.tok = h->sens_tok;                                          // [rows, L - 1], written by the forward
    sp.tok_stride = L - 1;
    sp.tok_internal = 1;
    sp.Bs = rows;
    sp.V1 = h->V1;
    sp.E = h->cfg.input_encoding_size;
    sp.R = h->cfg.rnn_size;
    sp.F = h->cfg.fc_feat_size;
    sp.L = L;
    sp.split = split;
    sp.K = h->V1 / split + 1;
    sp.D = h->D;
    sp.off_img_w = h->off[0]; sp.off_img_b = h->off[1]; sp.off_emb_w = h->off[2]; sp.off_log_w = h->off[3];
    sp.off_log_b = h->off[4]; sp.off_i2h_w = h->off[5]; sp.off_i2h_b = h->off[6]; sp.off_h2h_w = h->off[7];
    sp.off_h2h_b = h->off[8];
    sp.underflow = underflow;
    sp.out = out;
    const int rc = nicnes_sens_run(h->sens, &sp, s);
    if (rc) return fail(h, NICNES_ERR_HIP, "sensitivity kernels failed (code " + std::to_string(rc) + ")");
    return NICNES_OK;
}

int nicnes_rank_weights(nicnes_handle* h, const double* fitness, int32_t P, double* cr_out, float* w_out, void* stream) {
    if (!h || !fitness || !w_out || P < 1) return NICNES_ERR_INVALID;
    if (P > (1 << 29)) return fail(h, NICNES_ERR_UNSUPPORTED, "P > 2^29");
    HIPC(h, hipSetDevice(h->device));
    const size_t need = nicnes_rank_scratch_pairs(2 * P);
    if (need > h->rank_cap) {       // the first call at a larger population grows the sort scratch
        HIPC(h, hipStreamSynchronize((hipStream_t)stream));
        if (h->rank_key) (void)hipFree(h->rank_key);
        if (h->rank_idx) (void)hipFree(h->rank_idx);
        h->rank_key = nullptr;
        h->rank_idx = nullptr;
        h->rank_cap = 0;
        int rc = dalloc(h, &h->rank_key, need);
        if (!rc) rc = dalloc(h, &h->rank_idx, need);
        if (rc) return rc;
        h->rank_cap = need;
    }
    HIPC(h, nicnes_launch_rank(fitness, 2 * P, h->rank_key, h->rank_idx, cr_out, w_out, (hipStream_t)stream));
    return NICNES_OK;
}

int nicnes_grad_partial(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, const float* w,
                        float sigma, float* gsum_out, void* stream) {
    if (!h || !w || !gsum_out || member_begin < 0 || count < 0) return NICNES_ERR_INVALID;
    if (count > h->cfg.max_members) return fail(h, NICNES_ERR_INVALID, "count > max_members");
    if (!h->noise) return fail(h, NICNES_ERR_INVALID, "nicnes_set_noise_table first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, nicnes_launch_noise_index(h->cfg.noise_seed, iteration, (uint64_t)member_begin, count, h->cfg.noise_len,
                                      (uint64_t)h->D, h->nidx, s));
    // with a mutation the reference sums the mutated noise vectors it was sent (nic_nes_worker.py:156-161):
    // the kernel transforms each delta on the fly
    HIPC(h, nicnes_launch_grad(h->noise, h->nidx, w, count, sigma, h->D, h->mut_vec, h->mut_mode, gsum_out, s,
                               h->stats));
    return NICNES_OK;
}

int nicnes_grad_partial_range(nicnes_handle* h, uint64_t iteration, int32_t member_begin, int32_t count, const float* w,
                              float sigma, int64_t j0, int64_t j1, float* gsum_out, void* stream) {
    if (!h || !w || !gsum_out || member_begin < 0 || count < 0) return NICNES_ERR_INVALID;
    if (j0 < 0 || j1 > h->D || j0 >= j1 || (j0 & 63)) return fail(h, NICNES_ERR_INVALID, "range: 0 <= j0 < j1 <= D, j0 % 64 == 0");
    if (count > h->cfg.max_members) return fail(h, NICNES_ERR_INVALID, "count > max_members");
    if (!h->noise) return fail(h, NICNES_ERR_INVALID, "nicnes_set_noise_table first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, nicnes_launch_noise_index(h->cfg.noise_seed, iteration, (uint64_t)member_begin, count, h->cfg.noise_len,
                                      (uint64_t)h->D, h->nidx, s));
    // the same kernel on the parameter range (slices are 64-float aligned, so j0 % 64 keeps the f32x4 loads aligned)
    HIPC(h, nicnes_launch_grad(h->noise + j0, h->nidx, w, count, sigma, j1 - j0, h->mut_vec ? h->mut_vec + j0 : nullptr,
                               h->mut_mode, gsum_out + j0, s, h->stats));
    return NICNES_OK;
}

// A skipped optimizer step (NaN ratio, nicnes_adam_kernel): say why. This handle's decode lost rows (its
// counters), or another rank's did (the all-reduced noise sum came back NaN).
static int fault_error(nicnes_handle* h, bool from_noise_sum = true) {
    int32_t st[4];
    HIPC(h, hipMemcpy(st, h->stats, sizeof st, hipMemcpyDeviceToHost));
    if (st[2] != 0) return fail(h, NICNES_ERR_FAULT, "coop decode: a workgroup's partners never arrived (hand-off timeout); "
                                                     "the iteration's fitness is NaN and the optimizer step was skipped");
    if (st[3] != 0) return fail(h, NICNES_ERR_FAULT, "sampled decode: a workgroup found no free logit slot; "
                                                     "the iteration's fitness is NaN and the optimizer step was skipped");
    if (!from_noise_sum) return NICNES_OK;      // Optimizer.update(globalg) with a NaN globalg: as the reference
    return fail(h, NICNES_ERR_FAULT, "optimizer step skipped: the noise sum is NaN (a faulted decode on another rank)");
}

// the newest step was skipped (its flag read back as set): undo its host-side state once
static void rollback_skipped_step(nicnes_handle* h) {
    if (!h->step_pending_check) return;
    h->t = h->t_prev;
    h->theta_is_fp32 = h->theta_fp32_prev;
    h->step_pending_check = false;
}

// one optimizer update (kind 0 Adam, 1 SGD), from the fused NES form (gsum, P, l2coeff) or from a
// given globalg (Optimizer.update(globalg), optimizers.py:15-22)
static int opt_step(nicnes_handle* h, int kind, const float* gsum, int32_t P, double l2coeff, const double* globalg,
                    int globalg_fp32, double stepsize, double b1, double b2, double epsilon, double* ratio_out_host, void* stream) {
    if (!h->theta_set) return fail(h, NICNES_ERR_INVALID, "nicnes_set_theta first");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    h->t_prev = h->t;
    h->theta_fp32_prev = h->theta_is_fp32;
    h->step_pending_check = true;
    h->t += 1;
    AdamParams p;
    p.theta64 = h->theta64;
    p.theta32 = h->theta32;
    p.m = h->m;
    p.v = h->v;
    p.gsum = gsum;
    p.globalg = globalg;
    p.partials = h->partials;
    p.dim = h->D;
    p.two_f = (float)(2 * (P > 0 ? P : 1));
    p.theta_is_fp32 = h->theta_is_fp32;
    p.l2coeff = l2coeff;
    p.l2coeff32 = (float)l2coeff;
    p.kind = kind;
    // fused form: g' is fp32 exactly while theta is (nic_nes_master.py:126-133)
    p.g_is_fp32 = globalg ? (globalg_fp32 != 0) : h->theta_is_fp32;
    // Adam: a = stepsize * sqrt(1 - b2^t) / (1 - b1^t)   (optimizers.py:79, Python float arithmetic)
    p.a = kind == 0 ? stepsize * std::sqrt(1.0 - std::pow(b2, (double)h->t)) / (1.0 - std::pow(b1, (double)h->t)) : 0.0;
    p.neg_stepsize = -stepsize;
    p.beta1 = b1;                      // SGD: momentum
    p.beta2 = b2;
    p.one_minus_beta1 = 1.0 - b1;
    p.one_minus_beta2 = 1.0 - b2;
    p.one_minus_beta1_32 = (float)(1.0 - b1);
    p.one_minus_beta2_32 = (float)(1.0 - b2);
    p.epsilon = epsilon;
    p.fault = h->stats;
    p.skip_out = h->norms + 2;
    h->last_nes_form = globalg == nullptr;
    HIPC(h, nicnes_launch_adam(&p, h->norms, s));
    h->theta_is_fp32 = 0;
    if (ratio_out_host) {
        double n3[3];
        HIPC(h, hipMemcpyAsync(n3, h->norms, sizeof n3, hipMemcpyDeviceToHost, s));
        HIPC(h, hipStreamSynchronize(s));
        *ratio_out_host = std::sqrt(n3[0]) / std::sqrt(n3[1]);
        if (n3[2] != 0.0) {
            rollback_skipped_step(h);
            return fault_error(h, globalg == nullptr);
        }
        h->step_pending_check = false;
    }
    return NICNES_OK;
}

int nicnes_last_ratio(nicnes_handle* h, double* ratio_out_host, void* stream) {
    if (!h || !ratio_out_host) return NICNES_ERR_INVALID;
    if (h->t == 0) return fail(h, NICNES_ERR_INVALID, "no optimizer step yet");
    hipStream_t s = (hipStream_t)stream;
    HIPC(h, hipSetDevice(h->device));
    double n3[3];
    HIPC(h, hipMemcpyAsync(n3, h->norms, sizeof n3, hipMemcpyDeviceToHost, s));
    HIPC(h, hipStreamSynchronize(s));
    *ratio_out_host = std::sqrt(n3[0]) / std::sqrt(n3[1]);
    if (n3[2] != 0.0) {
        rollback_skipped_step(h);
        return fault_error(h, h->last_nes_form);
    }
    h->step_pending_check = false;
    return NICNES_OK;
}

int nicnes_clear_faults(nicnes_handle* h, int64_t* counters_out_host) {
    if (!h) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, hipDeviceSynchronize());            // every launch that could still count has finished
    int32_t st[4];
    HIPC(h, hipMemcpy(st, h->stats, sizeof st, hipMemcpyDeviceToHost));
    if (h->step_pending_check) {                 // the newest step's skip flag was not read yet
        double skip = 0.0;
        HIPC(h, hipMemcpy(&skip, h->norms + 2, sizeof skip, hipMemcpyDeviceToHost));
        if (skip != 0.0) rollback_skipped_step(h);
        else h->step_pending_check = false;
    }
    if (counters_out_host) {
        counters_out_host[0] = st[2];
        counters_out_host[1] = st[3];
    }
    // zero the fault words only (the fallback counters [0], [1] keep counting) and the logit-slot claim flags
    // (the coop hand-off counters are zeroed before every coop launch), then forget the pending read-back
    // that carried the fault
    HIPC(h, hipMemset(h->stats + 2, 0, 2 * sizeof(int32_t)));
    if (h->slog_slots) HIPC(h, hipMemset(h->slog_slots, 0, (size_t)h->slog_ns * sizeof(int32_t)));
    HIPC(h, hipDeviceSynchronize());
    h->stats_pending = false;
    return NICNES_OK;
}

int nicnes_adam_step(nicnes_handle* h, const float* gsum, int32_t P, double l2coeff, double stepsize, double beta1,
                     double beta2, double epsilon, double* ratio_out_host, void* stream) {
    if (!h || !gsum || P < 1) return NICNES_ERR_INVALID;
    return opt_step(h, 0, gsum, P, l2coeff, nullptr, 0, stepsize, beta1, beta2, epsilon, ratio_out_host, stream);
}

int nicnes_sgd_step(nicnes_handle* h, const float* gsum, int32_t P, double l2coeff, double stepsize, double momentum,
                    double* ratio_out_host, void* stream) {
    if (!h || !gsum || P < 1) return NICNES_ERR_INVALID;
    return opt_step(h, 1, gsum, P, l2coeff, nullptr, 0, stepsize, momentum, 0.0, 0.0, ratio_out_host, stream);
}

int nicnes_optimizer_update(nicnes_handle* h, int kind, const double* globalg, int globalg_fp32, double stepsize,
                            double beta1, double beta2, double epsilon, double* ratio_out_host, void* stream) {
    if (!h || !globalg || (kind != 0 && kind != 1)) return NICNES_ERR_INVALID;
    return opt_step(h, kind, nullptr, 0, 0.0, globalg, globalg_fp32, stepsize, beta1, beta2, epsilon, ratio_out_host, stream);
}

int nicnes_stats(nicnes_handle* h, int64_t* out4_host) {
    if (!h || !out4_host) return NICNES_ERR_INVALID;
    int32_t st[4];
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, hipMemcpy(st, h->stats, sizeof st, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out4_host[i] = st[i];
    return NICNES_OK;
}

int nicnes_set_timing(nicnes_handle* h, int on) {
    if (!h) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    if (on && !h->ev[0])
    {
        for (auto& e : h->ev) HIPC(h, hipEventCreate(&e));
        for (auto& e : h->dev) HIPC(h, hipEventCreate(&e));
    }
    h->timing = on != 0;
    return NICNES_OK;
}

int nicnes_kernel_times(nicnes_handle* h, float* out2_host) {
    if (!h || !out2_host || !h->ev[0]) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, hipEventSynchronize(h->ev[2]));
    HIPC(h, hipEventElapsedTime(&out2_host[0], h->ev[0], h->ev[1]));
    HIPC(h, hipEventElapsedTime(&out2_host[1], h->ev[1], h->ev[2]));
    return NICNES_OK;
}

int nicnes_decode_phase_times(nicnes_handle* h, float* out8_host) {
    if (!h || !out8_host) return NICNES_ERR_INVALID;
    if (h->timing && h->n_dev == 0 && h->multi_stream) {      // multi-stream decode: no per-launch events
        for (int i = 0; i < 8; ++i) out8_host[i] = 0.f;
        return NICNES_OK;
    }
    if (h->n_dev < 2) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    HIPC(h, hipEventSynchronize(h->dev[h->n_dev - 1]));
    // event k follows launch k. Fused: img, then steps (one launch), or step(t) for t = -1..T (the first
    // two launches run only a cell). Split: img, cell(-1), cell(0), then logit(t), cell(t) for t = 1..T.
    float o[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ms = 0.f;
    int n_cell_only = 0;
    for (int k = 1; k < h->n_dev; ++k) {
        HIPC(h, hipEventElapsedTime(&ms, h->dev[k - 1], h->dev[k]));
        switch (h->dev_kind[k]) {
            case DK_IMG: o[0] += ms; break;
            case DK_STEP:
                o[2] += ms; o[3] += 1;
                if (n_cell_only < 2) { o[1] += ms; ++n_cell_only; }
                break;
            case DK_STEPS: o[2] += ms; o[3] += 1; break;      // every step in one launch
            case DK_COOP: o[2] += ms; o[3] += 1; break;       // the split shape, every step in one launch
            case DK_STEPS2: o[2] += ms; o[3] += 1; break;     // 64-row slabs, every step in one launch
            case DK_LOGIT: o[4] += ms; o[5] += 1; break;
            default:
                o[6] += ms; o[7] += 1;
                if (n_cell_only < 2) { o[1] += ms; ++n_cell_only; }
                break;
        }
    }
    for (int i = 0; i < 8; ++i) out8_host[i] = o[i];
    return NICNES_OK;
}

int nicnes_set_decode_streams(nicnes_handle* h, int32_t n) {
    if (!h || n < 0 || n > 4) return NICNES_ERR_INVALID;
    h->dec_streams = n;
    return NICNES_OK;
}

int nicnes_set_decode_coop(nicnes_handle* h, int32_t mode) {
    if (!h || (mode != 0 && mode != 1)) return NICNES_ERR_INVALID;
    h->coop_mode = mode;
    return NICNES_OK;
}

int nicnes_last_decode_lse(nicnes_handle* h, int32_t* bounded_host) {
    if (!h || !bounded_host) return NICNES_ERR_INVALID;
    *bounded_host = h->last_decode_bounded;
    return NICNES_OK;
}

int nicnes_decode_path(nicnes_handle* h, int32_t B, int32_t count, int32_t* out_host) {
    if (!h || !out_host || B < 1 || count < 1) return NICNES_ERR_INVALID;
    int G = 0, nslabs = 0, S = 0;
    decode_shape(h, B, count, &G, &nslabs, &S);
    *out_host = S == 1 ? 0 : coop_fits(h, G, nslabs, S, count) ? 2 : 1;
    return NICNES_OK;
}

int nicnes_set_decode_split(nicnes_handle* h, int32_t S, int32_t G) {
    if (!h || S < 0 || S > 64 || (G != 0 && G != 2 && G != 4)) return NICNES_ERR_INVALID;
    HIPC(h, hipSetDevice(h->device));
    if (S > 0) {
        const int ns = std::max(nslabs_of(h->cfg.max_batch, 2), nslabs_of(h->cfg.max_batch, 4));
        const int64_t need = (int64_t)h->cfg.max_members * ns * S;
        if (need > h->part_cap) {
            float* np = nullptr;
            int rc = dalloc(h, &np, (size_t)need * PART_FLOATS);
            if (rc) return rc;
            HIPC(h, hipDeviceSynchronize());
            (void)hipFree(h->part);
            h->part = np;
            h->part_cap = need;
        }
    }
    h->dec_S = S;
    h->dec_G = G;
    return NICNES_OK;
}

// ---- multi-GPU exchange over RCCL (the data plane of SURVEY.md 8(e)) ---------------------------
#define NCCLC(h, expr)                                                                          \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess)                                                                  \
            return fail((h), NICNES_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

int nicnes_comm_unique_id(uint8_t* id_out_host) {
    if (!id_out_host) return NICNES_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == NICNES_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return NICNES_ERR_HIP;
    std::memcpy(id_out_host, &id, sizeof id);
    return NICNES_OK;
}

int nicnes_comm_init(nicnes_handle* h, int32_t nranks, int32_t rank, const uint8_t* id_host) {
    if (!h || !id_host || nranks < 1 || rank < 0 || rank >= nranks) return NICNES_ERR_INVALID;
    if (h->comm) return fail(h, NICNES_ERR_INVALID, "a communicator is already bound (nicnes_comm_destroy first)");
    HIPC(h, hipSetDevice(h->device));
    ncclUniqueId id;
    std::memcpy(&id, id_host, sizeof id);
    ncclComm_t c = nullptr;
    NCCLC(h, ncclCommInitRank(&c, nranks, id, rank));
    h->comm = c;
    h->comm_owned = true;
    h->comm_nranks = nranks;
    return NICNES_OK;
}

int nicnes_comm_attach(nicnes_handle* h, void* nccl_comm) {
    if (!h || !nccl_comm) return NICNES_ERR_INVALID;
    if (h->comm) return fail(h, NICNES_ERR_INVALID, "a communicator is already bound (nicnes_comm_destroy first)");
    int n = 0;
    NCCLC(h, ncclCommCount((ncclComm_t)nccl_comm, &n));
    h->comm = (ncclComm_t)nccl_comm;
    h->comm_owned = false;
    h->comm_nranks = n;
    return NICNES_OK;
}

int nicnes_comm_destroy(nicnes_handle* h) {
    if (!h) return NICNES_ERR_INVALID;
    if (h->comm && h->comm_owned) NCCLC(h, ncclCommDestroy(h->comm));
    h->comm = nullptr;
    h->comm_owned = false;
    h->comm_nranks = 1;
    return NICNES_OK;
}

int nicnes_comm_count(nicnes_handle* h, int32_t* nranks_out_host, int32_t* rank_out_host) {
    if (!h || !nranks_out_host || !rank_out_host) return NICNES_ERR_INVALID;
    int n = 1, r = 0;
    if (h->comm) {
        NCCLC(h, ncclCommCount(h->comm, &n));
        NCCLC(h, ncclCommUserRank(h->comm, &r));
    }
    *nranks_out_host = n;
    *rank_out_host = r;
    return NICNES_OK;
}

int nicnes_allgather_fitness(nicnes_handle* h, const double* fit_local, int32_t P_local, double* fit_all, void* stream) {
    if (!h || !fit_local || !fit_all || P_local < 1) return NICNES_ERR_INVALID;
    if (!h->comm) return fail(h, NICNES_ERR_INVALID, "no communicator (nicnes_comm_init / nicnes_comm_attach)");
    HIPC(h, hipSetDevice(h->device));
    NCCLC(h, ncclAllGather(fit_local, fit_all, (size_t)P_local * 2, ncclDouble, h->comm, (hipStream_t)stream));
    return NICNES_OK;
}

int nicnes_allreduce_grad(nicnes_handle* h, float* gsum, void* stream) {
    if (!h || !gsum) return NICNES_ERR_INVALID;
    if (!h->comm) return fail(h, NICNES_ERR_INVALID, "no communicator (nicnes_comm_init / nicnes_comm_attach)");
    HIPC(h, hipSetDevice(h->device));
    NCCLC(h, ncclAllReduce(gsum, gsum, (size_t)h->D, ncclFloat, ncclSum, h->comm, (hipStream_t)stream));
    return NICNES_OK;
}

int nicnes_decode_shape(nicnes_handle* h, int32_t B, int32_t count, int32_t* out3_host) {
    if (!h || !out3_host || B < 1 || count < 1) return NICNES_ERR_INVALID;
    int G, ns, S;
    decode_shape(h, B, count, &G, &ns, &S);
    out3_host[0] = G;
    out3_host[1] = ns;
    out3_host[2] = S;
    return NICNES_OK;
}

}  // extern "C"
