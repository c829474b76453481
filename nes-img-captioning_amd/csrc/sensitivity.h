// Internal (non-ABI) interface of the SM-G-SUM sensitivity (sensitivity.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct SensParams {
    const float* theta;          // fp32 theta [D] (flat order)
    const float* fc;             // [Bs, F] unique-image fc rows
    int32_t* tok;                // [Bs, tok_stride] greedy tokens of logit steps 1..L-1 (unmasked)
    int32_t tok_stride;
    int32_t tok_internal;        // 1: the forward picks them itself (argmax of its log_softmax) and writes tok
    int32_t Bs, V1, E, R, F;
    int32_t L;                   // greedy steps (forward_for_sensitivity length = 5)
    int32_t split;               // vocabulary group size (100)
    int32_t K;                   // groups = V1 / split + 1 (the zero padding always adds split - V1 % split)
    int64_t D;
    int64_t off_img_w, off_img_b, off_emb_w, off_log_w, off_log_b, off_i2h_w, off_i2h_b, off_h2h_w, off_h2h_b;
    float underflow;             // > 0: clamp + divide as calc_sensitivity; <= 0: the raw sensitivity
    float* out;                  // [D]
};

struct SensWork;
extern "C" SensWork* nicnes_sens_create();
extern "C" void nicnes_sens_destroy(SensWork* w);
// 0 on success; the work buffers grow to the largest (Bs, K) seen (K x D floats for the gradients)
extern "C" int nicnes_sens_run(SensWork* w, const SensParams* p, hipStream_t stream);
