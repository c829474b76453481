// mfma_probe.hip -- dev microbenchmark: v_mfma_f32_32x32x2_f32 throughput with 1 or 2 dependent
// accumulator chains per wave, 1 or 2 waves per SIMD, with/without interleaved VALU work.
// Build: hipcc --offload-arch=gfx950 -O3 scripts/mfma_probe.hip -o scripts/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CHAINS, int VALU>
__global__ __launch_bounds__(512) void probe(float* out, int iters, float seed) {
    f32x16 acc0 = {}, acc1 = {};
    float a = seed + threadIdx.x * 1e-3f, b = seed * 0.5f;
    float v0 = a, v1 = b, v2 = a * b;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 64 / CHAINS; ++k) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc0, 0, 0, 0);
            if (CHAINS == 2) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc1, 0, 0, 0);
#pragma unroll
            for (int q = 0; q < VALU; ++q) {
                v0 = __builtin_fmaf(v0, 1.0001f, v1);
                v1 = __builtin_fmaf(v1, 0.9999f, v2);
                v2 = __builtin_fmaf(v2, 1.0002f, v0);
            }
        }
    }
    float s = v0 + v1 + v2;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS, int VALU>
void run(const char* name, int threads, float* out) {
    const int iters = 200, blocks = 256;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((probe<CHAINS, VALU>), dim3(blocks), dim3(threads), 0, 0, out, 10, 1.0f);
    hipEventRecord(e0);
    hipLaunchKernelGGL((probe<CHAINS, VALU>), dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)blocks * (threads / 64) * iters * 64 * 32 * 32 * 2 * 2;
    printf("%-28s waves/SIMD=%d  %8.3f ms  %7.1f TFLOP/s\n", name, threads / 256, ms, flops / ms / 1e9);
}

int main() {
    float* out;
    hipMalloc(&out, 256 * 512 * sizeof(float));
    run<1, 0>("1 chain, no valu", 256, out);
    run<2, 0>("2 chains, no valu", 256, out);
    run<1, 0>("1 chain, no valu", 512, out);
    run<2, 0>("2 chains, no valu", 512, out);
    run<1, 1>("1 chain, 3 valu/mfma", 512, out);
    run<1, 2>("1 chain, 6 valu/mfma", 512, out);
    run<2, 1>("2 chains, 3 valu/mfma", 512, out);
    run<2, 2>("2 chains, 6 valu/mfma", 512, out);
    run<1, 1>("1 chain, 3 valu/mfma", 256, out);
    run<2, 1>("2 chains, 3 valu/mfma", 256, out);
    return 0;
}
