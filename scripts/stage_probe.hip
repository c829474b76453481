// stage_probe.hip -- dev microbenchmark of the decode's 64-row stage structure on gfx950:
// 8 waves per workgroup (2 per SIMD), one workgroup per CU (two 68 KB LDS buffers), each wave running
// 2 chains of 64 v_mfma_f32_32x32x2_f32 per stage (B operand in registers), for 150 stages. Variants
// add, one at a time: A operands read from LDS (ds_read_b128, as the kernel does), a barrier per stage,
// and the W+- staging (global loads one stage ahead, 3 VALU per element, ds_write_b128).
// Build: hipcc --offload-arch=gfx950 -O3 scripts/stage_probe.hip -o scripts/stage_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
#define LDS_ROW 132
#define STAGE_FLOATS (2 * 64 * LDS_ROW + 128)

template <bool LDS_A, bool BAR, int STAGE>
__global__ __launch_bounds__(512) void stage_probe(const float* __restrict__ w, const float* __restrict__ z,
                                                   float* out, int nst, float sigma) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, sgn = wave >> 2;
    float hB[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) hB[i] = 1e-3f * (float)((lane + i) & 7);
    f32x4 areg[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) areg[i] = (f32x4){1e-3f * i, 2e-3f, 3e-3f, 4e-3f};
    for (int i = tid; i < 2 * STAGE_FLOATS; i += 512) lds[i] = 1e-3f * (float)(i & 15);
    __syncthreads();
    f32x16 acc0 = {}, acc1 = {};
    f32x4 sw[4], sz[4];
    const size_t so = (size_t)blockIdx.x * 65536 + 4 * tid;
    const size_t zs = (size_t)blockIdx.x * (size_t)(nst + 1) * 8192 + 4 * tid;   // STAGE 7: the block's z stream
    if (STAGE == 1 || STAGE == 2 || STAGE == 5 || STAGE == 7) {
#pragma unroll
        for (int u = 0; u < 4; ++u) { sw[u] = *(const f32x4*)(w + so + 2048 * u); sz[u] = *(const f32x4*)(z + so + 2048 * u); }
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) { sw[u] = (f32x4){1.f * u, 2.f, 3.f, 4.f}; sz[u] = (f32x4){0.5f, 0.25f * u, 1.f, 2.f}; }
    }
    f32x4 sink = {};
    f32x4 sw2[4], sz2[4];                 // variant 6: second half of a sign-0 thread's rows
    if (STAGE == 6) {
#pragma unroll
        for (int u = 0; u < 4; ++u) { sw[u] = *(const f32x4*)(w + so + 2048 * u); sz[u] = *(const f32x4*)(z + so + 2048 * u);
                                      sw2[u] = sw[u]; sz2[u] = sz[u]; }
    }
    const int arow = (lane & 31) * LDS_ROW + 16 * (lane >> 5);
    for (int s = 0; s < nst; ++s) {
        const float* buf = lds + (s & 1) * STAGE_FLOATS + sgn * 64 * LDS_ROW;
        f32x4 nw[4], nz[4];
        const size_t o2 = so + (size_t)((s + 1) & 15) * 8192;
        if (STAGE == 6 && sgn == 0) {
            const size_t o4 = (size_t)blockIdx.x * 65536 + 4 * (tid & 255) + (size_t)((s + 1) & 15) * 8192 + 4096;
#pragma unroll
            for (int u = 0; u < 4; ++u) { nw[u] = *(const f32x4*)(w + o4 + 1024 * u); nz[u] = *(const f32x4*)(z + o4 + 1024 * u); }
        }
        if (STAGE == 1 || STAGE == 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) { nw[u] = *(const f32x4*)(w + o2 + 2048 * u); nz[u] = *(const f32x4*)(z + o2 + 2048 * u); }
        }
        if (STAGE == 7) {
#pragma unroll
            for (int u = 0; u < 4; ++u) { nw[u] = *(const f32x4*)(w + o2 + 2048 * u);
                                          nz[u] = *(const f32x4*)(z + zs + (size_t)(s + 1) * 8192 + 2048 * u); }
        }
#pragma unroll
        for (int T = 0; T < 4; ++T) {
            if (STAGE == 5) {             // the next stage's loads spread over the MFMA chunks
                nw[T] = *(const f32x4*)(w + o2 + 2048 * T);
                nz[T] = *(const f32x4*)(z + o2 + 2048 * T);
            }
            f32x4 a0[4], a1[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (LDS_A) {
                    a0[c] = *reinterpret_cast<const f32x4*>(buf + arow + T * 32 + 4 * c);
                    a1[c] = *reinterpret_cast<const f32x4*>(buf + 32 * LDS_ROW + arow + T * 32 + 4 * c);
                } else {
                    a0[c] = areg[c];
                    a1[c] = areg[4 + c];
                }
            }
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], hB[16 * T + jj], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], hB[16 * T + jj], acc1, 0, 0, 0);
            }
        }
        if (STAGE == 6 && sgn == 0) {
            const size_t o3 = (size_t)blockIdx.x * 65536 + 4 * (tid & 255) + (size_t)((s + 1) & 15) * 8192;
            f32x4 mw[4], mz[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { mw[u] = *(const f32x4*)(w + o3 + 1024 * u); mz[u] = *(const f32x4*)(z + o3 + 1024 * u); }
            float* b = lds + ((s + 1) & 1) * STAGE_FLOATS + ((tid & 255) >> 5) * LDS_ROW + 4 * (tid & 31);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f32x4 d = sigma * sz[u], d2 = sigma * sz2[u];
                *reinterpret_cast<f32x4*>(b + 8 * u * LDS_ROW) = sw[u] + d;
                *reinterpret_cast<f32x4*>(b + (64 + 8 * u) * LDS_ROW) = sw[u] - d;
                *reinterpret_cast<f32x4*>(b + (32 + 8 * u) * LDS_ROW) = sw2[u] + d2;
                *reinterpret_cast<f32x4*>(b + (96 + 8 * u) * LDS_ROW) = sw2[u] - d2;
                sw[u] = nw[u]; sz[u] = nz[u]; sw2[u] = mw[u]; sz2[u] = mz[u];
            }
        }
        if (STAGE == 1 || STAGE == 5 || STAGE == 7) {
            float* b = lds + ((s + 1) & 1) * STAGE_FLOATS + (tid >> 5) * LDS_ROW + 4 * (tid & 31);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f32x4 d = sigma * sz[u];
                *reinterpret_cast<f32x4*>(b + 16 * u * LDS_ROW) = sw[u] + d;
                *reinterpret_cast<f32x4*>(b + (64 + 16 * u) * LDS_ROW) = sw[u] - d;
                sw[u] = nw[u];
                sz[u] = nz[u];
            }
        } else if (STAGE == 2) {          // loads only: one add per loaded vector into a sink
#pragma unroll
            for (int u = 0; u < 4; ++u) { sink += sw[u]; sink += sz[u]; sw[u] = nw[u]; sz[u] = nz[u]; }
        } else if (STAGE == 3) {          // LDS writes only (of register constants)
            float* b = lds + ((s + 1) & 1) * STAGE_FLOATS + (tid >> 5) * LDS_ROW + 4 * (tid & 31);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                *reinterpret_cast<f32x4*>(b + 16 * u * LDS_ROW) = sw[u];
                *reinterpret_cast<f32x4*>(b + (64 + 16 * u) * LDS_ROW) = sz[u];
            }
        } else if (STAGE == 4) {          // the W+- VALU only
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f32x4 d = sigma * sz[u];
                sink += sw[u] + d;
                sink += sw[u] - d;
                sw[u] = sw[u] + (f32x4){1e-7f, 1e-7f, 1e-7f, 1e-7f};
            }
        }
        if (BAR) __syncthreads();
    }
    float r = sink[0] + sink[1] + sink[2] + sink[3];
#pragma unroll
    for (int i = 0; i < 16; ++i) r += acc0[i] + acc1[i];
    out[blockIdx.x * 512 + tid] = r;
}

template <bool LDS_A, bool BAR, int STAGE>
void run(const char* name, const float* w, const float* z, float* out) {
    const int nst = 150, blocks = 256;
    const size_t lds = 2 * STAGE_FLOATS * sizeof(float);
    hipFuncSetAttribute((const void*)stage_probe<LDS_A, BAR, STAGE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((stage_probe<LDS_A, BAR, STAGE>), dim3(blocks), dim3(512), lds, 0, w, z, out, 10, 0.01f);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((stage_probe<LDS_A, BAR, STAGE>), dim3(blocks), dim3(512), lds, 0, w, z, out, nst, 0.01f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double flops = (double)blocks * 8 * nst * 128 * 32 * 32 * 2 * 2;
    printf("%-40s %8.3f ms  %7.1f TFLOP/s  %5.1f%% of 157.3  %6.2f us/stage\n", name, best, flops / best / 1e9,
           flops / best / 1e9 / 157.3 * 100.0 / 1000.0, best * 1e3 / nst);
}


// sign-split layout: a 4-wave workgroup per (member, sign), two per CU; each stages its own sign's 64-row
// tile (W0 + z loaded per workgroup, so every element is loaded twice per CU, written once per sign)
__global__ __launch_bounds__(256) void stage_probe_split(const float* __restrict__ w, const float* __restrict__ z,
                                                         float* out, int nst, float sigma) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const float sg = (blockIdx.x & 1) ? -sigma : sigma;
    float hB[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) hB[i] = 1e-3f * (float)((lane + i) & 7);
    for (int i = tid; i < 2 * (64 * LDS_ROW + 64); i += 256) lds[i] = 1e-3f * (float)(i & 15);
    __syncthreads();
    f32x16 acc0 = {}, acc1 = {};
    f32x4 sw[8], sz[8];
    const size_t so = (size_t)(blockIdx.x >> 1) * 65536 + 4 * tid;
#pragma unroll
    for (int u = 0; u < 8; ++u) { sw[u] = *(const f32x4*)(w + so + 1024 * u); sz[u] = *(const f32x4*)(z + so + 1024 * u); }
    const int arow = (lane & 31) * LDS_ROW + 16 * (lane >> 5);
    for (int s = 0; s < nst; ++s) {
        const float* buf = lds + (s & 1) * (64 * LDS_ROW + 64);
        f32x4 nw[8], nz[8];
        const size_t o2 = so + (size_t)((s + 1) & 15) * 8192;
#pragma unroll
        for (int u = 0; u < 8; ++u) { nw[u] = *(const f32x4*)(w + o2 + 1024 * u); nz[u] = *(const f32x4*)(z + o2 + 1024 * u); }
#pragma unroll
        for (int T = 0; T < 4; ++T) {
            f32x4 a0[4], a1[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                a0[c] = *reinterpret_cast<const f32x4*>(buf + arow + T * 32 + 4 * c);
                a1[c] = *reinterpret_cast<const f32x4*>(buf + 32 * LDS_ROW + arow + T * 32 + 4 * c);
            }
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], hB[16 * T + jj], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], hB[16 * T + jj], acc1, 0, 0, 0);
            }
        }
        float* b = lds + ((s + 1) & 1) * (64 * LDS_ROW + 64) + (tid >> 5) * LDS_ROW + 4 * (tid & 31);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            *reinterpret_cast<f32x4*>(b + 8 * u * LDS_ROW) = sw[u] + sg * sz[u];
            sw[u] = nw[u];
            sz[u] = nz[u];
        }
        __syncthreads();
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += acc0[i] + acc1[i];
    out[blockIdx.x * 256 + tid] = r;
}

void run_split(const char* name, const float* w, const float* z, float* out) {
    const int nst = 150, blocks = 512;
    const size_t lds = 2 * (64 * LDS_ROW + 64) * sizeof(float);
    hipFuncSetAttribute((const void*)stage_probe_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(stage_probe_split, dim3(blocks), dim3(256), lds, 0, w, z, out, 10, 0.01f);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(stage_probe_split, dim3(blocks), dim3(256), lds, 0, w, z, out, nst, 0.01f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double flops = (double)blocks * 4 * nst * 128 * 32 * 32 * 2 * 2;
    printf("%-40s %8.3f ms  %7.1f TFLOP/s  %5.1f%% of 157.3  %6.2f us/stage\n", name, best, flops / best / 1e9,
           flops / best / 1e9 / 157.3 * 100.0 / 1000.0, best * 1e3 / nst);
}

// LDS-DMA staging (glds): W0 and z tiles go global -> LDS with no VGPR destination (8 x 1 KiB
// global_load_lds_dwordx4 per wave and stage); each wave forms its own sign's A operand at read time
// (w + z or w - z, VALU per A value). LDS image per plane: 32 "pair rows" of 1 KiB + 16 B pad, pair
// row p holding matrix rows r0(p) and r0(p) + 16 (r0 = (p & 15) + 32 (p >> 4)): one wave-instruction
// fills one pair row, and a ds_read_b128 lane group (16 distinct rows r & 15) is conflict-free.
#define PAIR_BYTES 1040
#define PLANE_BYTES (32 * PAIR_BYTES)
#define GBUF_BYTES (2 * PLANE_BYTES)
typedef __attribute__((address_space(3))) void lds_void;
template <int MODE, bool NEG>
__device__ __forceinline__ void glds_stage(const char* buf, int abase, const float (&hB)[64], f32x16& acc0, f32x16& acc1) {
#pragma unroll
    for (int T = 0; T < 4; ++T) {
        f32x4 a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int off = abase + 16 * (8 * T + c);
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(buf + off);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(buf + off + 16 * PAIR_BYTES);
            if (MODE == 1) { a0[c] = w0; a1[c] = w1; continue; }
            if (MODE >= 3) {              // pre-formed W+- planes: the sign's own plane, no VALU
                a0[c] = *reinterpret_cast<const f32x4*>(buf + (NEG ? PLANE_BYTES : 0) + off);
                a1[c] = *reinterpret_cast<const f32x4*>(buf + (NEG ? PLANE_BYTES : 0) + off + 16 * PAIR_BYTES);
                continue;
            }
            const f32x4 z0 = *reinterpret_cast<const f32x4*>(buf + PLANE_BYTES + off);
            const f32x4 z1 = *reinterpret_cast<const f32x4*>(buf + PLANE_BYTES + off + 16 * PAIR_BYTES);
            a0[c] = NEG ? w0 - z0 : w0 + z0;
            a1[c] = NEG ? w1 - z1 : w1 + z1;
        }
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[jj >> 2][jj & 3], hB[16 * T + jj], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[jj >> 2][jj & 3], hB[16 * T + jj], acc1, 0, 0, 0);
        }
    }
}

template <int MODE, bool NEG>
__device__ __forceinline__ void glds_loop(char* lds, const float* w, const float* z, int nst, const float (&hB)[64],
                                          f32x16& acc0, f32x16& acc1) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // this lane's A-operand base: row r = lane & 31 of chain a (chain b: + 16 pair rows), k chunk 4 (lane >> 5)
    const int r = lane & 31;
    const int abase = (r & 15) * PAIR_BYTES + (r >> 4) * 512 + 64 * (lane >> 5);
    // glds: wave w fills pair rows 8w .. 8w + 7 of the planes (waves 0-3: W0, 4-7: z)
    const float* src = (wave < 4) ? w : z;
    const size_t gl = (size_t)blockIdx.x * 65536 + (size_t)(16 * (lane >> 5)) * 128 + 4 * (lane & 31);
    for (int s = 0; s < nst; ++s) {
        if (s + 1 < nst || MODE == 2) {
            char* nb = lds + ((s + 1) & 1) * GBUF_BYTES + (wave >> 2) * PLANE_BYTES;
            if (MODE == 5) {              // as MODE 3 through a buffer resource (buffer_load ... lds, soffset per row)
                const size_t cyc = (size_t)nst + 1;
                const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                    (void*)(w + (size_t)blockIdx.x * cyc * 16384), (short)0, (int)(cyc * 16384 * 4), 0x00020000);
                const unsigned soff = 4u * (unsigned)(((s + 1) % cyc) * 16384 + (wave >> 2) * 8192);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p = 8 * (wave & 3) + j;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, (lds_void*)(nb + p * PAIR_BYTES), 16, 16 * lane,
                                                             (int)(soff + 1024u * p), 0, 0);
                }
            } else if (MODE >= 3) {              // pre-formed image: 1 KiB per pair row, the workgroup's own stream
                const size_t cyc = MODE == 3 ? (size_t)nst + 1 : 16;
                const size_t so = (size_t)blockIdx.x * cyc * 16384 + (size_t)((s + 1) % cyc) * 16384 +
                                  (size_t)(wave >> 2) * 8192 + 4 * lane;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p = 8 * (wave & 3) + j;
                    __builtin_amdgcn_global_load_lds((const void*)(w + so + 256 * p),
                                                     (lds_void*)(nb + p * PAIR_BYTES), 16, 0, 0);
                }
            } else {
            const size_t so = gl + (size_t)((s + 1) & 15) * 8192;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int p = 8 * (wave & 3) + j, r0 = (p & 15) + 32 * (p >> 4);
                __builtin_amdgcn_global_load_lds((const void*)(src + so + (size_t)r0 * 128),
                                                 (lds_void*)(nb + p * PAIR_BYTES), 16, 0, 0);
            }
            }
        }
        glds_stage<MODE, NEG>(lds + (s & 1) * GBUF_BYTES, abase, hB, acc0, acc1);
        __syncthreads();
    }
}

template <int MODE>
__global__ __launch_bounds__(512) void stage_probe_glds(const float* __restrict__ w, const float* __restrict__ z,
                                                        float* out, int nst) {
    extern __shared__ __attribute__((aligned(16))) char glds_buf[];
    const int tid = threadIdx.x, lane = tid & 63, sgn = tid >> 8;
    float hB[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) hB[i] = 1e-3f * (float)((lane + i) & 7);
    for (int i = tid; i < 2 * GBUF_BYTES / 4; i += 512) reinterpret_cast<float*>(glds_buf)[i] = 1e-3f * (float)(i & 15);
    __syncthreads();
    f32x16 acc0 = {}, acc1 = {};
    if (sgn) glds_loop<MODE, true>(glds_buf, w, z, nst, hB, acc0, acc1);
    else glds_loop<MODE, false>(glds_buf, w, z, nst, hB, acc0, acc1);
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += acc0[i] + acc1[i];
    out[blockIdx.x * 512 + tid] = r;
}

template <int MODE>
void run_glds(const char* name, const float* w, const float* z, float* out) {
    const int nst = 150, blocks = 256;
    const size_t lds = 2 * GBUF_BYTES;
    hipFuncSetAttribute((const void*)stage_probe_glds<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((stage_probe_glds<MODE>), dim3(blocks), dim3(512), lds, 0, w, z, out, 10);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((stage_probe_glds<MODE>), dim3(blocks), dim3(512), lds, 0, w, z, out, nst);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    const double flops = (double)blocks * 8 * nst * 128 * 32 * 32 * 2 * 2;
    printf("%-40s %8.3f ms  %7.1f TFLOP/s  %5.1f%% of 157.3  %6.2f us/stage\n", name, best, flops / best / 1e9,
           flops / best / 1e9 / 157.3 * 100.0 / 1000.0, best * 1e3 / nst);
}

int main() {
    float *w, *z, *out;
    const size_t n = (size_t)256 * 65536 + 16 * 8192 + 8192;
    hipMalloc(&w, n * sizeof(float));
    hipMalloc(&z, n * sizeof(float));
    hipMemset(w, 0, n * sizeof(float));
    hipMemset(z, 0, n * sizeof(float));
    hipMalloc(&out, 256 * 512 * sizeof(float));
    run<false, false, 0>("A in registers, no barrier", w, z, out);
    run<true, false, 0>("A from LDS, no barrier", w, z, out);
    run<true, true, 0>("A from LDS, barrier per stage", w, z, out);
    run<true, true, 1>("A from LDS, barrier, W+- staging", w, z, out);
    run<true, true, 2>("  staging: global loads only", w, z, out);
    run<true, true, 3>("  staging: LDS writes only", w, z, out);
    run<true, true, 4>("  staging: VALU only", w, z, out);
    run<true, true, 5>("W+- staging, loads spread over the MFMAs", w, z, out);
    run<true, true, 6>("W+- staging by the sign-0 waves only", w, z, out);
    run_split("sign-split: 2 x 4-wave workgroups per CU", w, z, out);
    run<true, true, 1>("A from LDS, barrier, W+- staging (again)", w, z, out);
    run_glds<1>("glds W0+z, A = W0 (no z read, no VALU)", w, z, out);
    float* big;
    const size_t nbig = (size_t)256 * 151 * 16384;
    hipMalloc(&big, nbig * sizeof(float));
    hipMemset(big, 0, nbig * sizeof(float));
    run<true, true, 7>("reg staging, z streamed from HBM", w, big, out);
    run_glds<3>("glds pre-formed W+- from HBM", big, z, out);
    run_glds<4>("glds pre-formed W+- (L2-resident)", big, z, out);
    run<true, true, 7>("reg staging, z streamed from HBM (again)", w, big, out);
    run_glds<3>("glds pre-formed W+- from HBM (again)", big, z, out);
    run_glds<5>("buffer_load lds pre-formed W+- from HBM", big, z, out);
    run_glds<5>("buffer_load lds pre-formed W+- (again)", big, z, out);
    run<true, true, 0>("A from LDS, barrier per stage (again)", w, z, out);
    return 0;
}
