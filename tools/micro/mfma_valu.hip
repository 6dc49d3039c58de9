// Does an f32 MFMA stream run beside a VALU stream for free?  Each wave runs
// ITER iterations of NV independent v_fma_f32 (8 chains) and NM
// v_mfma_f32_16x16x4_f32 (4 independent accumulators); 3 waves per SIMD
// (768-thread... 256-thread workgroups, 3 per CU).  Prints ms for each (NV, NM).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_valu.hip -o tools/micro/mfma_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NV, int NM>
__global__ void __launch_bounds__(256, 3) k(float* out, int iters, float s) {
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x * 1e-3f + c;
    f4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = f4{0.f, 0.f, 0.f, 0.f};
    float a = threadIdx.x * 1e-4f, b = 1.0f + threadIdx.x * 1e-5f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < NV / 8; ++r) {
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = fmaf(v[c], s, 0.5f);
            if (NM && (r % ((NV / 8) / (NM > NV / 8 ? NV / 8 : NM) ?: 1)) == 0) {
#pragma unroll
                for (int m = 0; m < (NM + (NV / 8) - 1) / (NV / 8); ++m)
                    acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
            }
        }
        if (NV == 0) {
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
        }
    }
    float t = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) t += v[c];
#pragma unroll
    for (int c = 0; c < 4; ++c) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NV, int NM>
void run(float* d, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 3;
    k<NV, NM><<<blocks, 256>>>(d, iters, 0.999f);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<NV, NM><<<blocks, 256>>>(d, iters, 0.999f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // per wave: iters * NV VALU, iters * NM MFMA
    printf("NV %4d NM %3d  %.3f ms/launch  (%.2f ns per VALU-instr-wave, iters %d)\n", NV, NM, ms / 5,
           NV ? ms / 5 * 1e6 / ((double)iters * NV) : 0.0, iters);
}

int main() {
    float* d;
    hipMalloc(&d, 256 * 3 * 256 * 4);
    const int it = 2000;
    run<256, 0>(d, it);
    run<0, 32>(d, it);
    run<256, 8>(d, it);
    run<256, 16>(d, it);
    run<256, 32>(d, it);
    run<256, 64>(d, it);
    run<0, 64>(d, it);
    run<512, 16>(d, it);
    run<512, 32>(d, it);
    run<512, 0>(d, it);
    return 0;
}
