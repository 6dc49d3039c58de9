// fp64 matrix vs vector rate on gfx950, and whether the two run side by side.
// Each wave runs ITER iterations of NV independent v_fma_f64 (8 chains) and NM
// v_mfma_f64_16x16x4_f64 (4 independent accumulators); 3 workgroups of 256
// threads per CU.  SPLIT: even waves run only the VALU stream, odd waves only
// the MFMA stream (the question for a wave-specialised STOI resampler: does an
// fp64 MFMA wave run beside an fp64 VALU wave of the same SIMD?).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f64.hip -o tools/micro/mfma_f64
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NV, int NM, bool SPLIT>
__global__ void __launch_bounds__(256, 3) k(double* out, int iters, double s) {
    const int wave = threadIdx.x >> 6;
    const bool do_v = !SPLIT || (wave & 1) == 0;
    const bool do_m = !SPLIT || (wave & 1) == 1;
    double v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x * 1e-3 + c;
    d4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
    const double a = threadIdx.x * 1e-4, b = 1.0 + threadIdx.x * 1e-5;
    if (do_v && do_m) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < NV / 8; ++r) {
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] = fma(v[c], s, 0.5);
                if (NM >= NV / 8 || (NM && r % ((NV / 8) / NM) == 0)) {
#pragma unroll
                    for (int m = 0; m < (NM + NV / 8 - 1) / (NV / 8); ++m)
                        acc[m & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m & 3], 0, 0, 0);
                }
            }
        }
    } else if (do_v) {
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int r = 0; r < NV / 8; ++r)
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] = fma(v[c], s, 0.5);
    } else if (do_m) {
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[m & 3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[m & 3], 0, 0, 0);
    }
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) t += v[c];
#pragma unroll
    for (int c = 0; c < 4; ++c) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NV, int NM, bool SPLIT>
void run(double* d, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 3;
    k<NV, NM, SPLIT><<<blocks, 256>>>(d, iters, 0.999);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<NV, NM, SPLIT><<<blocks, 256>>>(d, iters, 0.999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // whole-chip rates: VALU fp64 FMA lanes and MFMA flops actually issued
    const double waves = blocks * 4.0, vw = SPLIT ? waves / 2 : (NV ? waves : 0),
                 mw = SPLIT ? waves / 2 : (NM ? waves : 0);
    const double sec = ms / 5 * 1e-3;
    const double vtf = vw * iters * NV * 64 * 2 / sec / 1e12;
    const double mtf = mw * iters * NM * 2048.0 / sec / 1e12;
    printf("%s NV %3d NM %3d  %.3f ms/launch  valu %.1f TF/s  mfma %.1f TF/s  sum %.1f\n",
           SPLIT ? "split" : "same ", NV, NM, ms / 5, vtf, mtf, vtf + mtf);
}

int main() {
    double* d;
    hipMalloc(&d, 256 * 3 * 256 * 8);
    const int it = 1000;
    run<256, 0, false>(d, it);
    run<0, 32, false>(d, it);
    run<256, 16, false>(d, it);
    run<256, 32, false>(d, it);
    run<256, 32, true>(d, it);
    run<256, 64, true>(d, it);
    run<512, 32, true>(d, it);
    return 0;
}
