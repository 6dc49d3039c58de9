// Does an i8 MFMA stream run beside an fp64 VALU stream on one SIMD?  The
// question behind an integer-sliced STOI resampler: the
// 581-tap FIR as a Hankel GEMM on the matrix pipe while the rfft keeps the
// fp64 VALU busy.  Each wave runs ITER iterations of NV independent v_fma_f64
// (8 chains) and/or NM v_mfma_i32_16x16x64_i8 (4 accumulators); 3 workgroups
// of 256 threads per CU.  SPLIT: even waves VALU only, odd waves MFMA only.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_i8_f64.hip -o tools/micro/mfma_i8_f64
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef int i4 __attribute__((ext_vector_type(4)));

template <int NV, int NM, bool SPLIT>
__global__ void __launch_bounds__(256, 3) k(double* out, int iters, double s, int seed) {
    const int wave = threadIdx.x >> 6;
    const bool do_v = NV > 0 && (!SPLIT || (wave & 1) == 0);
    const bool do_m = NM > 0 && (!SPLIT || (wave & 1) == 1);
    double v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x * 1e-3 + c;
    i4 acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = i4{0, 0, 0, 0};
    // operands depend on a runtime seed so the MFMA stream is not folded away
    i4 a = i4{seed + (int)threadIdx.x, seed ^ 0x01010101, seed * 3, seed + 7};
    i4 b = i4{seed - (int)threadIdx.x, seed ^ 0x02020202, seed * 5, seed + 11};
    for (int it = 0; it < iters; ++it) {
        if (do_v) {
#pragma unroll
            for (int r = 0; r < NV / 8; ++r)
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] = fma(v[c], s, 0.5);
        }
        if (do_m) {
#pragma unroll
            for (int m = 0; m < NM; ++m)
                acc[m & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[m & 3], 0, 0, 0);
            a.x += acc[0].x & 1;  // a loop-carried operand: one MFMA stream per iteration
        }
    }
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) t += v[c];
#pragma unroll
    for (int c = 0; c < 4; ++c) t += (double)(acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3]);
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int NV, int NM, bool SPLIT>
void run(double* d, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int blocks = 256 * 3;
    k<NV, NM, SPLIT><<<blocks, 256>>>(d, iters, 0.999, 3);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k<NV, NM, SPLIT><<<blocks, 256>>>(d, iters, 0.999, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = blocks * 4.0, vw = SPLIT ? waves / 2 : (NV ? waves : 0),
                 mw = SPLIT ? waves / 2 : (NM ? waves : 0);
    const double sec = ms / 5 * 1e-3;
    const double vtf = vw * iters * NV * 64 * 2 / sec / 1e12;         // fp64 TF/s
    const double mto = mw * iters * NM * 16.0 * 16 * 64 * 2 / sec / 1e12;  // i8 TOP/s
    printf("%s NV %3d NM %3d  %.3f ms/launch  fp64 valu %.1f TF/s  i8 mfma %.0f TOP/s\n",
           SPLIT ? "split" : "same ", NV, NM, ms / 5, vtf, mto);
}

int main() {
    double* d;
    hipMalloc(&d, 256 * 3 * 256 * 8);
    const int it = 1000;
    run<256, 0, false>(d, it);   // fp64 VALU alone (every wave)
    run<0, 32, false>(d, it);    // i8 MFMA alone (every wave)
    run<256, 0, true>(d, it);    // fp64 VALU alone, half the waves
    run<0, 32, true>(d, it);     // i8 MFMA alone, half the waves
    run<256, 32, true>(d, it);   // both, wave-split: concurrent if ~max(), not sum()
    run<256, 64, true>(d, it);
    run<256, 32, false>(d, it);  // both in every wave
    return 0;
}
