// Throughput of v_exp_f32 / v_rcp_f32 vs v_fma_f32 per SIMD with many waves
// resident (the cost model of pmc_summary.py / bench.py's valu block).
// hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/micro/valu_rate.hip -o tools/micro/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, int iters, float s, long long* clk) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 1e-3f + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) a[j] = __builtin_fmaf(a[j], s, 0.5f);
            else if (OP == 1) a[j] = __builtin_amdgcn_exp2f(a[j]);
            else a[j] = __builtin_amdgcn_rcpf(a[j]);
        }
    }
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += a[j];
    out[blockIdx.x * 256 + threadIdx.x] = t;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = __builtin_amdgcn_s_memtime() - t0;
}

int main(int argc, char** argv) {
    const int blocks = 256 * 8, iters = argc > 1 ? atoi(argv[1]) : 65536;  // 8 WGs of 4 waves per CU: 8 waves per SIMD
    float* out;
    long long* clk;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipMalloc(&clk, sizeof(long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[3] = {"v_fma_f32", "v_exp_f32", "v_rcp_f32"};
    for (int op = 0; op < 3; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, clk);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, clk);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, clk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double wave_insts = (double)blocks * 4 * iters * 8;  // per SIMD: / 1024
            long long c = 0;
            hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
            // block 0's wave 0 shares its SIMD with 7 other waves for the whole loop
            if (rep) printf("%s: %.3f ms, %.3f ns and %.2f cycles (s_memtime) per wave-instruction per SIMD\n",
                            names[op], ms, ms * 1e6 / (wave_insts / 1024), (double)c / (8.0 * iters * 8));
        }
    }
    return 0;
}
