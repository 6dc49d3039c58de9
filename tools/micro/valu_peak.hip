// The VALU rate a SIMD actually sustains, in SHADER CYCLES (s_memtime,
// converted with s_memrealtime's 100 MHz), at W = 1, 2, 3, 4, 6, 8 waves per SIMD and C
// independent chains per lane: scalar v_fma_f32, packed v_pk_fma_f32 (two f32
// operations), v_exp_f32, and the OMLSA bin's mix (27 f32 VALU + 6
// transcendentals, tools' 2/4-cycle model: 66 cycles per bin).  The enhance
// kernel's roofline counts a wave64 f32 instruction as 2 SIMD cycles and a
// transcendental as 4; this says what a dense stream reaches on the part.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/micro/valu_peak.hip -o tools/micro/valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, long long* stamps, int iters, float s) {
    constexpr int C = 8;
    float a[C];
    f2 p[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        a[j] = threadIdx.x * 1e-3f + j;
        p[j] = f2{a[j], -a[j]};
    }
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < C; ++j) {
            if (OP == 0) {
                a[j] = __builtin_fmaf(a[j], s, 0.5f);
            } else if (OP == 1) {
                p[j] = __builtin_elementwise_fma(p[j], f2{s, s}, f2{0.5f, 0.25f});
            } else if (OP == 2) {
                a[j] = __builtin_amdgcn_exp2f(a[j]);
            } else {  // OMLSA-bin-like mix: 27 dependent-ish f32 ops + 6 transcendentals per item
                float x = a[j];
#pragma unroll
                for (int q = 0; q < 27; ++q) x = __builtin_fmaf(x, s, 0.125f);
                x = __builtin_amdgcn_rcpf(x);
                x = __builtin_amdgcn_rsqf(x);
                x = __builtin_amdgcn_logf(x);
                x = __builtin_amdgcn_exp2f(x);
                x = __builtin_amdgcn_rcpf(x);
                x = __builtin_amdgcn_exp2f(x);
                a[j] = x;
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) t += a[j] + p[j].x + p[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = t;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    float* out;
    long long* st;
    const int maxb = 256 * 8;
    (void)hipMalloc(&out, maxb * 256 * sizeof(float));
    (void)hipMalloc(&st, maxb * 2 * sizeof(long long));
    long long* h = (long long*)malloc(maxb * 2 * sizeof(long long));
    const char* names[4] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "omlsa-mix"};
    // wave-instructions per item: 1, 1, 1, 33 (27 + 6)
    const double per_item[4] = {1, 1, 1, 33};
    printf("waves/SIMD | shader cycles per wave-instruction per SIMD (clock GHz): fma  pk_fma  exp  mix(33/item)\n");
    const int ws[] = {1, 2, 3, 4, 6, 8};  // 3: the enhance kernel's own occupancy
    for (int w : ws) {
        const int blocks = 256 * w;  // 4 waves per block, one per SIMD
        printf("%d |", w);
        for (int op = 0; op < 4; ++op) {
            for (int rep = 0; rep < 2; ++rep) {
                if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, st, iters, 0.999f);
                if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, st, iters, 0.999f);
                if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, st, iters / 4, 0.999f);
                if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, st, iters / 16, 0.999f);
                (void)hipDeviceSynchronize();
            }
            (void)hipMemcpy(h, st, blocks * 2 * sizeof(long long), hipMemcpyDeviceToHost);
            double cyc = 0, real = 0;
            for (int b = 0; b < blocks; ++b) {
                cyc += h[2 * b];
                real += h[2 * b + 1];
            }
            cyc /= blocks;
            real /= blocks;
            const int it = op == 2 ? iters / 4 : (op == 3 ? iters / 16 : iters);
            // every wave of the SIMD runs the loop concurrently: SIMD cycles per
            // wave-instruction = cycles / (waves * iters * 8 chains * per_item)
            const double ipc = cyc / ((double)w * it * 8 * per_item[op]);
            printf("  %.2f (%.2f)", ipc, cyc / real * 0.1);
        }
        printf("\n");
    }
    return 0;
}
