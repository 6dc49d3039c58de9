// Issue cost of packed f32 VALU (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32,
// two f32 lanes per instruction) against v_fma_f32 with many waves resident
// and no MFMA: does a packed instruction retire two f32 operations in the
// issue slot of one?  8 independent chains per thread, 8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/pk_rate.hip -o tools/micro/pk_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, int iters, float s) {
    f2 a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = f2{threadIdx.x * 1e-3f + j, threadIdx.x * 2e-3f - j};
    const f2 s2 = f2{s, s * 0.5f};
    const f2 h2 = f2{0.5f, 0.25f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (OP == 0) {  // scalar: two v_fma_f32
                a[j].x = __builtin_fmaf(a[j].x, s2.x, h2.x);
                a[j].y = __builtin_fmaf(a[j].y, s2.y, h2.y);
                asm volatile("" : "+v"(a[j].x), "+v"(a[j].y));  // keep them unpacked
            } else if (OP == 1) {  // v_pk_fma_f32
                a[j] = __builtin_elementwise_fma(a[j], s2, h2);
            } else if (OP == 2) {  // v_pk_mul_f32
                a[j] = a[j] * s2;
            } else if (OP == 3) {  // v_pk_add_f32
                a[j] = a[j] + h2;
            } else {  // complex multiply by a constant rotor: (x c - y s, x s + y c)
                const f2 v = a[j];
                const f2 t = f2{v.x, v.x} * f2{s2.x, s2.y};
                a[j] = __builtin_elementwise_fma(f2{v.y, v.y}, f2{-s2.y, s2.x}, t);
            }
        }
    }
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) t += a[j].x + a[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main(int argc, char** argv) {
    const int blocks = 256 * 8, iters = argc > 1 ? atoi(argv[1]) : 32768;
    float* out;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[5] = {"2x v_fma_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32",
                            "complex rotor (pk)"};
    for (int op = 0; op < 5; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
            if (op == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // per SIMD: blocks*4 waves / 1024 SIMDs, iters*8 items (two f32 each)
            const double items = (double)blocks * 4 * iters * 8 / 1024;
            if (rep) printf("%-20s %.3f ms, %.3f ns per wave-item (2 f32 ops) per SIMD\n", names[op], ms,
                            ms * 1e6 / items);
        }
    }
    return 0;
}
