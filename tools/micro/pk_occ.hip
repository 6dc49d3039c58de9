// Packed against scalar f32 VALU at LOW occupancy: 1-4 waves per SIMD
// (256 threads per workgroup = one wave per SIMD, W workgroups per CU), C
// independent chains per lane.  The question for enhance_kernel (3 waves per
// SIMD, VALU issue 0.66-0.69): does one wave issue a v_pk_fma_f32 (two f32
// operations) at the per-wave cost of one v_fma_f32, so that packing the
// complex arithmetic and the paired gain chains raises what a few waves can
// issue?
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/micro/pk_occ.hip -o tools/micro/pk_occ
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP, int C>
__global__ void __launch_bounds__(256) k(float* out, int iters, float s) {
    f2 a[C];
#pragma unroll
    for (int j = 0; j < C; ++j) a[j] = f2{threadIdx.x * 1e-3f + j, threadIdx.x * 2e-3f - j};
    const f2 s2 = f2{s, s * 0.5f};
    const f2 h2 = f2{0.5f, 0.25f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < C; ++j) {
            if (OP == 0) {  // scalar: two v_fma_f32 per item
                float x = a[j].x, y = a[j].y;
                x = __builtin_fmaf(x, s2.x, h2.x);
                y = __builtin_fmaf(y, s2.y, h2.y);
                asm volatile("" : "+v"(x), "+v"(y));  // keep them unpacked
                a[j] = f2{x, y};
            } else if (OP == 1) {  // one v_pk_fma_f32 per item
                a[j] = __builtin_elementwise_fma(a[j], s2, h2);
            } else {  // complex multiply by a rotor: pk_mul + pk_fma (op_sel)
                const f2 v = a[j];
                const f2 t = f2{v.x, v.x} * s2;
                a[j] = __builtin_elementwise_fma(f2{v.y, v.y}, f2{-s2.y, s2.x}, t);
            }
        }
    }
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) t += a[j].x + a[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int OP, int C>
static double run(int blocks, int iters, float* out, hipEvent_t e0, hipEvent_t e1) {
    float ms = 0.f;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k<OP, C>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    return ms;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 8192;
    float* out;
    hipMalloc(&out, 256 * 8 * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("waves/SIMD chains | ns per wave-item (2 f32 ops): 2x v_fma_f32, v_pk_fma_f32, complex rotor (pk_mul+pk_fma)\n");
    for (int w = 1; w <= 4; ++w) {
        const int blocks = 256 * w;
        // per SIMD: w waves, iters * C items each
        auto per = [&](double ms, int C) { return ms * 1e6 / ((double)w * iters * C); };
        double a = run<0, 2>(blocks, iters, out, e0, e1), b = run<1, 2>(blocks, iters, out, e0, e1),
               c = run<2, 2>(blocks, iters, out, e0, e1);
        printf("%d  2 | %.3f %.3f %.3f\n", w, per(a, 2), per(b, 2), per(c, 2));
        a = run<0, 8>(blocks, iters, out, e0, e1), b = run<1, 8>(blocks, iters, out, e0, e1),
        c = run<2, 8>(blocks, iters, out, e0, e1);
        printf("%d  8 | %.3f %.3f %.3f\n", w, per(a, 8), per(b, 8), per(c, 8));
    }
    return 0;
}
