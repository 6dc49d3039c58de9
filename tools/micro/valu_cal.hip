// Chip-wide VALU rate calibration, timed by HIP events (r06).
//
// Settles what one wave64 VALU instruction costs a SIMD on gfx950, the price
// bench.py's roofline block puts on the enhance kernel's instruction counts:
// every SIMD of the chip runs W waves (W = 1, 2, 3, 4, 8) of dense,
// dependency-free streams (8 independent chains per lane, 128 instructions
// per loop iteration, so the loop branch is < 2 % of the stream), one op per
// kernel:
//   v_fma_f32      2 FLOP per lane
//   v_pk_fma_f32   4 FLOP per lane (two f32 FMAs)
//   v_pk_add_f32   2 FLOP per lane (two f32 adds)
//   v_add_f32      1 FLOP per lane
//   v_exp_f32      transcendental
//   v_fma_f64      2 FLOP per lane
// Every op takes the loop-invariant scalar s as an SGPR operand (tools/micro/
// valu_mix.hip: VGPR-only v_add_f32 / v_mul_f32 streams issue at 2.3-2.5
// cycles, the SGPR forms at 4).
// The launch is timed by HIP events (the whole chip, 256 CUs x 4 SIMDs x W
// waves); the clock the part held is s_memtime / s_memrealtime (100 MHz) of
// each workgroup's loop.  Printed per (op, W): ms, TFLOP/s (lane-op rate for
// exp), and SIMD cycles per wave-instruction at the held clock,
//   cycles = t * clk / (W * instructions per wave).
// MI355X_MICROARCH.md: 2 cycles per wave64 v_fma_f32 (SIMD-32), one wave
// alone 4; FP32 vector peak 157.3 TF = 64 FLOP/clk/SIMD, which puts a packed
// v_pk_fma_f32 (4 FLOP per lane) at 4 cycles; FP64 vector 78.6 TF = 4 cycles.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/micro/valu_cal.hip -o tools/micro/valu_cal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

enum { FMA = 0, PK_FMA, PK_ADD, ADD, EXP, FMA64, NOPS };
static const char* kNames[NOPS] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_add_f32",
                                   "v_exp_f32", "v_fma_f64"};
static const double kFlopPerLane[NOPS] = {2, 4, 2, 1, 1, 2};

constexpr int C = 8;    // independent chains per lane
constexpr int U = 16;   // unrolled rounds per loop iteration: 128 instructions

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, long long* stamps, int iters, float s) {
    float a[C];
    f2 p[C];
    double d[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        a[j] = threadIdx.x * 1e-3f + j * 0.01f;
        p[j] = f2{a[j], -a[j]};
        d[j] = (double)a[j];
    }
    const double sd = (double)s;
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int j = 0; j < C; ++j) {
                if (OP == FMA) a[j] = __builtin_fmaf(a[j], s, 0.5f);
                if (OP == PK_FMA) p[j] = __builtin_elementwise_fma(p[j], f2{s, s}, f2{0.5f, 0.25f});
                if (OP == PK_ADD) p[j] = p[j] + f2{s, 0.5f};
                if (OP == ADD) a[j] = a[j] + s;
                if (OP == EXP) a[j] = __builtin_amdgcn_exp2f(a[j]);
                if (OP == FMA64) d[j] = __builtin_fma(d[j], sd, 0.5);
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) t += a[j] + p[j].x + p[j].y + (float)d[j];
    out[blockIdx.x * 256 + threadIdx.x] = t;
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int OP>
static void launch(int blocks, float* out, long long* st, int iters) {
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, st, iters, 0.999f);
}

static void run(int op, int blocks, float* out, long long* st, int iters) {
    switch (op) {
        case FMA: launch<FMA>(blocks, out, st, iters); break;
        case PK_FMA: launch<PK_FMA>(blocks, out, st, iters); break;
        case PK_ADD: launch<PK_ADD>(blocks, out, st, iters); break;
        case ADD: launch<ADD>(blocks, out, st, iters); break;
        case EXP: launch<EXP>(blocks, out, st, iters); break;
        default: launch<FMA64>(blocks, out, st, iters); break;
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2048;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;  // 256 on MI355X
    const int simds = 4 * cus;
    const int maxb = cus * 8;
    float* out;
    long long* st;
    (void)hipMalloc(&out, (size_t)maxb * 256 * sizeof(float));
    (void)hipMalloc(&st, (size_t)maxb * 2 * sizeof(long long));
    long long* h = (long long*)malloc((size_t)maxb * 2 * sizeof(long long));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("# %d CUs, %d SIMDs; %d iterations x %d instructions per wave; HIP-event time of the whole launch\n",
           cus, simds, iters, U * C);
    printf("%-13s %2s %9s %9s %10s %8s\n", "op", "W", "ms", "TFLOP/s", "cyc/winst", "clk GHz");
    const int ws[] = {1, 2, 3, 4, 8};
    for (int op = 0; op < NOPS; ++op) {
        for (int w : ws) {
            const int blocks = cus * w;  // 4 waves per block: w waves on every SIMD
            const int it = op == EXP ? iters / 2 : iters;
            run(op, blocks, out, st, it);  // warm (clock ramp, code fetch)
            (void)hipDeviceSynchronize();
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0, 0);
                run(op, blocks, out, st, it);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms = 0.f;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            (void)hipMemcpy(h, st, (size_t)blocks * 2 * sizeof(long long), hipMemcpyDeviceToHost);
            double cyc = 0, real = 0;
            for (int b = 0; b < blocks; ++b) {
                cyc += (double)h[2 * b];
                real += (double)h[2 * b + 1];
            }
            const double clk = cyc / real * 0.1e9;           // shader cycles per second
            const double winst = (double)it * U * C;          // wave-instructions per wave
            const double lanes = (double)blocks * 256.0;
            const double flops = lanes * winst * kFlopPerLane[op];
            const double t = best * 1e-3;
            const double cyc_per = t * clk / (w * winst);     // SIMD cycles per wave-instruction
            printf("%-13s %2d %9.3f %9.2f %10.3f %8.3f\n", kNames[op], w, best, flops / t / 1e12, cyc_per,
                   clk / 1e9);
            printf("JSON {\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"tflops\": %.3f, "
                   "\"cycles_per_wave_inst\": %.4f, \"clock_ghz\": %.4f, \"simds\": %d}\n",
                   kNames[op], w, best, flops / t / 1e12, cyc_per, clk / 1e9, simds);
        }
    }
    return 0;
}
