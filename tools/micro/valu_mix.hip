// What a SIMD sustains for VALU instruction MIXES (r06), chip-wide, HIP-event
// timed: valu_cal.hip found a dense stream of one f32 instruction kind at 4.0
// SIMD cycles per wave64 instruction even at 8 waves/SIMD (v_fma_f32 77.5 TF,
// v_pk_fma_f32 153.5 TF), while the scalar n_fft 1024 enhance kernel's VALU
// instruction count priced at 4 cycles exceeds its SIMD cycles 1.4x (its
// SQ_ACTIVE_INST_VALU reads 1.48 waves VALU-active per SIMD).  So some VALU
// instructions of different waves overlap.  This times streams of exactly the
// instructions named (inline asm, 8 independent chains per lane, 128 per loop
// iteration), alone and pairwise interleaved, at 1, 3 and 8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_mix.hip -o tools/micro/valu_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

enum K { FMA = 0, FMAS, ADD, MUL, MAX, MED3, MOV, ADDU, PKFMA, PKADD, EXP, FMA64, CNDM, NK };
static const char* kName[NK] = {"v_fma_f32(vvv)", "v_fma_f32(vsc)", "v_add_f32", "v_mul_f32", "v_max_f32",
                                "v_med3_f32", "v_mov_b32", "v_add_u32", "v_pk_fma_f32", "v_pk_add_f32",
                                "v_exp_f32", "v_fma_f64", "v_cndmask_b32"};

struct Regs {
    float a, b, c;
    f2 p, q;
    double d, e;
    int u, v;
};

template <int KIND>
__device__ __forceinline__ void emit(Regs& r, float s) {
    if constexpr (KIND == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r.a) : "v"(r.b), "v"(r.c));
    if constexpr (KIND == FMAS) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(r.a) : "s"(s));
    if constexpr (KIND == ADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r.a) : "v"(r.b));
    if constexpr (KIND == MUL) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r.a) : "v"(r.b));
    if constexpr (KIND == MAX) asm volatile("v_max_f32 %0, %0, %1" : "+v"(r.a) : "v"(r.b));
    if constexpr (KIND == MED3) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(r.a) : "v"(r.b), "v"(r.c));
    if constexpr (KIND == MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(r.a) : "v"(r.b));
    if constexpr (KIND == ADDU) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r.u) : "v"(r.v));
    if constexpr (KIND == PKFMA) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(r.p) : "v"(r.q), "v"(r.q));
    if constexpr (KIND == PKADD) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r.p) : "v"(r.q));
    if constexpr (KIND == EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(r.a));
    if constexpr (KIND == FMA64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(r.d) : "v"(r.e), "v"(r.e));
    if constexpr (KIND == CNDM)
        asm volatile("v_cmp_gt_f32 vcc, %1, %2\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(r.a) : "v"(r.b), "v"(r.c) : "vcc");
}

constexpr int C = 8, U = 16;

template <int K1, int K2>
__global__ void __launch_bounds__(256) k(float* out, int iters, float s) {
    Regs r[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const float x = threadIdx.x * 1e-3f + j * 0.01f;
        r[j] = Regs{x, 0.999f, 0.25f, f2{x, -x}, f2{0.999f, 0.5f}, (double)x, 0.999, (int)threadIdx.x + j, 3};
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int uu = 0; uu < U; ++uu) {
#pragma unroll
            for (int j = 0; j < C; ++j) {
                if (j & 1) emit<K2>(r[j], s);
                else emit<K1>(r[j], s);
            }
        }
    }
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < C; ++j) t += r[j].a + r[j].p.x + (float)r[j].d + (float)r[j].u;
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int K1, int K2>
static float timed(int blocks, float* out, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<K1, K2>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL((k<K1, K2>), dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best;
}

static int g_cus;
static float* g_out;

template <int K1, int K2>
static void row(int iters) {
    const int ws[] = {1, 3, 8};
    printf("%-15s + %-15s", kName[K1], kName[K2]);
    for (int w : ws) {
        const float ms = timed<K1, K2>(g_cus * w, g_out, iters);
        // SIMD cycles per wave-instruction at 2.4 GHz (CNDM is a cmp + cndmask pair: 2 instructions)
        const double per_round = (C / 2) * ((K1 == CNDM ? 2 : 1) + (K2 == CNDM ? 2 : 1));
        const double winst = (double)iters * U * per_round;
        const double cyc = ms * 1e-3 * 2.4e9 / (w * winst);
        printf("  W=%d %7.3f ms %6.3f cyc", w, ms, cyc);
    }
    printf("\n");
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 1024;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    g_cus = prop.multiProcessorCount;
    (void)hipMalloc(&g_out, (size_t)g_cus * 8 * 256 * sizeof(float));
    printf("# SIMD cycles per wave64 instruction at 2.4 GHz (HIP-event time of the launch, %d CUs)\n", g_cus);
    row<FMA, FMA>(iters);
    row<FMAS, FMAS>(iters);
    row<ADD, ADD>(iters);
    row<MUL, MUL>(iters);
    row<MAX, MAX>(iters);
    row<MED3, MED3>(iters);
    row<MOV, MOV>(iters);
    row<ADDU, ADDU>(iters);
    row<PKFMA, PKFMA>(iters);
    row<PKADD, PKADD>(iters);
    row<EXP, EXP>(iters);
    row<FMA64, FMA64>(iters);
    row<CNDM, CNDM>(iters);
    row<FMA, ADD>(iters);
    row<FMA, MUL>(iters);
    row<FMA, MAX>(iters);
    row<FMA, MOV>(iters);
    row<FMA, ADDU>(iters);
    row<FMA, PKFMA>(iters);
    row<FMA, EXP>(iters);
    row<FMA, FMA64>(iters);
    row<PKFMA, EXP>(iters);
    row<PKFMA, ADD>(iters);
    row<FMA64, EXP>(iters);
    return 0;
}
