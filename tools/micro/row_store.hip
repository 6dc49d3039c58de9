// Store rate of the noise-row shape: one thread per (row, bin), a loop over T
// frames writing one float per frame at row stride S floats (257 bins, S = 257
// as the pool lays rows out, or padded), 1,400 rows x 1,251 frames.  Also the
// same rows with a serial fp64 recurrence per frame (finish_kernel's shape).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/row_store.hip -o tools/micro/row_store
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool REC>
__global__ void __launch_bounds__(256) rows(float* out, int64_t n_items, int B, int S, int T, float mu) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n_items) return;
    const int64_t row = idx / B;
    const int b = (int)(idx - row * B);
    float* o = out + row * (int64_t)T * S + b;
    double s = 1.0 + b;
    for (int t = 0; t < T; ++t) {
        if (REC) s = (double)mu * s + 0.01;
        o[(int64_t)t * S] = REC ? (float)s : (float)t;
    }
}

// tiled: a workgroup per row computes F frames of every bin into LDS, then
// the workgroup writes the F x B block (contiguous in memory) with
// consecutive dword stores: each wave sweeps contiguous bytes
template <int F>
__global__ void __launch_bounds__(256) rows_tiled(float* out, int B, int T, float mu) {
    __shared__ float tile[F * 260];
    const int64_t row = blockIdx.x;
    float* o = out + row * (int64_t)T * B;
    double s[2];
    for (int u = 0; u < 2; ++u) s[u] = 1.0 + threadIdx.x + 256 * u;
    for (int t0 = 0; t0 < T; t0 += F) {
        const int nf = min(F, T - t0);
        for (int u = 0; u < 2; ++u) {
            const int b = threadIdx.x + 256 * u;
            if (b < B)
                for (int f = 0; f < nf; ++f) {
                    s[u] = (double)mu * s[u] + 0.01;
                    tile[f * B + b] = (float)s[u];
                }
        }
        __syncthreads();
        float* dst = o + (int64_t)t0 * B;
        for (int i = threadIdx.x; i < nf * B; i += 256) dst[i] = tile[i];
        __syncthreads();
    }
}

int main() {
    const int B = 257, T = 1251, R = 1400;
    float* out;
    hipMalloc(&out, (size_t)R * T * 320 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int S : {257, 260, 288, 320}) {
        for (int rec = 0; rec < 2; ++rec) {
            const int64_t n = (int64_t)R * B;
            float best = 1e9f;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(e0);
                if (rec)
                    hipLaunchKernelGGL(rows<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, out, n, B, S, T, 0.98f);
                else
                    hipLaunchKernelGGL(rows<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, out, n, B, S, T, 0.98f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            const double bytes = (double)R * T * B * 4;
            printf("stride %3d floats  %s  %.3f ms  %.2f TB/s (useful bytes)\n", S, rec ? "fp64 recurrence" : "plain stores   ",
                   best, bytes / best / 1e9);
        }
    }
    for (int F : {8, 16, 32}) {
        float best = 1e9f;
        for (int rep = 0; rep < 4; ++rep) {
            hipEventRecord(e0);
            if (F == 8) hipLaunchKernelGGL(rows_tiled<8>, dim3(R), dim3(256), 0, 0, out, B, T, 0.98f);
            if (F == 16) hipLaunchKernelGGL(rows_tiled<16>, dim3(R), dim3(256), 0, 0, out, B, T, 0.98f);
            if (F == 32) hipLaunchKernelGGL(rows_tiled<32>, dim3(R), dim3(256), 0, 0, out, B, T, 0.98f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        const double bytes = (double)R * T * B * 4;
        printf("tiled F=%2d        fp64 recurrence  %.3f ms  %.2f TB/s (useful bytes)\n", F, best, bytes / best / 1e9);
    }
    return 0;
}
