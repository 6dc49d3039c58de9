// Checks the inline-assembly 4-byte LDS-DMA of cse_enhance.hip (glds4): every
// wave of a 256-thread block loads 64 floats into LDS at a wave-uniform byte
// base (M0) + 4 x lane, lanes of a partial exec mask only, then each lane reads
// back what its own wave loaded after s_waitcnt vmcnt(0).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/glds_check.hip -o tools/micro/glds_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void glds4(const float* src, unsigned char* dst) {
    const unsigned m = (unsigned)(uintptr_t)(lds_ptr_t)dst;
    int keep, base;
    asm volatile("v_readfirstlane_b32 %1, %3\n\ts_nop 4\n\ts_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "global_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep), "=&s"(base)
                 : "v"(src), "v"(m)
                 : "memory");
}

__global__ void k(const float* __restrict__ g, float* out, int* bad) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    for (int i = tid; i < 4096; i += 256) ((float*)smem)[i] = -1.0f;
    __syncthreads();
    glds4(g + 128 * wv + lane, smem + 1000 * 4 + 512 * wv);          // floats 1000 + 128 wv + lane
    glds4(g + 128 * wv + 64 + lane, smem + 1000 * 4 + 512 * wv + 256);
    if (wv == 0 && lane < 2) glds4(g + 512 + lane, smem + 1000 * 4 + 2048);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float* f = (const float*)(smem + 4000);
    int nb = 0;
    for (int u = 0; u < 2; ++u) {
        const int i = 128 * wv + 2 * lane + u;  // a float this wave loaded
        if (f[i] != g[i]) ++nb;
    }
    if (wv == 0 && lane < 2 && f[512 + lane] != g[512 + lane]) ++nb;
    out[tid] = f[2 * tid];
    if (nb) atomicAdd(bad, nb);
}

int main() {
    float *g, *out;
    int* bad;
    (void)hipMalloc(&g, 1024 * 4);
    (void)hipMalloc(&out, 256 * 4);
    (void)hipMalloc(&bad, 4);
    float h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = 1.0f + i;
    (void)hipMemcpy(g, h, sizeof(h), hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 16384, 0, g, out, bad);
    int hb = -1;
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    float ho[256];
    (void)hipMemcpy(ho, out, sizeof(ho), hipMemcpyDeviceToHost);
    printf("glds4 mismatches: %d  (out[0..4] = %g %g %g %g, expect 1 3 5 7)\n", hb, ho[0], ho[1], ho[2], ho[3]);
    return hb != 0;
}
