// Operand lane map of v_mfma_i32_16x16x64_i8 on gfx950, checked with exact
// integer data (asymmetric A and B): which K index does byte j (0..15) of lane
// l's A/B fragment hold?  Candidates:
//   H1: k = 16 (l >> 4) + j
//   H2: k = 8 (l >> 4) + j (j < 8), 32 + 8 (l >> 4) + (j - 8) (j >= 8)
// C/D: col = l & 15, row = 4 (l >> 4) + reg (the dtype-independent map).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_i8_layout.hip -o tools/micro/mfma_i8_layout
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int i4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline int kmap(int hyp, int l, int j) {
    return hyp == 1 ? 16 * (l >> 4) + j : (j < 8 ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + (j - 8));
}

__global__ void k(const signed char* A, const signed char* B, int* C, int hyp) {
    const int l = threadIdx.x;
    i4 a, b;
    signed char* pa = (signed char*)&a;
    signed char* pb = (signed char*)&b;
    for (int j = 0; j < 16; ++j) {
        const int kk = kmap(hyp, l, j);
        pa[j] = A[(l & 15) * 64 + kk];  // A[row][k]
        pb[j] = B[kk * 16 + (l & 15)];  // B[k][col]
    }
    i4 c = i4{0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
    signed char hA[16 * 64], hB[64 * 16];
    int ref[256], hC[256];
    srand(7);
    for (int i = 0; i < 16 * 64; ++i) hA[i] = (signed char)((rand() % 255) - 127);
    for (int i = 0; i < 64 * 16; ++i) hB[i] = (signed char)((rand() % 255) - 127);
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            int s = 0;
            for (int kk = 0; kk < 64; ++kk) s += hA[r * 64 + kk] * hB[kk * 16 + c];
            ref[r * 16 + c] = s;
        }
    signed char *dA, *dB;
    int* dC;
    (void)hipMalloc(&dA, sizeof hA);
    (void)hipMalloc(&dB, sizeof hB);
    (void)hipMalloc(&dC, sizeof hC);
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    for (int hyp = 1; hyp <= 2; ++hyp) {
        k<<<1, 64>>>(dA, dB, dC, hyp);
        (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
        printf("H%d: %d of 256 entries differ (C[0]=%d ref %d)\n", hyp, bad, hC[0], ref[0]);
    }
    return 0;
}
