// Is r1 = fma(fma(-x, r, 1), r, r), r = v_rcp_f32(x), the correctly rounded
// f32 reciprocal (== 1.0f / x, IEEE) for every positive normal x in
// [2^-60, 2^60]?  Counts mismatches over all such x (finish_kernel's inversion
// of noise rows, x = max(N, eps) with eps >= 1e-12).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/rcp_check.hip -o tools/micro/rcp_check
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void check(unsigned lo, unsigned n, unsigned long long* bad, unsigned* first) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned bits = lo + i;
    const float x = __builtin_bit_cast(float, bits);
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    const float r1 = __builtin_fmaf(e, r, r);
    const float ref = 1.0f / x;
    if (__builtin_bit_cast(unsigned, r1) != __builtin_bit_cast(unsigned, ref)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, bits);
    }
}

int main() {
    // exponents -60 .. 60: biased 67 .. 187
    const unsigned lo = 67u << 23, hi = 188u << 23, n = hi - lo;
    unsigned long long* bad;
    unsigned* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 4);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0xff, 4);
    hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, lo, n, bad, first);
    unsigned long long hb = 0;
    unsigned hf = 0;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    printf("values %u  mismatches %llu  first bits 0x%08x (%g)\n", n, hb, hf,
           hb ? (double)__builtin_bit_cast(float, hf) : 0.0);
    return hb ? 1 : 0;
}
