// Batched centred STFT (fp64) and ISTFT normalisation tables.
//
// Replaces librosa.stft at spectral_subtractor.py:25, wiener_filter.py:35,
// mmse.py:29, advanced_mmse.py:39, noise_estimation.py:184-188 and :136-144
// (window="hann", center=True, pad_mode="reflect", win_length=n_fft), and the
// window-sum-square normalisation inside librosa.istft.
//
// The analysis runs in fp64: it is <0.5 % of the grid's work, and an exact P
// keeps the percentile estimator's frame ranking (noise_estimation.py:44-47)
// identical to the fp64 reference.  Y is stored complex64 for the hot path.
#include "cse_common.hpp"

namespace cse {

// index of np.pad(x, (h, h), mode='reflect') applied repeatedly
__device__ __forceinline__ int64_t reflect_index(int64_t p, int64_t len) {
    if (len == 1) return 0;
    const int64_t period = 2 * (len - 1);
    int64_t q = p % period;
    if (q < 0) q += period;
    return q < len ? q : period - q;
}

// One workgroup per FPB consecutive frames of one signal.  Radix-2 DIT FFT in
// LDS, fp64; the twiddles and the window are computed once per workgroup and
// shared by its frames (r03: they were recomputed per frame, one fp64
// sincospi / cospi per point), and only frames that reach past either end of
// the signal take the 64-bit reflect arithmetic.  Every element sees the same
// operations as before, so Y and P are bit-identical to the one-frame form.
// (n_fft 2048 / 4096, r06: one frame per workgroup)
constexpr int STFT_FPB = 4;
__host__ __device__ constexpr int stft_fpb(int nfft) { return nfft > 1024 ? 1 : STFT_FPB; }
template <int NFFT>
__global__ void __launch_bounds__(256) stft_kernel(const double* __restrict__ x,
                                                   const double* __restrict__ x_sub,
                                                   int64_t len, int hop, int T,
                                                   float2* __restrict__ Y,
                                                   double* __restrict__ P) {
    constexpr int LOG2N = __builtin_ctz(NFFT);
    constexpr int B = NFFT / 2 + 1;
    constexpr int F = stft_fpb(NFFT);
    __shared__ double re[F][NFFT], im[F][NFFT];
    __shared__ double twr[NFFT / 2], twi[NFFT / 2], win[NFFT];
    const int tb = blockIdx.x * F;
    const int nfr = min(F, T - tb);
    const int64_t sig = blockIdx.y;
    const double* xs = x + sig * len;
    const double* xd = x_sub ? x_sub + sig * len : nullptr;
    for (int k = threadIdx.x; k < NFFT / 2; k += blockDim.x) {
        double sn, c;
        sincospi(-2.0 * (double)k / (double)NFFT, &sn, &c);
        twr[k] = c;
        twi[k] = sn;
    }
    for (int n = threadIdx.x; n < NFFT; n += blockDim.x)
        win[n] = 0.5 - 0.5 * cospi(2.0 * (double)n / (double)NFFT);
    __syncthreads();
    // load the frames of the reflect-padded signal, windowed, in bit-reversed order
    for (int f = 0; f < nfr; ++f) {
        const int64_t p0 = (int64_t)(tb + f) * hop - NFFT / 2;
        const bool inside = p0 >= 0 && p0 + NFFT <= len;  // uniform per frame
        for (int n = threadIdx.x; n < NFFT; n += blockDim.x) {
            const int64_t p = p0 + n;
            const int64_t si = inside ? p : reflect_index(p, len);
            double v = xs[si];
            if (xd) v = v - xd[si];
            const int r = (int)(__brev((unsigned)n) >> (32 - LOG2N));
            re[f][r] = v * win[n];
            im[f][r] = 0.0;
        }
    }
    __syncthreads();
    for (int st = 1; st <= LOG2N; ++st) {
        const int half = 1 << (st - 1);
        for (int e = threadIdx.x; e < nfr * (NFFT / 2); e += blockDim.x) {
            const int f = e / (NFFT / 2), b = e % (NFFT / 2);
            const int grp = b >> (st - 1);
            const int j = b & (half - 1);
            const int i0 = grp * (half << 1) + j;
            const int i1 = i0 + half;
            const int tw = j << (LOG2N - st);
            const double wr = twr[tw], wi = twi[tw];
            const double br = re[f][i1] * wr - im[f][i1] * wi;
            const double bi = re[f][i1] * wi + im[f][i1] * wr;
            const double ar = re[f][i0], ai = im[f][i0];
            re[f][i0] = ar + br;
            im[f][i0] = ai + bi;
            re[f][i1] = ar - br;
            im[f][i1] = ai - bi;
        }
        __syncthreads();
    }
    for (int f = 0; f < nfr; ++f) {
        const int64_t row = (sig * T + tb + f) * (int64_t)B;
        for (int k = threadIdx.x; k < B; k += blockDim.x) {
            double r = re[f][k], i = im[f][k];
            if (k == 0 || k == NFFT / 2) i = 0.0;  // pocketfft r2c: exact zero imag
            if (Y) Y[row + k] = make_float2((float)r, (float)i);
            if (P) P[row + k] = r * r + i * i;
        }
    }
}

// ---------------------------------------------------------------------------
// n_fft = 512 (r03): the real transform as a complex 256-point FFT of
// z[m] = xw[2m] + i xw[2m+1], factored 16 x 16 in registers, fp64.  16 lanes
// per frame (4 frames per wavefront, 16 per workgroup): lane m2 holds
// z[16 m1 + m2], m1 < 16, takes the DFT16 over m1, the twiddles W256^{m2 k1},
// and the LDS transpose hands lane k1 the column k1; the second DFT16 gives
// Z[k1 + 16 k2].  The split X[k] = (Z_k + conj Z_{M-k})/2 +
// W512^k (Z_k - conj Z_{M-k})/(2i) reads the mirror through LDS.  Every
// exchange stays inside the frame's wavefront (no block barrier after the
// tables); ~95 LDS accesses per lane and frame where the radix-2 form made
// 9 passes over the frame.  Results differ from the radix-2 form in the
// last bits only (fp64 either way; neither is pocketfft's order).
// ---------------------------------------------------------------------------
struct __attribute__((aligned(16))) dcx {
    double x, y;
};
__device__ __forceinline__ dcx dmk(double x, double y) { return dcx{x, y}; }
__device__ __forceinline__ dcx dadd(dcx a, dcx b) { return dcx{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ dcx dsub(dcx a, dcx b) { return dcx{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ dcx dmul(dcx a, dcx b) {
    return dcx{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}

// forward DFT4 (e^{-2πi nk/4}) in place
__device__ __forceinline__ void fdft4(dcx& a0, dcx& a1, dcx& a2, dcx& a3) {
    const dcx s02 = dadd(a0, a2), d02 = dsub(a0, a2);
    const dcx s13 = dadd(a1, a3), t = dsub(a1, a3);
    const dcx d13 = dmk(t.y, -t.x);  // -i (a1 - a3)
    a0 = dadd(s02, s13);
    a2 = dsub(s02, s13);
    a1 = dadd(d02, d13);
    a3 = dsub(d02, d13);
}

// W16^m = e^{-2πi m/16}, m in [0, 9]
__device__ __forceinline__ dcx fw16(int m) {
    constexpr double c1 = 0.92387953251128674, s1 = 0.38268343236508978;
    constexpr double r2 = 0.70710678118654752;
    switch (m) {
        case 0: return dcx{1.0, 0.0};
        case 1: return dcx{c1, -s1};
        case 2: return dcx{r2, -r2};
        case 3: return dcx{s1, -c1};
        case 4: return dcx{0.0, -1.0};
        case 5: return dcx{-s1, -c1};
        case 6: return dcx{-r2, -r2};
        case 7: return dcx{-c1, -s1};
        case 8: return dcx{-1.0, 0.0};
        default: return dcx{-c1, s1};  // 9
    }
}

// forward DFT16, natural order in and out: n = 4a + b, k = c + 4d
__device__ __forceinline__ void fdft16(dcx (&v)[16]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) fdft4(v[b], v[4 + b], v[8 + b], v[12 + b]);  // -> v[b + 4c]
#pragma unroll
    for (int b = 1; b < 4; ++b)
#pragma unroll
        for (int c = 1; c < 4; ++c) v[b + 4 * c] = dmul(v[b + 4 * c], fw16(b * c));
#pragma unroll
    for (int c = 0; c < 4; ++c) fdft4(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]);  // v[4c + d]
    dcx t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 4; ++d) t[c + 4 * d] = v[4 * c + d];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int S512_FPB = 16;  // frames per workgroup (4 per wavefront)
__global__ void __launch_bounds__(256) stft512_kernel(const double* __restrict__ x,
                                                      const double* __restrict__ x_sub,
                                                      int64_t len, int hop, int T,
                                                      float2* __restrict__ Y,
                                                      double* __restrict__ P) {
    constexpr int M = 256, NF = 512, B = 257;
    __shared__ dcx buf[S512_FPB][M + 16];  // +16: the transposed reads of 16 lanes spread banks
    __shared__ dcx tw256[M], tw512[M];
    __shared__ double win[NF];
    const int tid = threadIdx.x;
    for (int k = tid; k < M; k += blockDim.x) {
        double sn, c;
        sincospi(-2.0 * (double)k / 256.0, &sn, &c);
        tw256[k] = dmk(c, sn);
        sincospi(-2.0 * (double)k / 512.0, &sn, &c);
        tw512[k] = dmk(c, sn);
    }
    for (int n = tid; n < NF; n += blockDim.x) win[n] = 0.5 - 0.5 * cospi(2.0 * (double)n / 512.0);
    __syncthreads();
    const int fl = tid >> 4, lane = tid & 15;  // frame slot, lane in the frame
    const int t = blockIdx.x * S512_FPB + fl;
    if (t >= T) return;  // whole 16-lane groups; no block barrier below
    const int64_t sig = blockIdx.y;
    const double* xs = x + sig * len;
    const double* xd = x_sub ? x_sub + sig * len : nullptr;
    const int64_t p0 = (int64_t)t * hop - NF / 2;
    const bool inside = p0 >= 0 && p0 + NF <= len;
    dcx* fb = buf[fl];
    // pass 1: lane m2 = lane loads z[16 m1 + m2] = xw[32 m1 + 2 m2 + (0, 1)]
    dcx v[16];
#pragma unroll
    for (int m1 = 0; m1 < 16; ++m1) {
        const int n = 32 * m1 + 2 * lane;
        const int64_t pa = p0 + n, pb = pa + 1;
        const int64_t ia = inside ? pa : reflect_index(pa, len);
        const int64_t ib = inside ? pb : reflect_index(pb, len);
        double a = xs[ia], b = xs[ib];
        if (xd) {
            a -= xd[ia];
            b -= xd[ib];
        }
        v[m1] = dmk(a * win[n], b * win[n + 1]);
    }
    fdft16(v);  // v[k1], column m2 = lane
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = dmul(v[k1], tw256[(lane * k1) & (M - 1)]);
    // transpose: entry (m2, k1) at fb[k1 * 17 + m2]
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) fb[k1 * 17 + lane] = v[k1];
    wave_lds_sync();
#pragma unroll
    for (int m2 = 0; m2 < 16; ++m2) v[m2] = fb[lane * 17 + m2];
    fdft16(v);  // v[k2] = Z[k1 + 16 k2], k1 = lane
    wave_lds_sync();
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) fb[lane + 16 * k2] = v[k2];  // natural index k
    wave_lds_sync();
    const int64_t row = (sig * T + t) * (int64_t)B;
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
        const int k = lane + 16 * k2;
        const dcx z = v[k2];
        const dcx w = fb[(M - k) & (M - 1)];  // Z_{M-k} (Z_0 for k = 0)
        // E = (z + conj w)/2, O = (z - conj w)/(2i)
        const dcx e = dmk(0.5 * (z.x + w.x), 0.5 * (z.y - w.y));
        const dcx o = dmk(0.5 * (z.y + w.y), -0.5 * (z.x - w.x));
        dcx X = dadd(e, dmul(tw512[k], o));
        if (k == 0) X = dmk(z.x + z.y, 0.0);  // X_0 = Re Z_0 + Im Z_0, exact zero imag
        if (Y) Y[row + k] = make_float2((float)X.x, (float)X.y);
        if (P) P[row + k] = X.x * X.x + X.y * X.y;
    }
    if (lane == 0) {  // Nyquist: X_256 = Re Z_0 - Im Z_0
        const double r = v[0].x - v[0].y;
        if (Y) Y[row + 256] = make_float2((float)r, 0.0f);
        if (P) P[row + 256] = r * r;
    }
}

// Even n_fft that is not a power of two (e.g. 400, r06): the direct real DFT
// X_k = sum_n xw[n] e^{-2πi kn/N}, fp64, one workgroup per frame, the windowed
// frame and the N twiddles e^{-2πi m/N} in LDS (index kn mod N).  O(N B) per
// frame where the radix-2 forms are O(N log N): the shapes the grids never use.
constexpr int DFT_NMAX = 4096;
__global__ void __launch_bounds__(256) stft_dft_kernel(const double* __restrict__ x,
                                                       const double* __restrict__ x_sub,
                                                       int64_t len, int N, int hop, int T,
                                                       float2* __restrict__ Y,
                                                       double* __restrict__ P) {
    __shared__ double xw[DFT_NMAX], twr[DFT_NMAX], twi[DFT_NMAX];
    const int t = blockIdx.x;
    const int64_t sig = blockIdx.y;
    const int B = N / 2 + 1;
    const double* xs = x + sig * len;
    const double* xd = x_sub ? x_sub + sig * len : nullptr;
    const int64_t p0 = (int64_t)t * hop - N / 2;
    for (int n = threadIdx.x; n < N; n += blockDim.x) {
        double sn, c;
        sincospi(-2.0 * (double)n / (double)N, &sn, &c);
        twr[n] = c;
        twi[n] = sn;
        const int64_t si = reflect_index(p0 + n, len);
        double v = xs[si];
        if (xd) v = v - xd[si];
        xw[n] = v * (0.5 - 0.5 * cospi(2.0 * (double)n / (double)N));
    }
    __syncthreads();
    const int64_t row = (sig * T + t) * (int64_t)B;
    for (int k = threadIdx.x; k < B; k += blockDim.x) {
        double r = 0.0, i = 0.0;
        int m = 0;  // k n mod N
        for (int n = 0; n < N; ++n) {
            r = fma(xw[n], twr[m], r);
            i = fma(xw[n], twi[m], i);
            m += k;
            if (m >= N) m -= N;
        }
        if (k == 0 || k == N / 2) i = 0.0;  // pocketfft r2c: exact zero imag
        if (Y) Y[row + k] = make_float2((float)r, (float)i);
        if (P) P[row + k] = r * r + i * i;
    }
}

// 1/wss for output sample o (padded position o + n_fft/2); 1 where wss <= DBL_MIN
__global__ void istft_norm_kernel(int n_fft, int hop, int64_t len, int nf, float* out) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= len) return;
    const int64_t p = o + n_fft / 2;
    int64_t t_lo = (p - n_fft + 1 + hop - 1) / hop;
    if (p - n_fft + 1 <= 0) t_lo = 0;
    int64_t t_hi = p / hop;
    if (t_hi > nf - 1) t_hi = nf - 1;
    double wss = 0.0;
    for (int64_t t = t_lo; t <= t_hi; ++t) {
        const int64_t n = p - t * hop;
        const double w = 0.5 - 0.5 * cospi(2.0 * (double)n / (double)n_fft);
        wss += w * w;
    }
    out[o] = (wss > 2.2250738585072014e-308) ? (float)(1.0 / wss) : 1.0f;
}

}  // namespace cse

using namespace cse;

extern "C" int cse_stft(const double* x, const double* x_sub, int64_t n_sig, int64_t len,
                        int n_fft, int hop, float* Y, double* P, cse_stream_t stream) {
    CSE_CHECK_ARG(x != nullptr, "cse_stft: x is NULL");
    CSE_CHECK_ARG(n_sig > 0 && n_sig < 65536, "cse_stft: n_sig=%lld out of range", (long long)n_sig);
    CSE_CHECK_ARG(len >= 1, "cse_stft: len=%lld", (long long)len);
    CSE_CHECK_ARG(n_fft >= 64 && n_fft <= 4096 && n_fft % 2 == 0,
                  "cse_stft: n_fft=%d (even, in [64, 4096])", n_fft);
    CSE_CHECK_ARG(hop >= 1 && hop <= n_fft, "cse_stft: hop=%d", hop);
    const int T = n_frames_for(len, hop);
    dim3 grid((unsigned)ceil_div(T, stft_fpb(n_fft)), (unsigned)n_sig);
    hipStream_t st = (hipStream_t)stream;
    if (n_fft & (n_fft - 1)) {  // even, not a power of two: the direct DFT
        hipLaunchKernelGGL(stft_dft_kernel, dim3((unsigned)T, (unsigned)n_sig), dim3(256), 0, st, x,
                           x_sub, len, n_fft, hop, T, (float2*)Y, P);
        CSE_CHECK_LAUNCH("cse_stft");
        return CSE_OK;
    }
    switch (n_fft) {  // 512: its own register-resident form; the rest radix 2 in LDS
        case 512:
            hipLaunchKernelGGL(stft512_kernel, dim3((unsigned)ceil_div(T, S512_FPB), (unsigned)n_sig),
                               dim3(256), 0, st, x, x_sub, len, hop, T, (float2*)Y, P);
            break;
        case 1024:
            hipLaunchKernelGGL(stft_kernel<1024>, grid, dim3(256), 0, st, x, x_sub, len, hop, T,
                               (float2*)Y, P);
            break;
        case 64:
            hipLaunchKernelGGL(stft_kernel<64>, grid, dim3(256), 0, st, x, x_sub, len, hop, T,
                               (float2*)Y, P);
            break;
        case 128:
            hipLaunchKernelGGL(stft_kernel<128>, grid, dim3(256), 0, st, x, x_sub, len, hop, T,
                               (float2*)Y, P);
            break;
        case 256:
            hipLaunchKernelGGL(stft_kernel<256>, grid, dim3(256), 0, st, x, x_sub, len, hop, T,
                               (float2*)Y, P);
            break;
        case 2048:
            hipLaunchKernelGGL(stft_kernel<2048>, grid, dim3(256), 0, st, x, x_sub, len, hop, T,
                               (float2*)Y, P);
            break;
        default:  // 4096
            hipLaunchKernelGGL(stft_kernel<4096>, grid, dim3(256), 0, st, x, x_sub, len, hop, T,
                               (float2*)Y, P);
            break;
    }
    CSE_CHECK_LAUNCH("cse_stft");
    return CSE_OK;
}

extern "C" int cse_istft_norm(int n_fft, int hop, int64_t len, float* out, cse_stream_t stream) {
    CSE_CHECK_ARG(out != nullptr, "cse_istft_norm: out is NULL");
    CSE_CHECK_ARG(n_fft >= 64 && n_fft <= 4096 && n_fft % 2 == 0, "cse_istft_norm: n_fft=%d",
                  n_fft);
    CSE_CHECK_ARG(hop >= 1 && hop <= n_fft && len >= 1, "cse_istft_norm: hop=%d len=%lld", hop,
                  (long long)len);
    const int T = n_frames_for(len, hop);
    const int64_t need = (len + n_fft + hop - 1) / hop;  // ceil((len + 2*(n_fft/2)) / hop)
    const int nf = (int)(need < T ? need : T);
    hipLaunchKernelGGL(istft_norm_kernel, dim3(ceil_div(len, 256)), dim3(256), 0,
                       (hipStream_t)stream, n_fft, hop, len, nf, out);
    CSE_CHECK_LAUNCH("cse_istft_norm");
    return CSE_OK;
}
