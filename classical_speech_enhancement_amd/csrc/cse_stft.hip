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
constexpr int STFT_FPB = 4;
template <int NFFT>
__global__ void __launch_bounds__(256) stft_kernel(const double* __restrict__ x,
                                                   const double* __restrict__ x_sub,
                                                   int64_t len, int hop, int T,
                                                   float2* __restrict__ Y,
                                                   double* __restrict__ P) {
    constexpr int LOG2N = (NFFT == 512) ? 9 : 10;
    constexpr int B = NFFT / 2 + 1;
    constexpr int F = STFT_FPB;
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
    CSE_CHECK_ARG(n_fft == 512 || n_fft == 1024, "cse_stft: n_fft=%d (512|1024)", n_fft);
    CSE_CHECK_ARG(hop >= 1 && hop <= n_fft, "cse_stft: hop=%d", hop);
    const int T = n_frames_for(len, hop);
    dim3 grid((unsigned)ceil_div(T, STFT_FPB), (unsigned)n_sig);
    if (n_fft == 512)
        hipLaunchKernelGGL(stft_kernel<512>, grid, dim3(256), 0, (hipStream_t)stream, x, x_sub,
                           len, hop, T, (float2*)Y, P);
    else
        hipLaunchKernelGGL(stft_kernel<1024>, grid, dim3(256), 0, (hipStream_t)stream, x, x_sub,
                           len, hop, T, (float2*)Y, P);
    CSE_CHECK_LAUNCH("cse_stft");
    return CSE_OK;
}

extern "C" int cse_istft_norm(int n_fft, int hop, int64_t len, float* out, cse_stream_t stream) {
    CSE_CHECK_ARG(out != nullptr, "cse_istft_norm: out is NULL");
    CSE_CHECK_ARG(n_fft == 512 || n_fft == 1024, "cse_istft_norm: n_fft=%d", n_fft);
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
