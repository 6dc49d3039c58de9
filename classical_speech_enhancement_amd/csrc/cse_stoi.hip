// STOI (short-time objective intelligibility) of many enhanced outputs against
// their clean references — the score the reference's sweep optimises
// (evaluation_metrics.py:30-36: pystoi 0.4.1 `stoi(clean, enhanced, sr,
// extended=False)`, called per grid cell at speech_enhancement_comparison.py:180
// after finalize_enhanced :92-106).  Restated from the published algorithm
// (Taal et al. 2011, as implemented by pystoi 0.4.1; oracle/stoi_ref.py):
//
//   resample 16 kHz -> 10 kHz   Octave `resample` filter (Kaiser sinc, 581 taps
//                               at the 5x upsampled rate) through resample_poly:
//                               e10[5q + r] = sum_k c_r[k] e[8q + k], k in [-58, 64]
//   silent frames               256-sample MATLAB-Hann frames at hop 128 of the
//                               CLEAN signal more than 40 dB below its loudest
//                               are dropped in both signals; the kept frames
//                               are overlap-added back (frame k of the kept
//                               list lands at 128 k)
//   STFT                        256-sample frames of that signal at hop 128,
//                               MATLAB-Hann, 512-point rfft
//   bands                       15 one-third-octave bands (bins [7, 219)):
//                               env = sqrt(sum_band |X|^2)
//   segments                    30 frames: y scaled to x's norm, clipped at
//                               x (1 + 10^(15/20)), both mean-removed and
//                               normalised, correlated; mean over bands and
//                               segments.  Fewer than 30 frames -> 1e-5.
//
// The clean side (resampled clean in fp64, silent-frame mask, kept-frame list,
// band envelopes and segment statistics) is prepared once per signal
// (cse_stoi_prepare).  Per cell one workgroup (stoi_cells_kernel):
//   phase A  blocks of 16 STFT frames: stage the needed 16-kHz samples in LDS,
//            polyphase-resample the distinct 128-sample 10-kHz half-blocks the
//            block's overlap-add needs (one thread = 5 outputs of one phase
//            group, coefficients from the scalar cache), overlap-add, window,
//            512-point real FFT as a 256-point complex DFT16 x DFT16 over 16
//            lanes per frame (LDS transpose one component at a time), band
//            energies -> envelope rows in a scratch buffer;
//   phase B  tiles of 64 segments x 15 bands from LDS, one (segment, band)
//            correlation per thread, fp64 accumulation.
// All arithmetic is fp64, like the reference: STOI normalises every band of
// every 30-frame segment separately, so a band that holds only a noise floor
// turns an fp32 FFT's roundoff (~1e-7 of the frame energy) into a visible
// score error (measured: 1e-5 STOI on a synthetic pair).  The 16-kHz cell
// outputs themselves are f32 (the enhance kernel's output type).
#include "cse_common.hpp"

#include <math.h>
#include <numeric>
#include <type_traits>

namespace cse {

namespace stoi {
constexpr int UP = 5, DOWN = 8;          // 10 kHz / 16 kHz
constexpr int HALF_LEN = 290;            // (581 - 1) / 2
constexpr int KLO = -58, KN = 123;       // tap span of the 5 phases: k in [-58, 64]
constexpr int CST = 128;                 // coefficient row stride
constexpr int FR = 256, HOP = 128;       // frames at 10 kHz
constexpr int NBAND = 15, NSEG = 30;
constexpr int FB = 16;                   // most STFT frames per phase-A block
// most distinct 10-kHz half-blocks per block: 16 consecutive kept frames need
// 17, so only blocks around dropped frames hold fewer than FB frames (r05: 28
// before; 4,096 cells 4.35 / 4.44 -> 4.24 / 4.31 ms, profiles/r05_ab_stoi_maxd.txt.
// Staging the samples as f64 instead, converted once rather than by each
// phase group, measured 4.94 / 4.99 ms: not kept)
constexpr int MAXD = 18;
// block table (ints): D, j0, nf, p[MAXD], sa[FB + 1], sb[FB + 1].  A block takes
// frames while nf <= FB and its OLA rows need <= MAXD distinct half-blocks
// (a row needs at most 2, so every block but the last holds >= MINF = 8 frames)
constexpr int T_D = 0, T_J0 = 1, T_NF = 2, T_P = 3, T_SA = T_P + MAXD, T_SB = T_SA + FB + 1;
constexpr int BT = 72;
static_assert(T_SB + FB + 1 <= BT, "block table size");
constexpr int MINF = MAXD / 2 - 1;       // frames every block but the last holds
constexpr int META = 8;                  // ints per signal: K, M, J, ok, nblk
constexpr int SLOTS = 9;                 // half-blocks resampled per pass (9 x 27 tasks <= 256)
constexpr int GRP = 27;                  // phase groups (5 outputs) covering one half-block
// staging (r05): the slot's samples in order, st[uu], so a phase group's 8
// samples of one tap block are 32 contiguous, aligned bytes: two ds_read_b128
// instead of eight ds_read_b32 per block (the slot stride a multiple of 16 B).
// 4,096 10-s cells, two alternating rounds: 4.55 / 4.50 -> 4.24 / 4.30 ms
// against r04's 8 rows by sample mod 8 (43 columns, slot stride 347 = 27 mod 64
// so that the slots sharing a wave did not collide; r06 removed that layout).
// Slot strides 348 / 352 / 360 and blocks padded to 12 floats measured no
// faster.
constexpr int SSTR = 344;  // floats per staged slot
static_assert(SSTR >= 8 * (GRP + 15) + 8 && SSTR % 4 == 0, "staging slot stride");
// (r03's opt-in i8-sliced resampler on the matrix pipe, level with this fp64 FIR
// at best, left the product in r04: tools/stoi_mf.md says how to rebuild it)
constexpr int STAGE_F = SLOTS * SSTR;
constexpr int NT = 256;                  // threads per workgroup
constexpr double EPS = 2.220446049250313e-16; // np.finfo(float).eps
__constant__ int BAND_EDGE[NBAND + 1] = {7, 9, 11, 14, 17, 22, 27, 34, 43, 55,
                                         69, 87, 109, 138, 174, 219};
}  // namespace stoi

constexpr int stoi_fs10 = 10000;  // pystoi's working rate

struct StoiLayout {
    int64_t n10, F, Mmax, Jmax, NBLK;
    int64_t coef64, meta, x10, en, kf, btab, xtob, xstat, hgen, total;
};

static inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// Input rates other than 16 kHz: pystoi resamples any fs_sig != 10 kHz with
// utils.resample_oct(x, 10000, fs_sig), scipy's resample_poly(x, up, down)
// with Octave's Kaiser window normalised to unit sum (oracle/stoi_ref.py
// resample_oct).  The filter and resample_poly's padding, per rate:
struct Resamp {
    int up, down;             // 10000 / sr reduced; 1 / 1 at 10 kHz (no resampling)
    int64_t half;             // window half length L: 2L + 1 taps
    int64_t pre_pad, pre_rm;  // resample_poly's leading zero taps and dropped outputs
    int64_t n_out;            // ceil(len up / down)
};

static Resamp resamp_for(int sr, int64_t len) {
    Resamp r;
    if (sr == stoi_fs10) {
        r.up = r.down = 1;
        r.half = r.pre_pad = r.pre_rm = 0;
        r.n_out = len;
        return r;
    }
    const int g = std::gcd(stoi_fs10, sr);
    r.up = stoi_fs10 / g;
    r.down = sr / g;
    // _resample_window_oct: stopband 1/(2 max(p, q)), roll-off a tenth of it,
    // L = ceil((60 - 8) / (28.714 roll-off)) (rejection 60 dB)
    const double stop = 1.0 / (2.0 * (double)(r.up > r.down ? r.up : r.down));
    r.half = (int64_t)ceil((60.0 - 8.0) / (28.714 * (stop / 10.0)));
    r.n_out = (len * r.up + r.down - 1) / r.down;
    r.pre_pad = r.down - r.half % r.down;
    r.pre_rm = (r.half + r.pre_pad) / r.down;
    return r;
}

static StoiLayout stoi_layout(int64_t n_sig, int64_t len, int sr = 16000) {
    using namespace stoi;
    StoiLayout L;
    int64_t ntap = 0;  // the generic filter (other rates)
    if (sr == 16000) {
        L.n10 = (len * UP + DOWN - 1) / DOWN;  // resample_poly: ceil(len * up / down)
    } else {
        const Resamp r = resamp_for(sr, len);
        L.n10 = r.n_out;
        ntap = 2 * r.half + 1;
    }
    L.F = L.n10 >= FR ? (L.n10 - FR) / HOP + 1 : 0;
    L.Mmax = L.F > 1 ? L.F - 1 : 0;
    L.Jmax = L.Mmax >= NSEG ? L.Mmax - NSEG + 1 : 0;
    L.NBLK = (L.Mmax + MINF - 1) / MINF + 1;
    int64_t o = 0;
    L.coef64 = o; o = align256(o + 5 * CST * 8);
    L.meta = o;   o = align256(o + n_sig * META * 4);
    L.x10 = o;    o = align256(o + n_sig * L.n10 * 8);
    L.en = o;     o = align256(o + n_sig * L.F * 8);
    L.kf = o;     o = align256(o + n_sig * L.F * 4);
    L.btab = o;   o = align256(o + n_sig * L.NBLK * BT * 4);
    L.xtob = o;   o = align256(o + n_sig * L.Mmax * 16 * 8);
    L.xstat = o;  o = align256(o + n_sig * L.Jmax * 16 * 32);
    L.hgen = o;   o = align256(o + ntap * 8);
    L.total = o;
    return L;
}

// ---------------------------------------------------------------------------
// prepare 1: the resampling filter (pystoi utils._resample_window_oct for
// p = 5, q = 8, normalised to unit sum, times up = 5 as resample_poly does),
// laid out by phase: c_r[k] = 5 hn[290 + 8r - 5k] for |8r - 5k| <= 290.
// ---------------------------------------------------------------------------
__device__ double bessel_i0(double x) {
    // power series; x <= 5.7 here, 40 terms reach full double precision
    const double q = 0.25 * x * x;
    double term = 1.0, sum = 1.0;
    for (int j = 1; j < 60; ++j) {
        term *= q / ((double)j * (double)j);
        sum += term;
        if (term < 1e-18 * sum) break;
    }
    return sum;
}

__global__ void __launch_bounds__(1024) stoi_coef_kernel(double* coef64) {
    using namespace stoi;
    __shared__ double h[2 * HALF_LEN + 1];
    __shared__ double red[1024];
    const int tid = threadIdx.x;
    const double beta = 0.1102 * (60.0 - 8.7);  // rejection 60 dB
    const double i0b = bessel_i0(beta);
    double part = 0.0;
    for (int i = tid; i < 2 * HALF_LEN + 1; i += 1024) {
        const double a = (double)HALF_LEN;
        const double u = ((double)i - a) / a;
        const double kais = bessel_i0(beta * sqrt(1.0 - u * u)) / i0b;
        const double t = (double)(i - HALF_LEN);
        const double x = t / 8.0;  // 2 * stopband_cutoff * t, cutoff = 1/16
        const double sinc = (i == HALF_LEN) ? 1.0 : sinpi(x) / (M_PI * x);
        h[i] = kais * (2.0 * UP / 16.0) * sinc;
        part += h[i];
    }
    red[tid] = part;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double total = red[0];
    for (int i = tid; i < 5 * CST; i += 1024) {
        const int r = i / CST, kk = i % CST;
        const int d = 8 * r - 5 * (kk + KLO);
        double v = 0.0;
        if (kk < KN && d >= -HALF_LEN && d <= HALF_LEN) v = UP * h[HALF_LEN + d] / total;
        coef64[i] = v;
    }
}

// prepare 2: clean resampled to 10 kHz in fp64; one thread per phase group
__global__ void __launch_bounds__(256) stoi_resample_clean_kernel(const double* __restrict__ clean,
                                                                   int64_t len, int64_t n10,
                                                                   const double* __restrict__ coef,
                                                                   double* __restrict__ x10) {
    using namespace stoi;
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int sig = blockIdx.y;
    if (5 * q >= n10) return;
    const double* x = clean + (int64_t)sig * len;
    double acc[5] = {0, 0, 0, 0, 0};
    for (int kk = 0; kk < KN; ++kk) {
        const int64_t n = 8 * q + kk + KLO;
        const double v = (n >= 0 && n < len) ? x[n] : 0.0;
#pragma unroll
        for (int r = 0; r < 5; ++r) acc[r] = fma(coef[r * CST + kk], v, acc[r]);
    }
    double* o = x10 + (int64_t)sig * n10;
#pragma unroll
    for (int r = 0; r < 5; ++r)
        if (5 * q + r < n10) o[5 * q + r] = acc[r];
}

// Other input rates, prepare: the normalised Octave filter times up (what
// resample_poly multiplies the supplied window by), 2 half + 1 taps
// (np.kaiser(2L + 1, 0.1102 (60 - 8.7)) x 2 up stop sinc(2 stop t)); half = 0
// is the 10-kHz identity.
__global__ void __launch_bounds__(1024) stoi_coef_generic_kernel(double* __restrict__ h,
                                                                  int64_t half, int up, int down) {
    __shared__ double red[1024];
    const int tid = threadIdx.x;
    if (half == 0) {
        if (tid == 0) h[0] = 1.0;
        return;
    }
    const int64_t n = 2 * half + 1;
    const double beta = 0.1102 * (60.0 - 8.7);
    const double i0b = bessel_i0(beta);
    const double stop = 1.0 / (2.0 * (double)(up > down ? up : down));
    double part = 0.0;
    for (int64_t i = tid; i < n; i += 1024) {
        const double a = (double)half;  // np.kaiser: alpha = (M - 1) / 2
        const double u = ((double)i - a) / a;
        const double kais = bessel_i0(beta * sqrt(fmax(1.0 - u * u, 0.0))) / i0b;
        const double x = 2.0 * stop * (double)(i - half);
        const double sinc = (i == half) ? 1.0 : sinpi(x) / (M_PI * x);
        const double v = kais * (2.0 * up * stop * sinc);
        h[i] = v;
        part += v;
    }
    red[tid] = part;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double total = red[0];
    for (int64_t i = tid; i < n; i += 1024) h[i] = up * (h[i] / total);
}

// Other input rates: resample_poly as upfirdn(h padded by pre_pad zeros)
// with its first pre_rm outputs dropped, out[i] = sum over n of
// h[(i + pre_rm) down - pre_pad - n up] e[n], fp64, one thread per output.
// TEST: e[n] = y[off + n - lag] (f32, zero outside [0, len) like
// cse_stoi_cells, clipped to [-1, 1] if clip); else e = x (f64 clean rows).
template <bool TEST>
__global__ void __launch_bounds__(256) stoi_resample_kernel(
    const double* __restrict__ x, const float* __restrict__ y, const int64_t* __restrict__ y_off,
    const int32_t* __restrict__ lag, int clip, int64_t len, const double* __restrict__ h,
    int64_t ntap, int up, int down, int64_t pre_pad, int64_t pre_rm, int64_t n_out,
    double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t s = blockIdx.y;
    if (i >= n_out) return;
    const int64_t base = (i + pre_rm) * down - pre_pad;  // tap index of n = 0
    // taps j = base - n up in [0, ntap): n in [ceil((base - ntap + 1) / up), floor(base / up)]
    auto fdiv = [](int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); };
    int64_t nlo = -fdiv(-(base - ntap + 1), up), nhi = fdiv(base, up);
    int lg = 0;
    const float* ys = nullptr;
    const double* xs = nullptr;
    if (TEST) {
        lg = lag ? lag[s] : 0;
        ys = y + y_off[s];
        // e[n] = y[n - lag] for n and n - lag in [0, len)
        nlo = nlo > (int64_t)lg ? nlo : (int64_t)lg;
        nhi = nhi < len - 1 + lg ? nhi : len - 1 + lg;
    } else {
        xs = x + s * len;
    }
    nlo = nlo > 0 ? nlo : 0;
    nhi = nhi < len - 1 ? nhi : len - 1;
    double acc = 0.0;
    for (int64_t n = nlo; n <= nhi; ++n) {
        double e;
        if (TEST) {
            float v = ys[n - lg];
            if (clip) v = fminf(fmaxf(v, -1.0f), 1.0f);
            e = (double)v;
        } else {
            e = xs[n];
        }
        acc = fma(h[base - n * up], e, acc);
    }
    out[s * n_out + i] = acc;
}

// MATLAB hanning(256) = scipy hann(258)[1:-1]
__device__ __forceinline__ double hann_m(int n) {
    return 0.5 - 0.5 * cospi(2.0 * (double)(n + 1) / (double)(stoi::FR + 1));
}

// prepare 3: frame energies 20 log10(||w x_f|| + eps) in fp64 (utils.remove_silent_frames)
__global__ void __launch_bounds__(256) stoi_energy_kernel(const double* __restrict__ x10,
                                                           int64_t n10, int64_t F,
                                                           double* __restrict__ en) {
    using namespace stoi;
    const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int sig = blockIdx.y;
    if (f >= F) return;
    const double* x = x10 + (int64_t)sig * n10 + f * HOP;
    double s = 0.0;
    for (int n = lane; n < FR; n += 64) {
        const double v = hann_m(n) * x[n];
        s = fma(v, v, s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) en[(int64_t)sig * F + f] = 20.0 * log10(sqrt(s) + EPS);
}

// prepare 4 (one workgroup per signal): mask (max - 40 dB - e < 0), kept-frame
// list, K/M/J, and the per-block tables of distinct 10-kHz half-blocks:
// overlap-added half-block h takes w[n] e10[kf[h]] + w[128 + n] e10[kf[h-1] + 1]
__global__ void __launch_bounds__(256) stoi_select_kernel(const double* __restrict__ en,
                                                           int64_t F, int64_t NBLK,
                                                           int* __restrict__ meta,
                                                           int* __restrict__ kf_all,
                                                           int* __restrict__ btab_all) {
    using namespace stoi;
    __shared__ double red[256];
    __shared__ int cnt[256];
    const int sig = blockIdx.x, tid = threadIdx.x;
    const double* e = en + (int64_t)sig * F;
    int* kf = kf_all + (int64_t)sig * F;
    double mx = -INFINITY;
    for (int64_t f = tid; f < F; f += 256) mx = fmax(mx, e[f]);
    red[tid] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red[tid] = fmax(red[tid], red[tid + s]);
        __syncthreads();
    }
    const double thr = red[0];
    // ordered compaction, 256 frames per round
    int K = 0;
    for (int64_t f0 = 0; f0 < F; f0 += 256) {
        const int64_t f = f0 + tid;
        const int keep = (f < F) && ((thr - 40.0 - e[f]) < 0.0);
        cnt[tid] = keep;
        __syncthreads();
        for (int s = 1; s < 256; s <<= 1) {  // inclusive scan
            const int v = tid >= s ? cnt[tid - s] : 0;
            __syncthreads();
            cnt[tid] += v;
            __syncthreads();
        }
        if (keep) kf[K + cnt[tid] - 1] = (int)f;
        K += cnt[255];
        __syncthreads();
    }
    const int M = K > 1 ? K - 1 : 0;
    const int J = M >= NSEG ? M - NSEG + 1 : 0;
    __threadfence_block();
    __syncthreads();
    // blocks (one thread per signal: greedy over the kept frames)
    if (tid == 0) {
        int nblk = 0, j0 = 0;
        while (j0 < M) {
            int* t = btab_all + ((int64_t)sig * NBLK + nblk) * BT;
            int D = 0, last = -1;
            auto add = [&](int p) {
                if (p != last) { t[T_P + D] = p; last = p; ++D; }
                return D - 1;
            };
            // row hl of the block = kept frame h = j0 + hl: w[n] e10[kf[h]] +
            // w[128 + n] e10[kf[h - 1] + 1] (the second term only for h >= 1)
            auto row = [&](int hl) {
                const int h = j0 + hl;
                t[T_SB + hl] = h >= 1 ? add(kf[h - 1] + 1) : -1;
                t[T_SA + hl] = add(kf[h]);
            };
            row(0);
            int nf = 0;
            while (nf < FB && j0 + nf < M) {
                const int h = j0 + nf + 1;
                const int pb = kf[h - 1] + 1, pa = kf[h];
                const int extra = (pb != last) + (pa != pb);
                if (D + extra > MAXD) break;
                row(nf + 1);
                ++nf;
            }
            t[T_D] = D;
            t[T_J0] = j0;
            t[T_NF] = nf;
            j0 += nf;
            ++nblk;
        }
        meta[META * sig + 0] = K;
        meta[META * sig + 1] = M;
        meta[META * sig + 2] = J;
        meta[META * sig + 3] = F > 0 ? 1 : 0;  // 0: no frame at all (pystoi raises)
        meta[META * sig + 4] = nblk;
    }
}

// ---------------------------------------------------------------------------
// phase A: band envelopes of STFT frames [j0, j0 + nf) of one signal, fp64.
// (fp32 is not enough here: STOI normalises every band separately, and an
// fp32 FFT's roundoff, ~1e-7 of the frame's energy, is a large fraction of a
// band that holds only a noise floor.)
// ---------------------------------------------------------------------------
struct __attribute__((aligned(16))) cd {
    double x, y;
};
__device__ __forceinline__ cd dmk(double x, double y) { return cd{x, y}; }
__device__ __forceinline__ cd dadd(cd a, cd b) { return cd{a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cd dsub(cd a, cd b) { return cd{a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cd dmul(cd a, cd b) {
    return cd{fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x)};
}

// forward DFT4: X = [a0+a1+a2+a3, a0-i a1-a2+i a3, a0-a1+a2-a3, a0+i a1-a2-i a3]
__device__ __forceinline__ void fdft4(cd& a0, cd& a1, cd& a2, cd& a3) {
    const cd s02 = dadd(a0, a2), d02 = dsub(a0, a2);
    const cd s13 = dadd(a1, a3), t = dsub(a1, a3);
    const cd d13 = dmk(t.y, -t.x);  // -i (a1 - a3)
    a0 = dadd(s02, s13);
    a2 = dsub(s02, s13);
    a1 = dadd(d02, d13);
    a3 = dsub(d02, d13);
}

// e^{-2πi m/16}, m in [0, 9]
__device__ __forceinline__ cd w16f(int m) {
    constexpr double c1 = 0.92387953251128674, s1 = 0.38268343236508978, r2 = 0.70710678118654752;
    switch (m) {
        case 0: return dmk(1.0, 0.0);
        case 1: return dmk(c1, -s1);
        case 2: return dmk(r2, -r2);
        case 3: return dmk(s1, -c1);
        case 4: return dmk(0.0, -1.0);
        case 5: return dmk(-s1, -c1);
        case 6: return dmk(-r2, -r2);
        case 7: return dmk(-c1, -s1);
        case 8: return dmk(-1.0, 0.0);
        default: return dmk(-c1, s1);  // 9
    }
}

// forward DFT4 of (a0, a1, 0, 0): [a0+a1, a0-i a1, a0-a1, a0+i a1]
__device__ __forceinline__ void fdft4_half(cd& a0, cd& a1, cd& a2, cd& a3) {
    const cd s = dadd(a0, a1), d = dsub(a0, a1);
    const cd m = dmk(a1.y, -a1.x);  // -i a1
    a2 = d;
    a3 = dsub(a0, m);
    a1 = dadd(a0, m);
    a0 = s;
}

// forward DFT16 in registers (radix 4 x 4), natural order in and out;
// HALF: v[8..15] are zero on entry
template <bool HALF = false>
__device__ __forceinline__ void fdft16(cd (&v)[16]) {
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
        if (HALF)
            fdft4_half(v[k2], v[4 + k2], v[8 + k2], v[12 + k2]);
        else
            fdft4(v[k2], v[4 + k2], v[8 + k2], v[12 + k2]);
    }
#pragma unroll
    for (int n1 = 1; n1 < 4; ++n1)
#pragma unroll
        for (int k2 = 1; k2 < 4; ++k2) {
            const int m = n1 * k2;
            const cd a = v[4 * n1 + k2];
            v[4 * n1 + k2] = (m == 4) ? dmk(a.y, -a.x) : dmul(a, w16f(m));
        }
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) fdft4(v[4 * n1], v[4 * n1 + 1], v[4 * n1 + 2], v[4 * n1 + 3]);
    cd t[16];
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1)
#pragma unroll
        for (int n2 = 0; n2 < 4; ++n2) t[n1 + 4 * n2] = v[4 * n1 + n2];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = t[i];
}

// ordering of LDS accesses among the lanes of ONE wave: a compiler-level
// barrier suffices (the LDS executes a wave's DS instructions in issue order)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Per-stage timing (analysis builds only, -DCSE_STOI_STAMPS): shader-cycle
// (s_memtime) deltas of the workgroup between its barriers, by stage, stored
// per cell by thread 0 into the buffer cse_stoi_stamp_buffer() installs.
//   0 tables + first block table   1 staging writes   2 resampling
//   3 rfft (OLA/window, DFT16 x DFT16, transposes, |X|^2)   4 band sums
//   5 phase B   6 whole kernel
struct StoiStamps {
#ifdef CSE_STOI_STAMPS
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long last = 0, t0 = 0;
    __device__ void start() { t0 = last = __builtin_amdgcn_s_memtime(); }
    __device__ void mark(int k) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        acc[k] += now - last;
        last = now;
    }
#else
    __device__ void start() {}
    __device__ void mark(int) {}
#endif
};
#ifdef CSE_STOI_STAMPS
__device__ unsigned long long* g_stoi_stamps;
#endif

struct StoiLds {
    double wnd[stoi::FR];
    cd tw256[256];          // e^{-2πi k/256}
    cd tw512[256];          // e^{-2πi k/512}
    union {
        struct {
            // 16-kHz input, f32 as the cells hold it
            float stage[stoi::STAGE_F];
            double e10[stoi::MAXD][stoi::HOP];
        } a;
        double t[stoi::FB][16 * 17];   // transpose, one component at a time; then |X|^2
        struct {
            double y[94 * 17];
            double x[94 * 17];
        } b;
    } u;
    double red[stoi::NT / 64];
    int tab[2][stoi::BT];  // this block's table and the next one's (prefetch)
};

// e (16 kHz) sample n of a cell: the finalize_enhanced output — y shifted by
// the alignment lag, length-matched (zero outside [0, len)), clipped
__device__ __forceinline__ float cell_sample(const float* y, int64_t n, int64_t len, int lag,
                                             bool clip) {
    const int64_t s = n - lag;
    if (n < 0 || n >= len || s < 0 || s >= len) return 0.0f;
    float v = y[s];
    if (clip) v = fminf(fmaxf(v, -1.0f), 1.0f);
    return v;
}

__device__ __forceinline__ void stoi_tables(StoiLds& L) {
    const int tid = threadIdx.x;
    for (int n = tid; n < stoi::FR; n += stoi::NT) L.wnd[n] = hann_m(n);
    for (int k = tid; k < 256; k += stoi::NT) {
        double s, c;
        sincospi(-2.0 * k / 256.0, &s, &c);
        L.tw256[k] = dmk(c, s);
        sincospi(-2.0 * k / 512.0, &s, &c);
        L.tw512[k] = dmk(c, s);
    }
}

// PRE: the 10-kHz signal is given (fp64 x10: the clean side, and the cells at
// input rates other than 16 kHz); otherwise the 16-kHz cell output is
// resampled here.
template <bool PRE>
__device__ __forceinline__ void stoi_phase_a(StoiLds& L, const float* __restrict__ y, int64_t len,
                                             int lag, bool clip, const double* __restrict__ x10,
                                             const double* __restrict__ coef,
                                             const int* __restrict__ btab, int nblk,
                                             double* __restrict__ env, StoiStamps& ts) {
    using namespace stoi;
    const int tid = threadIdx.x;
    // 16-kHz input samples of one staging chunk, loaded into registers one
    // chunk ahead (the global-load latency overlaps the previous chunk's
    // resampling instead of stalling every chunk).  The loads go through a raw
    // buffer over the y samples finalize_enhanced keeps, src in [lo, hi) (src and
    // src + lag inside [0, len)): the range check returns 0 for every other
    // index, so the loads carry no masks and issue back to back.
    // Lane tid stages slot fs = tid / FW (FW = 28 lanes per slot, 9 slots), samples
    // uu = fr + FW u: one block-table read and one base index per fetch, the
    // loads at constant strides from it
    constexpr int NSL = SLOTS;                            // slots per chunk
    constexpr int FW = 28, NU = 8 * GRP + KN;             // NU = 339 samples staged per slot
    constexpr int PF = (NU + FW - 1) / FW;                // 13 loads per lane
    static_assert(SLOTS * FW <= NT, "staging lanes");
    const int fs = tid / FW, fr = tid - FW * (tid / FW);
    // finalize_enhanced keeps y[src] for src and src + lag inside [0, len):
    // src - lo in [0, cnt).  Indices are clamped into that range for the load and
    // the sample is zeroed at staging when it was outside (no reliance on the
    // buffer range check, which does not see a folded immediate offset).
    float pre[PF];
    const int lo = (int)max((int64_t)0, -(int64_t)lag);
    const int cnt = max((int)min(len, len - lag) - lo, 0);
    const __amdgpu_buffer_rsrc_t yrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(y + lo), (short)0, 4 * cnt, 0x00020000);
    int fbase = 0;  // src - lo of the lane's sample uu = fr in the fetched chunk
    auto fetch = [&](const int* tb, int c0) {
        // lanes past the 9 slots (and slots past the chunk) read a table entry
        // in range and are never staged
        const int q0 = (HOP * tb[T_P + c0 + min(fs, NSL - 1)]) / UP;
        fbase = 8 * q0 + KLO + fr - lag - lo;
#pragma unroll
        for (int u = 0; u < PF; ++u)
            pre[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                yrc, 4 * min(max(fbase + FW * u, 0), max(cnt - 1, 0)), 0, 0));
    };
    if (nblk > 0) {
        __syncthreads();
        if (tid < BT) L.tab[0][tid] = btab[tid];
        __syncthreads();
        if (!PRE) fetch(L.tab[0], 0);
    }
    ts.mark(0);
    for (int blk = 0; blk < nblk; ++blk) {
        const int* tb = L.tab[blk & 1];
        const int j0 = tb[T_J0], nf = tb[T_NF];
        const int* tn = L.tab[(blk + 1) & 1];
        __syncthreads();  // previous block's readers of the union and of tn are done
        if (blk + 1 < nblk && tid < BT) L.tab[(blk + 1) & 1][tid] = btab[(int64_t)(blk + 1) * BT + tid];
        const int D = tb[T_D];
        // ---- 10-kHz half-blocks p = tb[T_P + d] into e10[d]
        if (PRE) {
            for (int i = tid; i < D * HOP; i += NT) {
                const int d = i >> 7, n = i & (HOP - 1);
                L.u.a.e10[d][n] = x10[(int64_t)tb[T_P + d] * HOP + n];
            }
        } else {
            for (int c0 = 0; c0 < D; c0 += NSL) {
                const int ns = min(NSL, D - c0);
                // stage e[8 q0 - 58 + uu], uu < 339, at [uu] (LIN) or [uu & 7][uu >> 3]
                if (fs < ns) {
                    float* st = L.u.a.stage + fs * SSTR;
#pragma unroll
                    for (int u = 0; u < PF; ++u) {
                        const int uu = fr + FW * u;
                        float v = (unsigned)(fbase + FW * u) < (unsigned)cnt ? pre[u] : 0.0f;
                        if (clip) v = fminf(fmaxf(v, -1.0f), 1.0f);
                        if (u < PF - 1 || uu < NU) st[uu] = v;
                    }
                }
                __syncthreads();  // stage (and the next block's table) visible
                ts.mark(1);
                if (c0 + NSL < D)
                    fetch(tb, c0 + NSL);
                else if (blk + 1 < nblk)
                    fetch(tn, 0);
                if (tid < ns * GRP) {
                    const int s = tid / GRP, g = tid - s * GRP;
                    const int64_t p = tb[T_P + c0 + s];
                    const int64_t q0 = (HOP * p) / UP;
                    const int64_t q = q0 + g;
                    const float* st = L.u.a.stage + s * SSTR + 8 * g;
                    // sample j of tap block kb (j < 8): st[8 kb + j]
                    auto sidx = [](int kb, int j) { return 8 * kb + j; };
                    double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
                    // taps kk = 8 kb + j of phase r; c_r[kk] = 0 outside
                    // 8r <= 5kk <= 8r + 580 (and kk >= 123): the edge blocks
                    // kb = 0, 14, 15 are unrolled with those taps left out
                    auto taps = [&](auto kbc) {
                        constexpr int kb = decltype(kbc)::value;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const int kk = 8 * kb + j;
                            const double e = (double)st[sidx(kb, j)];
#pragma unroll
                            for (int r = 0; r < 5; ++r)
                                if (5 * kk >= 8 * r && 5 * kk <= 8 * r + 580)
                                    acc[r] = fma(coef[r * CST + kk], e, acc[r]);
                        }
                    };
                    // interior blocks: the 8 samples of block kb + 1 are read
                    // from LDS while block kb's 40 FMAs run.  The coefficients
                    // come through the scalar cache, and an s_load makes the
                    // wait before their first use an lgkmcnt(0), which also
                    // covers every LDS read then in flight: the next block's
                    // reads are issued only after that wait (after tap j = 0),
                    // so one block costs one scalar-load latency instead of a
                    // scalar load plus four LDS round trips
                    float sv[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) sv[j] = st[sidx(1, j)];
                    taps(std::integral_constant<int, 0>());
#pragma unroll 1
                    for (int kb = 1; kb < 14; ++kb) {  // every tap nonzero
                        double e[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) e[j] = (double)sv[j];
#pragma unroll
                        for (int r = 0; r < 5; ++r) acc[r] = fma(coef[r * CST + 8 * kb], e[0], acc[r]);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int j = 0; j < 8; ++j) sv[j] = st[sidx(kb + 1, j)];
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int j = 1; j < 8; ++j) {
#pragma unroll
                            for (int r = 0; r < 5; ++r)
                                acc[r] = fma(coef[r * CST + 8 * kb + j], e[j], acc[r]);
                        }
                    }
                    taps(std::integral_constant<int, 14>());
                    taps(std::integral_constant<int, 15>());
#pragma unroll
                    for (int r = 0; r < 5; ++r) {
                        const int64_t off = 5 * q + r - HOP * p;
                        if (off >= 0 && off < HOP) L.u.a.e10[c0 + s][off] = acc[r];
                    }
                }
                __syncthreads();  // e10 complete (also ends the chunk loop's last pass)
                ts.mark(2);
            }
        }
        if (PRE) __syncthreads();
        // ---- 512-point rfft of frame fl, 16 lanes per frame: sample n of the
        // frame is w[n] ola[fl + n/128][n mod 128], the overlap-added row
        // ola[hl][o] = w[o] e10[sa][o] + w[128 + o] e10[sb][o] read straight
        // from the half-blocks; z[m] = s[2m] + i s[2m+1] (m < 128, 0 above),
        // Z = DFT256(z) as DFT16 x DFT16
        {
            const int fl = tid >> 4, n1 = tid & 15;
            cd v[16];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int hl = min(fl + hh, nf);  // rows of frame fl (fl < nf for the lanes kept)
                const double* ea = L.u.a.e10[tb[T_SA + hl]];
                const int sb = tb[T_SB + hl];
                const double* eb = L.u.a.e10[sb >= 0 ? sb : 0];
                const double wb = sb >= 0 ? 1.0 : 0.0;
#pragma unroll
                for (int n2 = 4 * hh; n2 < 4 * hh + 4; ++n2) {
                    const int n = 2 * (n1 + 16 * n2), o = n - HOP * hh;
                    const double r0 = fma(wb * L.wnd[HOP + o], eb[o], L.wnd[o] * ea[o]);
                    const double r1 = fma(wb * L.wnd[HOP + o + 1], eb[o + 1], L.wnd[o + 1] * ea[o + 1]);
                    v[n2] = dmk(L.wnd[n] * r0, L.wnd[n + 1] * r1);
                }
            }
            fdft16<true>(v);                           // v[k1] = A[n1][k1] (v[8..15] = 0)
            // twiddles e^{-2πi n1 k1/256} from the table (n1 k1 <= 225): 15
            // independent reads instead of a 14-deep chain of fp64 complex products
#pragma unroll
            for (int k1 = 1; k1 < 16; ++k1) v[k1] = dmul(v[k1], L.tw256[n1 * k1]);
            // the transposes stay inside the frame's 16 lanes (one wave): after
            // the one workgroup barrier (t aliases e10), wave-level ordering
            double* t = L.u.t[fl];
            const int k1 = n1;
            double re[16];
            __syncthreads();  // every lane's e10 reads are done: t aliases e10
#pragma unroll
            for (int a = 0; a < 16; ++a) t[a * 17 + n1] = v[a].x;
            wave_sync();
#pragma unroll
            for (int a = 0; a < 16; ++a) re[a] = t[k1 * 17 + a];
            wave_sync();
#pragma unroll
            for (int a = 0; a < 16; ++a) t[a * 17 + n1] = v[a].y;
            wave_sync();
#pragma unroll
            for (int a = 0; a < 16; ++a) v[a] = dmk(re[a], t[k1 * 17 + a]);
            fdft16(v);                                 // v[k2] = Z[k1 + 16 k2]
            wave_sync();                               // t reads issued before |X|^2 overwrites them
            // partner Z[(256 - k) mod 256]: lane (16 - k1) & 15, register 15 - k2 (k1 > 0)
            const int src = (tid & 48) | ((16 - k1) & 15);  // lane within the wave
            double* pw = L.u.t[fl];  // 4 |X|^2 of the frame, bins < 224, in its own rows
#pragma unroll
            for (int k2 = 0; k2 < 14; ++k2) {  // k < 224 (the bands end at bin 219)
                const cd zo = v[15 - k2];
                cd zp = dmk(__shfl(zo.x, src), __shfl(zo.y, src));
                if (k1 == 0) zp = v[(16 - k2) & 15];
                const cd z = v[k2];
                // 2X[k] = 2E + e^{-2πi k/512} 2O, 2E = z + conj(zp), 2O = -i (z - conj(zp)):
                // the halves are left out (exact power-of-two scalings) and the
                // band sums take 1/4 (sqrt(s/4) = sqrt(s)/2 exactly)
                const double ex = z.x + zp.x, ey = z.y - zp.y;
                const double ox = z.y + zp.y, oy = zp.x - z.x;
                const cd w = L.tw512[k1 + 16 * k2];
                const double xr = fma(w.x, ox, fma(-w.y, oy, ex));
                const double xi = fma(w.x, oy, fma(w.y, ox, ey));
                pw[k1 + 16 * k2] = fma(xr, xr, xi * xi);
            }
            // ---- band envelopes of the frame by its own 16 lanes (one wave:
            // no workgroup barrier; the next block's first barrier protects pw)
            wave_sync();
            ts.mark(3);
            if (n1 < NBAND && fl < nf) {
                // 8 reads in flight per round into 4 partial sums: the serial
                // read-and-add over the top band (45 bins) was 12 % of the
                // kernel (tools/stoi_stages.py); the oracle's band sum is a
                // matrix product, its order unspecified
                const int k0 = BAND_EDGE[n1], k1e = BAND_EDGE[n1 + 1];
                double s4[4] = {0.0, 0.0, 0.0, 0.0};
                for (int k = k0; k < k1e; k += 8) {
                    double q[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) q[u] = (k + u < k1e) ? pw[k + u] : 0.0;
#pragma unroll
                    for (int u = 0; u < 8; ++u) s4[u & 3] += q[u];
                }
                const double s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
                env[(int64_t)(j0 + fl) * 16 + n1] = 0.5 * sqrt(s);
            }
            ts.mark(4);
        }
    }
}

// clean side: envelopes, then per (segment, band) statistics
__global__ void __launch_bounds__(stoi::NT) stoi_clean_env_kernel(const double* __restrict__ x10all,
                                                                   int64_t n10, int64_t NBLK,
                                                                   int64_t Mmax,
                                                                   const int* __restrict__ meta,
                                                                   const int* __restrict__ btab,
                                                                   double* __restrict__ xtob) {
    __shared__ StoiLds L;
    const int sig = blockIdx.x;
    stoi_tables(L);
    const int nblk = meta[stoi::META * sig + 4];
    StoiStamps ts;
    stoi_phase_a<true>(L, nullptr, 0, 0, false, x10all + (int64_t)sig * n10, nullptr,
                       btab + (int64_t)sig * NBLK * stoi::BT, nblk, xtob + (int64_t)sig * Mmax * 16, ts);
}

// (||x||, mean, 1/(||x - mean|| + eps)) of the clean envelope over each segment
__global__ void __launch_bounds__(256) stoi_clean_stat_kernel(const double* __restrict__ xtob,
                                                               int64_t Mmax, int64_t Jmax,
                                                               const int* __restrict__ meta,
                                                               double4* __restrict__ xstat) {
    using namespace stoi;
    const int sig = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int J = meta[META * sig + 2];
    const int j = (int)(i / 16), b = (int)(i % 16);
    if (j >= J || b >= NBAND) return;
    const double* x = xtob + ((int64_t)sig * Mmax + j) * 16 + b;
    double s = 0.0, s2 = 0.0;
    for (int t = 0; t < NSEG; ++t) {
        const double v = x[t * 16];
        s += v;
        s2 = fma(v, v, s2);
    }
    const double mean = s / NSEG;
    double c2 = 0.0;
    for (int t = 0; t < NSEG; ++t) {
        const double v = x[t * 16] - mean;
        c2 = fma(v, v, c2);
    }
    xstat[((int64_t)sig * Jmax + j) * 16 + b] = make_double4(sqrt(s2), mean, 1.0 / (sqrt(c2) + EPS), 0.0);
}

// ---------------------------------------------------------------------------
// per cell: phase A into env scratch, phase B correlations -> stoi[c]
// ---------------------------------------------------------------------------
struct StoiArgs {
    const float* y;
    const int64_t* y_offset;
    const int32_t* lag;
    const int32_t* sig_of;
    int64_t len, NBLK, Mmax, Jmax;
    int clip;
    const double* coef;
    const int* meta;
    const int* btab;
    const double* xtob;
    const double4* xstat;
    double* scratch;  // [n_cells][Mmax][16]
    double* out;
};

// PRE: the cell's test signal is given at 10 kHz (y10 + c n10, fp64: other
// input rates, resampled by stoi_resample_kernel); otherwise the 16-kHz
// output y is resampled in phase A.
template <bool PRE>
__device__ __forceinline__ void stoi_cells_body(StoiLds& L, const StoiArgs& a,
                                                const double* __restrict__ coef,
                                                const double* __restrict__ y10, int64_t n10) {
    using namespace stoi;
    const int64_t c = blockIdx.x;
    const int tid = threadIdx.x;
    const int sig = a.sig_of[c];
    const int J = a.meta[META * sig + 2];
    if (a.meta[META * sig + 3] == 0) {  // no 256-sample frame at all: pystoi raises -> None
        if (tid == 0) a.out[c] = __builtin_nan("");
        return;
    }
    if (J <= 0) {  // fewer than 30 STFT frames after silent-frame removal
        if (tid == 0) a.out[c] = 1e-5;
        return;
    }
    StoiStamps ts;
    ts.start();
    stoi_tables(L);
    double* env = a.scratch + c * a.Mmax * 16;
    const int lag = a.lag ? a.lag[c] : 0;
    if constexpr (PRE)
        stoi_phase_a<true>(L, nullptr, 0, 0, false, y10 + c * n10, nullptr,
                           a.btab + (int64_t)sig * a.NBLK * BT, a.meta[META * sig + 4], env, ts);
    else
        stoi_phase_a<false>(L, a.y + a.y_offset[c], a.len, lag, a.clip != 0, nullptr, coef,
                            a.btab + (int64_t)sig * a.NBLK * BT, a.meta[META * sig + 4], env, ts);
    __syncthreads();  // env rows of this workgroup are visible to it
    ts.mark(4);
    // ---- phase B: segment j, band b
    const double* xt = a.xtob + (int64_t)sig * a.Mmax * 16;
    const double4* xs = a.xstat + (int64_t)sig * a.Jmax * 16;
    constexpr double clipf = 6.623413251903491;  // 1 + 10^(-BETA/20)
    double dsum = 0.0;
    const int seg = tid & 63, bg = tid >> 6;
    for (int j0 = 0; j0 < J; j0 += 64) {
        const int rows = min(64, J - j0) + NSEG - 1;
        __syncthreads();
        {   // the tile's <= 6 rows per lane of both envelopes: every load issued
            // before the first store (clamped indices, masked stores)
            constexpr int TU = (94 * 16 + NT - 1) / NT;
            double ty[TU], tx[TU];
#pragma unroll
            for (int u = 0; u < TU; ++u) {
                const int i = min(tid + u * NT, rows * 16 - 1);
                ty[u] = env[(int64_t)j0 * 16 + i];
                tx[u] = xt[(int64_t)j0 * 16 + i];
            }
#pragma unroll
            for (int u = 0; u < TU; ++u) {
                const int i = tid + u * NT;
                if (i < rows * 16) {
                    L.u.b.y[(i >> 4) * 17 + (i & 15)] = ty[u];
                    L.u.b.x[(i >> 4) * 17 + (i & 15)] = tx[u];
                }
            }
        }
        __syncthreads();
        const int j = j0 + seg;
        if (j < J) {
#pragma unroll 1
            for (int b = bg; b < NBAND; b += 4) {
                const double4 st = xs[(int64_t)j * 16 + b];
                const double* yr = L.u.b.y + seg * 17 + b;
                const double* xr = L.u.b.x + seg * 17 + b;
                double yv[NSEG];
                double ny2 = 0.0;
#pragma unroll
                for (int t = 0; t < NSEG; ++t) {
                    yv[t] = yr[t * 17];
                    ny2 = fma(yv[t], yv[t], ny2);
                }
                const double alpha = st.x / (sqrt(ny2) + EPS);
                double sy = 0.0;
#pragma unroll
                for (int t = 0; t < NSEG; ++t) {
                    yv[t] = fmin(yv[t] * alpha, xr[t * 17] * clipf);
                    sy += yv[t];
                }
                const double my = sy / NSEG;
                double c2 = 0.0, cr = 0.0;
#pragma unroll
                for (int t = 0; t < NSEG; ++t) {
                    const double d = yv[t] - my;
                    c2 = fma(d, d, c2);
                    cr = fma(d, xr[t * 17] - st.y, cr);
                }
                dsum += (cr * st.z) / (sqrt(c2) + EPS);
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dsum += __shfl_xor(dsum, o);
    if ((tid & 63) == 0) L.red[tid >> 6] = dsum;
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int w = 0; w < NT / 64; ++w) s += L.red[w];
        a.out[c] = s / ((double)J * NBAND);
    }
#ifdef CSE_STOI_STAMPS
    ts.mark(5);
    if (tid == 0 && g_stoi_stamps) {
        ts.acc[6] = ts.last - ts.t0;
#pragma unroll
        for (int k = 0; k < 8; ++k) g_stoi_stamps[c * 8 + k] = ts.acc[k];
    }
#endif
}

// coef is a separate const __restrict__ argument so the compiler can prove it
// is never written and read it through the scalar cache (s_load): inside the
// argument struct it became per-lane vector loads waited on right after issue
__global__ void __launch_bounds__(stoi::NT, 3) stoi_cells_kernel(StoiArgs a,
                                                              const double* __restrict__ coef) {
    __shared__ StoiLds L;
    stoi_cells_body<false>(L, a, coef, nullptr, 0);
}

// input rates other than 16 kHz: the cells' test signals already at 10 kHz
__global__ void __launch_bounds__(stoi::NT, 3) stoi_cells_pre_kernel(StoiArgs a,
                                                                  const double* __restrict__ y10,
                                                                  int64_t n10) {
    __shared__ StoiLds L;
    stoi_cells_body<true>(L, a, nullptr, y10, n10);
}

}  // namespace cse

using namespace cse;

// input rates: 16 kHz (the sweep's, resampled inside the cell kernel) and,
// through the generic resampler, any rate in [1 kHz, 768 kHz] whose filter
// stays below 2^25 taps
static bool stoi_rate_ok(int sr, int64_t len) {
    if (sr == 16000) return true;
    if (sr < 1000 || sr > 768000) return false;
    return 2 * resamp_for(sr, len).half + 1 < (1 << 25);
}

extern "C" int64_t cse_stoi_workspace_bytes_sr(int64_t n_sig, int64_t len, int sr) {
    if (n_sig < 1 || len < 1 || !stoi_rate_ok(sr, len)) return -1;
    return stoi_layout(n_sig, len, sr).total;
}

extern "C" int64_t cse_stoi_workspace_bytes(int64_t n_sig, int64_t len) {
    return cse_stoi_workspace_bytes_sr(n_sig, len, 16000);
}

extern "C" int64_t cse_stoi_scratch_bytes_sr(int64_t n_cells, int64_t len, int sr) {
    if (n_cells < 0 || len < 1 || !stoi_rate_ok(sr, len)) return -1;
    const StoiLayout L = stoi_layout(1, len, sr);
    // per cell: band envelopes [Mmax][16], and at other rates the 10-kHz test signal
    return n_cells * (L.Mmax * 16 + (sr == 16000 ? 0 : L.n10)) * 8;
}

extern "C" int64_t cse_stoi_scratch_bytes(int64_t n_cells, int64_t len) {
    return cse_stoi_scratch_bytes_sr(n_cells, len, 16000);
}

extern "C" int cse_stoi_prepare(const double* clean, int64_t n_sig, int64_t len, int sr,
                                void* workspace, cse_stream_t stream) {
    CSE_CHECK_ARG(clean && workspace, "cse_stoi_prepare: NULL clean/workspace");
    CSE_CHECK_ARG(n_sig >= 1 && n_sig < 65536 && len >= 1, "cse_stoi_prepare: n_sig=%lld len=%lld",
                  (long long)n_sig, (long long)len);
    CSE_CHECK_ARG(stoi_rate_ok(sr, len), "cse_stoi_prepare: sr=%d not supported", sr);
    const StoiLayout L = stoi_layout(n_sig, len, sr);
    unsigned char* ws = (unsigned char*)workspace;
    hipStream_t st = (hipStream_t)stream;
    double* coef64 = (double*)(ws + L.coef64);
    int* meta = (int*)(ws + L.meta);
    double* x10 = (double*)(ws + L.x10);
    double* en = (double*)(ws + L.en);
    int* kf = (int*)(ws + L.kf);
    int* btab = (int*)(ws + L.btab);
    double* xtob = (double*)(ws + L.xtob);
    double4* xstat = (double4*)(ws + L.xstat);
    if (sr == 16000) {
        hipLaunchKernelGGL(stoi_coef_kernel, dim3(1), dim3(1024), 0, st, coef64);
        const int64_t groups = (L.n10 + 4) / 5;
        hipLaunchKernelGGL(stoi_resample_clean_kernel, dim3(ceil_div(groups, 256), (unsigned)n_sig),
                           dim3(256), 0, st, clean, len, L.n10, (const double*)coef64, x10);
    } else {
        const Resamp r = resamp_for(sr, len);
        double* h = (double*)(ws + L.hgen);
        hipLaunchKernelGGL(stoi_coef_generic_kernel, dim3(1), dim3(1024), 0, st, h, r.half, r.up,
                           r.down);
        hipLaunchKernelGGL(stoi_resample_kernel<false>, dim3(ceil_div(L.n10, 256), (unsigned)n_sig),
                           dim3(256), 0, st, clean, nullptr, nullptr, nullptr, 0, len,
                           (const double*)h, 2 * r.half + 1, r.up, r.down, r.pre_pad, r.pre_rm,
                           L.n10, x10);
    }
    if (L.F > 0)
        hipLaunchKernelGGL(stoi_energy_kernel, dim3(ceil_div(L.F, 4), (unsigned)n_sig), dim3(256), 0,
                           st, x10, L.n10, L.F, en);
    hipLaunchKernelGGL(stoi_select_kernel, dim3((unsigned)n_sig), dim3(256), 0, st, en, L.F, L.NBLK,
                       meta, kf, btab);
    if (L.Mmax > 0)
        hipLaunchKernelGGL(stoi_clean_env_kernel, dim3((unsigned)n_sig), dim3(stoi::NT), 0, st, x10,
                           L.n10, L.NBLK, L.Mmax, meta, btab, xtob);
    if (L.Jmax > 0)
        hipLaunchKernelGGL(stoi_clean_stat_kernel, dim3(ceil_div(L.Jmax * 16, 256), (unsigned)n_sig),
                           dim3(256), 0, st, xtob, L.Mmax, L.Jmax, meta, xstat);
    CSE_CHECK_LAUNCH("cse_stoi_prepare");
    return CSE_OK;
}

#ifdef CSE_STOI_STAMPS
// analysis builds only: per-cell stage cycles into buf [n_cells][8] (u64), or off (NULL)
extern "C" int cse_stoi_stamp_buffer(void* buf) {
    unsigned long long* p = (unsigned long long*)buf;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stoi_stamps), &p, sizeof(p)) == hipSuccess ? CSE_OK
                                                                                        : CSE_ELAUNCH;
}
#endif

static int stoi_cells_launch(const char* name, const float* y, const int64_t* y_offset,
                             const int32_t* lag, const int32_t* sig_of, int64_t n_cells,
                             int64_t n_sig, int64_t len, int sr, int clip, const void* workspace,
                             void* scratch, double* stoi_out, cse_stream_t stream) {
    CSE_CHECK_ARG(y && y_offset && sig_of && workspace && stoi_out, "%s: NULL argument", name);
    CSE_CHECK_ARG(n_sig >= 1 && len >= 1, "%s: n_sig=%lld len=%lld", name, (long long)n_sig,
                  (long long)len);
    CSE_CHECK_ARG(stoi_rate_ok(sr, len), "%s: sr=%d not supported", name, sr);
    if (n_cells == 0) return CSE_OK;
    const StoiLayout L = stoi_layout(n_sig, len, sr);
    CSE_CHECK_ARG((L.Mmax == 0 && sr == 16000) || scratch, "%s: NULL scratch", name);
    CSE_CHECK_ARG(sr == 16000 || n_cells < 65536,
                  "%s: n_cells=%lld (< 65536 per call at sr != 16000)", name, (long long)n_cells);
    const unsigned char* ws = (const unsigned char*)workspace;
    StoiArgs a;
    a.y = y;
    a.y_offset = y_offset;
    a.lag = lag;
    a.sig_of = sig_of;
    a.len = len;
    a.NBLK = L.NBLK;
    a.Mmax = L.Mmax;
    a.Jmax = L.Jmax;
    a.clip = clip;
    a.coef = (const double*)(ws + L.coef64);
    a.meta = (const int*)(ws + L.meta);
    a.btab = (const int*)(ws + L.btab);
    a.xtob = (const double*)(ws + L.xtob);
    a.xstat = (const double4*)(ws + L.xstat);
    a.scratch = (double*)scratch;
    a.out = stoi_out;
    hipStream_t st = (hipStream_t)stream;
    if (sr == 16000) {
        hipLaunchKernelGGL(stoi_cells_kernel, dim3((unsigned)n_cells), dim3(stoi::NT), 0, st, a,
                           a.coef);
    } else {
        // the cells' shifted, clipped outputs resampled to 10 kHz after their envelopes
        const Resamp r = resamp_for(sr, len);
        double* y10 = (double*)scratch + n_cells * L.Mmax * 16;
        hipLaunchKernelGGL(stoi_resample_kernel<true>,
                           dim3(ceil_div(L.n10, 256), (unsigned)n_cells), dim3(256), 0, st, nullptr, y, y_offset, lag, clip, len,
                           (const double*)(ws + L.hgen), 2 * r.half + 1, r.up, r.down, r.pre_pad,
                           r.pre_rm, L.n10, y10);
        hipLaunchKernelGGL(stoi_cells_pre_kernel, dim3((unsigned)n_cells), dim3(stoi::NT), 0, st, a,
                           (const double*)y10, L.n10);
    }
    CSE_CHECK_LAUNCH(name);
    return CSE_OK;
}

extern "C" int cse_stoi_cells(const float* y, const int64_t* y_offset, const int32_t* lag,
                              const int32_t* sig_of, int64_t n_cells, int64_t n_sig, int64_t len,
                              int clip, const void* workspace, void* scratch, double* stoi_out,
                              cse_stream_t stream) {
    return stoi_cells_launch("cse_stoi_cells", y, y_offset, lag, sig_of, n_cells, n_sig, len,
                             16000, clip, workspace, scratch, stoi_out, stream);
}

extern "C" int cse_stoi_cells_sr(const float* y, const int64_t* y_offset, const int32_t* lag,
                                 const int32_t* sig_of, int64_t n_cells, int64_t n_sig,
                                 int64_t len, int sr, int clip, const void* workspace,
                                 void* scratch, double* stoi_out, cse_stream_t stream) {
    return stoi_cells_launch("cse_stoi_cells_sr", y, y_offset, lag, sig_of, n_cells, n_sig, len,
                             sr, clip, workspace, scratch, stoi_out, stream);
}
