// The hot path at any STFT shape the sweep kernels do not run: even n_fft
// in [64, 4096], any hop in [1, n_fft] (e.g. 512 / 160, 1024 / 512, 256 / 64,
// 2048 / 512, 400 / 160).  The reference's plugins take any n_fft and
// hop_length (spectral_subtractor.py:6, wiener_filter.py:7, mmse.py:6,
// advanced_mmse.py:7); its grids use 512 / 1024 at hop 128 / 256, which
// cse_enhance_cells runs (the short hops: cse_enhance_cells_short_hop).
//
// One workgroup per cell, frames in order, everything in LDS:
//   gains     each thread a strided set of bins: the same per-bin gain
//             functions as the sweep kernels (gain_bin, the n_fft-1024 row
//             form: gamma = max(|Y|^2 inv, eps) from the 1/max(N, eps) row,
//             SS from N itself), the decision-directed state rr per bin in LDS
//   irfft     x = irfft(S, n_fft) as a complex n_fft/2-point inverse FFT
//             (radix 2, LDS; a direct DFT when n_fft/2 is not a power of
//             two) of Z_k = E_k + i O_k with
//             E_k = (S_k + conj S_{M-k}) / 2, O_k = (S_k - conj S_{M-k}) W^-k / 2
//   OLA       periodic-Hann synthesis window, overlap-add into an n_fft ring
//   retire    the hop samples no later frame touches: divided by the window
//             square sum of the frames that cover them (librosa istft,
//             fp64 table), scored (clip, SNR error sum with the cell's lag),
//             written out (y_out) if asked
// The sweep kernels fold 1/wss into their window table and split the FFTs
// over 16 or 32 lanes per cell; this path keeps the librosa order of
// operations and favours generality over speed (it is not on the sweep).
#define CSE_ENHANCE_DEVICE_ONLY 1
#include "cse_enhance.hip"

namespace cse {

constexpr int GEN_NT = 256;  // threads per workgroup (one cell)

// the sweep kernels' per-cell parameter preparation (run_wg)
template <int ALGO>
__device__ CellParam gen_cell_param(const cse_cell_t* cp) {
    CellParam prm;
    prm.p0 = cp->param[0];
    prm.p1 = cp->param[1];
    prm.p2 = cp->param[2];
    prm.p3 = cp->param[3];
    prm.p4 = cp->param[4];
    prm.lg2_floor = (ALGO == CSE_ALGO_OMLSA) ? fast_log2(prm.p2) : 0.0f;
    prm.q_spp = 0.0f;
    if (ALGO == CSE_ALGO_OMLSA) {
        const double q = fmin(fmax((double)prm.p3, 1e-3), 1.0 - 1e-3);
        prm.q_spp = (float)(1e-10 / q);
        prm.p3 = (float)((1.0 - q) / q);
    }
    prm.gclip = 0.0f;
    if (ALGO == CSE_ALGO_WIENER) prm.p1 = fminf(prm.p1, 1.0f);
    if (ALGO == CSE_ALGO_MMSE) prm.p2 = fminf(prm.p2, prm.p3);
    if (ALGO == CSE_ALGO_OMLSA) prm.gclip = fminf(prm.p2, 1.0f);
    if (ALGO == CSE_ALGO_OMLSA) prm.p4 = fminf(prm.p4, 80.0f);
    return prm;
}

// LDS layout for n_fft N (M = N/2, B = M + 1), in bytes
struct GenLds {
    int N, M, B;
    int zr, zi, sr, si, twm, twn, win, wsq, rr, ring, red, total;
    __host__ __device__ GenLds(int n) : N(n), M(n / 2), B(n / 2 + 1) {
        int o = 0;
        auto take = [&](int bytes) {  // 16-B aligned regions
            const int at = o;
            o = (o + bytes + 15) & ~15;
            return at;
        };
        wsq = take(8 * N);              // double w(n)^2
        red = take(8 * GEN_NT);         // double reduction scratch
        zr = take(4 * M);               // float IFFT work (re, im)
        zi = take(4 * M);
        sr = take(4 * B);               // float S_k (re, im)
        si = take(4 * B);
        twm = take(8 * M);              // float2 e^{+2πi j/M}
        twn = take(8 * M);              // float2 e^{+2πi k/N}
        win = take(4 * N);              // float w(n)
        rr = take(4 * B);               // float decision-directed state
        ring = take(4 * N);             // float overlap-add ring
        total = o;
    }
};

template <int ALGO>
__device__ void gen_cell(const Args& a, int64_t c, int N, int log2m, unsigned char* smem) {
    const cse_cell_t* cp = a.cells + c;
    const int hop = cp->hop;
    if (hop < 1 || hop > N) {  // the reference's skip, as the sweep kernels report a bad cell
        if (threadIdx.x == 0) reject_cell(a, c);
        return;
    }
    const GenLds Ly(N);
    const int M = Ly.M, B = Ly.B;
    const int tid = threadIdx.x;
    double* wsq = (double*)(smem + Ly.wsq);
    double* red = (double*)(smem + Ly.red);
    float* zr = (float*)(smem + Ly.zr);
    float* zi = (float*)(smem + Ly.zi);
    float* sr = (float*)(smem + Ly.sr);
    float* si = (float*)(smem + Ly.si);
    float2* twm = (float2*)(smem + Ly.twm);
    float2* twn = (float2*)(smem + Ly.twn);
    float* win = (float*)(smem + Ly.win);
    float* rr = (float*)(smem + Ly.rr);
    float* ring = (float*)(smem + Ly.ring);
    constexpr float EPS = (ALGO == CSE_ALGO_MMSE) ? 1e-12f : 1e-10f;

    const int64_t len = a.len;
    const int T = (int)(1 + len / hop);
    const float2* Yb = a.Y + cp->y_offset;
    const float* Nb = a.noise + cp->noise_offset;
    const int64_t nstride = cp->noise_stride;
    const double* cb = (a.clean && cp->clean_offset >= 0) ? a.clean + cp->clean_offset : nullptr;
    const int lag = cp->lag;
    float* yout = (a.y_out && cp->out_offset >= 0) ? a.y_out + cp->out_offset : nullptr;
    float* gout = (a.g_out && cp->gain_offset >= 0) ? a.g_out + cp->gain_offset : nullptr;
    const int64_t out_len = a.out_len;
    const CellParam prm = gen_cell_param<ALGO>(cp);

    for (int n = tid; n < N; n += GEN_NT) {
        const double w = 0.5 - 0.5 * cospi(2.0 * (double)n / (double)N);
        win[n] = (float)w;
        wsq[n] = w * w;
        ring[n] = 0.0f;
    }
    for (int j = tid; j < M; j += GEN_NT) {
        double s, co;
        sincospi(2.0 * (double)j / (double)M, &s, &co);
        twm[j] = make_float2((float)co, (float)s);
    }
    for (int k = tid; k < M; k += GEN_NT) {
        double s, co;
        sincospi(2.0 * (double)k / (double)N, &s, &co);
        twn[k] = make_float2((float)co, (float)s);
    }
    for (int k = tid; k < B; k += GEN_NT) rr[k] = 0.0f;
    __syncthreads();

    double sse = 0.0;
    float chk = 0.0f;
    // retire output positions [p0, p1): ola / wss, clip, score, write
    auto retire = [&](int64_t p0, int64_t p1, int64_t covered_end) {
        for (int64_t p = p0 + tid; p < p1; p += GEN_NT) {
            float v = 0.0f;
            if (p < covered_end) {  // taken and cleared for the position N later
                const int64_t ri = (p + N / 2) % N;
                v = ring[ri];
                ring[ri] = 0.0f;
            }
            if (p < 0 || p >= len) continue;  // the centre padding / past the signal
            // frames t with 0 <= p + N/2 - t hop < N, t < T
            const int64_t q = p + N / 2;
            int64_t tlo = q - N + 1 <= 0 ? 0 : (q - N + 1 + hop - 1) / hop;
            int64_t thi = q / hop;
            if (thi > T - 1) thi = T - 1;
            double wss = 0.0;
            for (int64_t t = tlo; t <= thi; ++t) wss += wsq[q - t * hop];
            const float y = wss > 2.2250738585072014e-308 ? (float)((double)v / wss) : v;
            if (yout && p < out_len) yout[p] = y;
            // scored against clean[p + lag] (zeros without a clean reference, as
            // in the sweep kernels); samples whose partner lies outside are dropped
            const int64_t o = p + lag;
            if (o >= 0 && o < len) {
                chk = fmaf(y, 0.0f, chk);
                const double cv = cb ? cb[o] : 0.0;
                const double d = cv - (double)__builtin_amdgcn_fmed3f(y, -1.0f, 1.0f);
                sse = fma(d, d, sse);
            }
        }
    };

    for (int t = 0; t < T; ++t) {
        // ---- gains and S = Y s
        const float alpha_t = t == 0 ? 0.0f : prm.p0;
        for (int k = tid; k < B; k += GEN_NT) {
            float2 y = Yb[(int64_t)t * B + k];
            const float nv = Nb[t * nstride + k];
            RowV rv{0.0f, 0.0f, 0.0f};
            if (ALGO == CSE_ALGO_SS) {
                rv.g = nv;
            } else {
                const float gam = fmaxf((y.x * y.x + y.y * y.y) * nv, EPS);
                rv.g = ALGO == CSE_ALGO_OMLSA ? gam * kLog2e : gam;
            }
            float st = rr[k], g;
            const float s = gain_bin<1024, ALGO>(y, rv, st, alpha_t, prm, g);
            rr[k] = st;
            if (gout) gout[(int64_t)t * B + k] = g;
            float re = y.x * s, im = y.y * s;
            if (k == 0 || k == M) im = 0.0f;  // irfft ignores these imaginary parts
            sr[k] = re;
            si[k] = im;
        }
        __syncthreads();
        // ---- Z_k = E_k + i O_k into bit-reversed order for the radix-2 IFFT
        for (int k = tid; k < M; k += GEN_NT) {
            const float ar = sr[k], ai = si[k];
            const float br = sr[M - k], bi = -si[M - k];  // conj S_{M-k}
            const float er = 0.5f * (ar + br), ei = 0.5f * (ai + bi);
            const float dr = 0.5f * (ar - br), di = 0.5f * (ai - bi);
            const float2 w = twn[k];  // W^-k = e^{+2πi k/N}
            const float orr = dr * w.x - di * w.y, oi = dr * w.y + di * w.x;
            // radix 2: bit-reversed order; the direct DFT (log2m < 0): natural
            const int r = log2m >= 0 ? (int)(__brev((unsigned)k) >> (32 - log2m)) : k;
            zr[r] = er - oi;  // E + i O
            zi[r] = ei + orr;
        }
        __syncthreads();
        // M not a power of two (even n_fft such as 400): z[n] = sum_k Z_k
        // e^{+2πi kn/M} directly into the S rows (consumed above)
        float* xr = zr;
        float* xi = zi;
        if (log2m < 0) {
            for (int n = tid; n < M; n += GEN_NT) {
                float ar = 0.0f, ai = 0.0f;
                int m = 0;  // k n mod M
                for (int k = 0; k < M; ++k) {
                    const float2 w = twm[m];
                    ar = fmaf(zr[k], w.x, fmaf(-zi[k], w.y, ar));
                    ai = fmaf(zr[k], w.y, fmaf(zi[k], w.x, ai));
                    m += n;
                    if (m >= M) m -= M;
                }
                sr[n] = ar;
                si[n] = ai;
            }
            __syncthreads();
            xr = sr;
            xi = si;
        }
        for (int s = 1; s <= log2m; ++s) {
            const int half = 1 << (s - 1);
            for (int e = tid; e < M / 2; e += GEN_NT) {
                const int j = e & (half - 1);
                const int i0 = ((e >> (s - 1)) << s) + j, i1 = i0 + half;
                const float2 w = twm[j << (log2m - s)];
                const float br = zr[i1] * w.x - zi[i1] * w.y;
                const float bi = zr[i1] * w.y + zi[i1] * w.x;
                const float ar = zr[i0], ai = zi[i0];
                zr[i0] = ar + br;
                zi[i0] = ai + bi;
                zr[i1] = ar - br;
                zi[i1] = ai - bi;
            }
            __syncthreads();
        }
        // ---- window, overlap-add: x[2n] = Re z[n] / M, x[2n + 1] = Im z[n] / M
        const float inv_m = 1.0f / (float)M;
        for (int n = tid; n < N; n += GEN_NT) {
            const float x = ((n & 1) ? xi[n >> 1] : xr[n >> 1]) * inv_m;
            const int ri = (int)(((int64_t)t * hop + n) % N);
            ring[ri] = fmaf(win[n], x, ring[ri]);
        }
        __syncthreads();
        // ---- positions [t hop - N/2, (t + 1) hop - N/2) are final
        const int64_t p0 = (int64_t)t * hop - N / 2;
        retire(p0, p0 + hop, (int64_t)t * hop + N / 2);
        __syncthreads();
    }
    // the rest of the signal: covered by the last frames only (or by none)
    retire((int64_t)T * hop - N / 2, len, (int64_t)(T - 1) * hop + N / 2);

    // ---- reductions
    red[tid] = sse;
    __syncthreads();
    for (int s = GEN_NT / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double tot = red[0];
    __syncthreads();
    const int bad = __syncthreads_or(chk != 0.0f);
    if (tid == 0) {
        if (a.sse) a.sse[c] = tot;
        if (a.finite) a.finite[c] = bad ? 0 : 1;
    }
}

__global__ void __launch_bounds__(GEN_NT) enhance_generic_kernel(Args a, int N, int log2m) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t c = blockIdx.x;
    if (c >= a.n_cells) return;
    const int algo = a.cells[c].algo;
    switch (algo) {
        case CSE_ALGO_SS: gen_cell<CSE_ALGO_SS>(a, c, N, log2m, smem); break;
        case CSE_ALGO_WIENER: gen_cell<CSE_ALGO_WIENER>(a, c, N, log2m, smem); break;
        case CSE_ALGO_MMSE: gen_cell<CSE_ALGO_MMSE>(a, c, N, log2m, smem); break;
        case CSE_ALGO_OMLSA: gen_cell<CSE_ALGO_OMLSA>(a, c, N, log2m, smem); break;
        default: break;  // padding (CSE_ALGO_NONE) or unknown: nothing written
    }
}

}  // namespace cse

using namespace cse;

extern "C" int cse_enhance_cells_generic(int n_fft, int64_t len, const cse_cell_t* cells,
                                         int64_t n_cells, const float* Y, const float* noise,
                                         const double* clean, float* y_out, int64_t out_len,
                                         float* g_out, double* sse, uint8_t* finite,
                                         cse_stream_t stream) {
    const char* name = "cse_enhance_cells_generic";
    CSE_CHECK_ARG(n_fft >= 64 && n_fft <= 4096 && n_fft % 2 == 0,
                  "%s: n_fft=%d (even, in [64, 4096])", name, n_fft);
    CSE_CHECK_ARG(cells && Y && noise, "%s: NULL cells/Y/noise", name);
    CSE_CHECK_ARG(len >= 1 && len < (1ll << 30) && n_cells >= 0 && n_cells < (1ll << 31),
                  "%s: len=%lld n_cells=%lld", name, (long long)len, (long long)n_cells);
    CSE_CHECK_ARG(!y_out || (out_len >= 0 && out_len <= len), "%s: out_len=%lld not in [0, len]",
                  name, (long long)out_len);
    if (n_cells == 0) return CSE_OK;
    Args a;
    a.len = len;
    a.cells = cells;
    a.n_cells = n_cells;
    a.Y = (const float2*)Y;
    a.noise = noise;
    a.clean = clean;
    a.y_out = y_out;
    a.out_len = y_out ? out_len : 0;
    a.g_out = g_out;
    a.sse = sse;
    a.finite = finite;
    int log2m = 0;  // M = n_fft / 2 = 2^log2m; -1: M not a power of two (direct DFT)
    while ((2 << log2m) < n_fft) ++log2m;
    if ((2 << log2m) != n_fft) log2m = -1;
    const int bytes = GenLds(n_fft).total;
    const void* fn = (const void*)enhance_generic_kernel;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
        ::cse::set_error("%s: cannot reserve %d bytes of LDS", name, bytes);
        return CSE_ELAUNCH;
    }
    hipLaunchKernelGGL(enhance_generic_kernel, dim3((unsigned)n_cells), dim3(GEN_NT), bytes,
                       (hipStream_t)stream, a, n_fft, log2m);
    CSE_CHECK_LAUNCH(name);
    return CSE_OK;
}
