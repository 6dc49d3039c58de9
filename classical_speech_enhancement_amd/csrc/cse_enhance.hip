// THE HOT PATH: fused per-cell gain recursion + ISTFT + score reductions.
//
// One grid cell = one call of the reference's alg_fn(noisy, sr, **params)
// (speech_enhancement_comparison.py:165) after STFT/noise estimation:
//   SS     spectral_subtractor.py:37-53   (elementwise)
//   Wiener wiener_filter.py:55-85         (decision-directed, serial over frames)
//   MMSE   mmse.py:65-109                 (DD + Ephraim-Malah MMSE-STSA gain)
//   OMLSA  advanced_mmse.py:82-127        (DD + LSA gain x speech-presence soft gain)
// followed by librosa.istft(S, length=len) (spectral_subtractor.py:55, wiener_filter.py:87,
// mmse.py:111, advanced_mmse.py:128) and the SNR numerator/denominator of
// evaluation_metrics.py:39-58 on the clipped waveform.
//
// Mapping (CDNA4, wave64).  A cell's spectrum row has B = M+1 bins (M = n_fft/2).
// L = M/16 lanes own one cell (16 lanes @512, 32 @1024), so a wave carries
// CPW = 64/L cells.  Each lane holds 16 bins (+ the Nyquist bin on lane 0):
// the serial-in-t recursion state lives in registers, the frames stream
// through.  Per frame the cell's 257/513 complex bins go through LDS twice
// (mirror pairing for the real-IFFT packing, one 16 x L transpose); the
// two length-16 DFT passes run in registers.  The inverse FFT's outputs land
// on lanes so that every lane owns output samples with fixed residues mod 32
// (mod 64 @1024): the overlap-add accumulator never leaves registers, and
// each frame retires its HOP finished samples straight into the SNR sums.
// Nothing per-frame touches HBM except the (L2-shared) Y/N rows.
#include "cse_common.hpp"
#include "cse_special.hpp"

namespace cse {

template <int NFFT>
struct Geo {
    static constexpr int M = NFFT / 2;        // complex IFFT length
    static constexpr int B = M + 1;           // bins
    static constexpr int L = M / 16;          // lanes per cell
    static constexpr int CPW = 64 / L;        // cells per wave
    static constexpr int SP = NFFT / 16;      // spacing of a lane's output samples
    static constexpr int SROW = M + 16;       // S row stride (complex), bank-shifted
    static constexpr int TROW = L + 1;        // transpose row stride (complex)
    static constexpr int TCELL = 16 * TROW;   // transpose block per cell
    static constexpr int REGION = (CPW * SROW > CPW * TCELL) ? CPW * SROW : CPW * TCELL;
};

struct Args {
    int64_t len;
    const cse_cell_t* cells;
    int64_t n_cells;
    const float2* Y;
    const float* noise;
    const double* clean;
    const float* inv_wss128;
    const float* inv_wss256;
    float* y_out;
    float* g_out;
    double* sse;
    uint8_t* finite;
};

// ---------------------------------------------------------------------------
// special functions (fp32), coefficients from tools/gen_special.py
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ float horner(const float (&c)[N], float t) {
    float acc = c[N - 1];
#pragma unroll
    for (int k = N - 2; k >= 0; --k) acc = fmaf(acc, t, c[k]);
    return acc;
}

__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// exp(-v/2)[(1+v)I0(v/2) + v I1(v/2)] for v in [1e-12, 80]
__device__ __forceinline__ float mmse_bracket_over_sqrtv_times(float v, float sqrtv) {
    // returns h(v) (not divided): v<=4 -> PA(t); v>4 -> sqrt(v)*PB(t(1/v))
    const float ta = (v - 2.0f) * 0.5f;
    const float u = fast_rcp(v);
    const float tb = (2.0f * u - (CSE_HB_U0 + CSE_HB_U1)) * (1.0f / (CSE_HB_U1 - CSE_HB_U0));
    const float pa = horner(CSE_HA, ta);
    const float pb = horner(CSE_HB, tb);
    return v <= 4.0f ? pa : sqrtv * pb;
}

// E1(v) = expn(1, v) for v in [1e-12, 80]; exp_v = exp(v) (shared with the SPP term)
__device__ __forceinline__ float expint_e1(float v, float exp_v) {
    const float small = -0.5772156649015329f - fast_log2(v) * kLn2 + v * horner(CSE_EIN, v);
    const float u = fast_rcp(v);
    const float te = (2.0f * u - (1.0f / 80.0f + 1.0f)) * (1.0f / (1.0f - 1.0f / 80.0f));
    const float large = fast_rcp(exp_v) * u * horner(CSE_E1L, te);
    return v <= 1.0f ? small : large;
}

// ---------------------------------------------------------------------------
// per-bin gains.  P = |Y|^2, N = noise PSD of this frame/bin.  gp/gm = the
// decision-directed state (previous gain / previous a-posteriori SNR).
// ---------------------------------------------------------------------------
// The decision-directed recursion only ever uses prev_gain**2 * prev_gamma
// (wiener_filter.py:133, mmse.py:82, advanced_mmse.py:215), so the carried
// state is that one product, rr = (G*G)*gamma, evaluated in the reference order.
__device__ __forceinline__ float gain_wiener(float P, float N, bool first, float& rr,
                                             float alpha, float gfloor) {
    const float n = fmaxf(N, 1e-10f);
    const float gam = fmaxf(__fdividef(P, n), 1e-10f);
    const float d = fmaxf(gam - 1.0f, 0.0f);
    float xi = first ? d : alpha * rr + (1.0f - alpha) * d;
    xi = fmaxf(xi, 1e-10f);
    const float g = fminf(fmaxf(__fdividef(xi, 1.0f + xi), gfloor), 1.0f);
    rr = (g * g) * gam;
    return g;
}

__device__ __forceinline__ float gain_mmse(float P, float N, bool first, float& rr,
                                           float alpha, float ksi_min, float gmin, float gmax) {
    const float n = fmaxf(N, 1e-12f);
    const float gam = fmaxf(__fdividef(P, n), 1e-12f);
    float xi;
    if (first)
        xi = fmaxf(gam - 1.0f, ksi_min);
    else
        xi = fmaxf(alpha * rr + (1.0f - alpha) * fmaxf(gam - 1.0f, 0.0f), ksi_min);
    const float v = fminf(fmaxf(__fdividef(xi * gam, 1.0f + xi), 1e-12f), 80.0f);
    const float sv = __builtin_sqrtf(v);
    const float h = mmse_bracket_over_sqrtv_times(v, sv);
    float g = (0.88622692545275801f * (sv * fast_rcp(gam + 1e-12f))) * h;
    if (__builtin_isnan(g)) g = gmin;
    if (__builtin_isinf(g)) g = g > 0.0f ? gmax : gmin;
    g = fminf(fmaxf(g, gmin), gmax);
    rr = (g * g) * gam;
    return g;
}

__device__ __forceinline__ float gain_omlsa(float P, float N, bool first, float& rr,
                                            float alpha, float ksi_min, float gfloor,
                                            float lg2_floor, float q, float vmax) {
    const float n = fmaxf(N, 1e-10f);
    const float gam = fmaxf(__fdividef(P, n), 1e-10f);
    float xi;
    if (first)
        xi = fmaxf(gam - 1.0f, ksi_min);
    else
        xi = fmaxf(alpha * rr + (1.0f - alpha) * fmaxf(gam - 1.0f, 0.0f), ksi_min);
    const float r = fast_rcp(1.0f + xi);
    const float v = fminf(fmaxf(xi * gam * r, 1e-12f), vmax);
    const float ev = fast_exp2(v * kLog2e);
    const float e1 = expint_e1(v, ev);
    // log2 of g_lsa = xi/(1+xi) * exp(0.5*E1); nan_to_num(nan->gf, +inf->1, -inf->gf)
    float lg = fast_log2(xi * r) + (0.5f * kLog2e) * e1;
    if (__builtin_isnan(lg)) lg = lg2_floor;
    if (__builtin_isinf(lg)) lg = lg > 0.0f ? 0.0f : lg2_floor;
    const float lam = r * ev;
    const float term = __fdividef(1.0f - q, q * lam + 1e-10f);
    const float p = fminf(fmaxf(fast_rcp(1.0f + term), 0.0f), 1.0f);
    const float g = fast_exp2(p * lg + (1.0f - p) * lg2_floor);
    const float G = fminf(fmaxf(g, gfloor), 1.0f);
    rr = (G * G) * gam;
    return G;
}

// ---------------------------------------------------------------------------
// XCD-aware wave order: blocks are dealt round-robin over the 8 XCDs, so give
// each XCD a contiguous slice of the (cost-sorted, group-clustered) cell list.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    const int q = nb / 8, r = nb % 8;
    const int xcd = b % 8, idx = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

struct LaneCell {
    bool valid;
    int algo;
    const float2* Y;
    const float* N;
    int64_t nstride;
    const double* clean;
    float* out;
    float* gout;
    float p[8];
};

// gain stage of one frame: S[j] = Y[k_j] * G(k_j) for the lane's 16 (+1) bins
template <int ALGO, int NFFT>
__device__ __forceinline__ void gain_stage(const LaneCell& c, int i, int t, float (&rr)[17],
                                           float lg2_floor, float q_spp, cf* sb) {
    using G = Geo<NFFT>;
    constexpr int M = G::M, L = G::L, B = G::B;
    const float2* Yt = c.Y + (int64_t)t * B;
    const float* Nt = c.N + (int64_t)t * c.nstride;
    const bool first = (t == 0);
#pragma unroll
    for (int j = 0; j < 17; ++j) {
        const int k = (j < 16) ? i + L * j : M;
        const float2 y = c.valid ? Yt[k] : make_float2(0.f, 0.f);
        const float nz = c.valid ? Nt[k] : 1.0f;
        const float P = y.x * y.x + y.y * y.y;
        float g;
        cf Sj;
        if (ALGO == CSE_ALGO_SS) {
            // spectral_subtractor.py:44-53: Ps = max(P - a N, b N); |S| = sqrt(Ps), phase of Y.
            // No eps floor here: the reference floors BEFORE fix_length, so its
            // zero-padded frames really subtract 0 (engine.noise_key).
            const float n = nz;
            const float ps = fmaxf(P - c.p[0] * n, c.p[1] * n);
            const float sp = __builtin_amdgcn_sqrtf(ps);
            if (P > 0.0f) {
                g = sp * __builtin_amdgcn_rsqf(P);
                Sj = cmk(y.x * g, y.y * g);
            } else {  // angle(0) = 0
                g = 0.0f;
                Sj = cmk(sp, 0.0f);
            }
        } else {
            if (ALGO == CSE_ALGO_WIENER)
                g = gain_wiener(P, nz, first, rr[j], c.p[0], c.p[1]);
            else if (ALGO == CSE_ALGO_MMSE)
                g = gain_mmse(P, nz, first, rr[j], c.p[0], c.p[1], c.p[2], c.p[3]);
            else
                g = gain_omlsa(P, nz, first, rr[j], c.p[0], c.p[1], c.p[2], lg2_floor, q_spp,
                               c.p[4]);
            Sj = cmk(y.x * g, y.y * g);
        }
        if (j < 16 || i == 0) {
            sb[k] = Sj;
            if (c.gout) c.gout[(int64_t)t * B + k] = g;
        }
    }
}

template <int NFFT, int HOP>
__device__ void run_cells(const Args& a, const LaneCell& c, int algo, cf* lds, const cf* tw1,
                          int64_t cell_idx) {
    using G = Geo<NFFT>;
    constexpr int M = G::M, L = G::L, B = G::B, SP = G::SP;
    constexpr int R = NFFT / HOP;       // frames overlapping one sample
    constexpr int F = 2 * HOP / SP;     // samples a lane retires per frame
    static_assert(F >= 2 && F <= 32 && (F % 2) == 0, "hop/n_fft combination");
    const int lane = threadIdx.x;
    const int cs = lane / L, i = lane % L;
    cf* sb = lds + cs * G::SROW;
    cf* tb = lds + cs * G::TCELL;
    const int64_t len = a.len;
    const int T = 1 + (int)(len / HOP);
    const int need = (int)((len + NFFT + HOP - 1) / HOP);
    const int nf = need < T ? need : T;
    const float* invw = (HOP == 128) ? a.inv_wss128 : a.inv_wss256;

    // lane-constant rotors: e^{2πi i/NFFT} (real-IFFT packing) and the window phase
    float bs, bc;
    sincospif(2.0f * (float)i / (float)NFFT, &bs, &bc);
    const cf base = cmk(bc, bs);
    const int b2 = (L == 16) ? i : (i & 15);
    const int h2 = (L == 16) ? 0 : (i >> 4);
    const int off = 2 * b2 + 32 * h2;  // lane's first sample offset inside a frame
    float wc[2], ws[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        float s_, c_;
        sincospif(2.0f * (float)(off + e) / (float)NFFT, &s_, &c_);
        wc[e] = (0.5f / NFFT) * c_;
        ws[e] = (0.5f / NFFT) * s_;
    }

    // decision-directed state: previous gain / previous a-posteriori SNR
    // (wiener_filter.py:115-116, mmse.py:62-63, advanced_mmse.py:198-199)
    // rr = prev_gain**2 * prev_gamma; only read from frame 1 on
    float rr[17];
#pragma unroll
    for (int j = 0; j < 17; ++j) rr[j] = 0.0f;
    const float lg2_floor = fast_log2(algo == CSE_ALGO_OMLSA ? c.p[2] : 1.0f);
    const float q_spp = fminf(fmaxf(c.p[3], 1e-3f), 1.0f - 1e-3f);

    float acc[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) acc[q] = 0.0f;
    double sse = 0.0;
    bool fin = true;

    for (int t = 0; t < nf + R - 1; ++t) {
        if (t < nf) {
            // ---------------- gain stage: S = Y * G straight into LDS ------
            __syncthreads();  // previous frame's transpose reads are done
            switch (algo) {
                case CSE_ALGO_SS:
                    gain_stage<CSE_ALGO_SS, NFFT>(c, i, t, rr, lg2_floor, q_spp, sb);
                    break;
                case CSE_ALGO_WIENER:
                    gain_stage<CSE_ALGO_WIENER, NFFT>(c, i, t, rr, lg2_floor, q_spp, sb);
                    break;
                case CSE_ALGO_MMSE:
                    gain_stage<CSE_ALGO_MMSE, NFFT>(c, i, t, rr, lg2_floor, q_spp, sb);
                    break;
                default:
                    gain_stage<CSE_ALGO_OMLSA, NFFT>(c, i, t, rr, lg2_floor, q_spp, sb);
                    break;
            }
            __syncthreads();

            // ---------------- pass 1: real-IFFT packing + DFT16 over j -----
            // Z'[k] = (X_k + X*_{M-k}) + i (X_k - X*_{M-k}) e^{2πi k/NFFT}
            cf z[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int k = i + L * j;
                cf A = sb[k];
                cf Bm = sb[M - k];
                if (k == 0) {  // irfft ignores the imaginary parts of DC and Nyquist
                    A.y = 0.0f;
                    Bm.y = 0.0f;
                }
                const cf Bc = cconj(Bm);
                const cf tw = cmul(base, cmk(Rot32::c[j], Rot32::s[j]));  // e^{2πi k/NFFT}
                z[j] = cadd(cadd(A, Bc), cmuli(cmul(csub(A, Bc), tw)));
            }
            idft16(z);
#pragma unroll
            for (int b = 1; b < 16; ++b) z[b] = cmul(z[b], tw1[b * L + i]);
            __syncthreads();  // all S reads done before the transpose overwrites
#pragma unroll
            for (int b = 0; b < 16; ++b) tb[b * G::TROW + i] = z[b];
            __syncthreads();

            // ---------------- pass 2: DFT over the lane index --------------
            cf v[16];
            if (L == 16) {
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = tb[i * G::TROW + r];
            } else {  // DFT32 = butterfly (lo +- hi) * W32^{r h}, then DFT16
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const cf lo = tb[b2 * G::TROW + r];
                    const cf hi = tb[b2 * G::TROW + r + 16];
                    const cf u = h2 ? csub(lo, hi) : cadd(lo, hi);
                    v[r] = h2 ? cmul(u, cmk(Rot32::c[r], Rot32::s[r])) : u;
                }
            }
            idft16(v);

            // ---------------- synthesis window (/n_fft) + overlap-add ------
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const int av = q >> 1, e = q & 1;
                const float ca = Rot32::c[(2 * av) & 31], sa = Rot32::s[(2 * av) & 31];
                const float w = 0.5f / NFFT - (ca * wc[e] - sa * ws[e]);
                const float x = e ? v[av].y : v[av].x;
                acc[q] = fmaf(x, w, acc[q]);
            }
        }

        // ---------------- retire HOP finished samples ----------------------
#pragma unroll
        for (int q = 0; q < F; ++q) {
            const int64_t o = (int64_t)t * HOP + SP * (q >> 1) + off + (q & 1) - NFFT / 2;
            if (c.valid && o >= 0 && o < len) {
                const float y = acc[q] * invw[o];
                fin = fin && __builtin_isfinite(y);
                if (c.out) c.out[o] = y;
                if (c.clean) {
                    const float yc = fminf(fmaxf(y, -1.0f), 1.0f);
                    const double d = c.clean[o] - (double)yc;
                    sse = fma(d, d, sse);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 32 - F; ++q) acc[q] = acc[q + F];
#pragma unroll
        for (int q = 32 - F; q < 32; ++q) acc[q] = 0.0f;
    }

    // ---------------- per-cell reductions over the cell's L lanes ----------
#pragma unroll
    for (int m = L / 2; m > 0; m >>= 1) sse += __shfl_xor(sse, m, 64);
    const unsigned long long bad = __ballot(!fin);
    const unsigned long long my = (bad >> (cs * L)) & ((1ull << L) - 1);
    if (i == 0 && c.valid) {
        if (a.sse) a.sse[cell_idx] = sse;
        if (a.finite) a.finite[cell_idx] = my == 0 ? 1 : 0;
    }
}

template <int NFFT>
__global__ void __launch_bounds__(64) enhance_kernel(Args a) {
    using G = Geo<NFFT>;
    __shared__ __attribute__((aligned(16))) cf lds[G::REGION];
    __shared__ __attribute__((aligned(16))) cf tw1[16 * G::L];
    const int lane = threadIdx.x;
    // pass-1 twiddles e^{2πi i b/M}, [b][i]
    for (int e = lane; e < 16 * G::L; e += 64) {
        const int b = e / G::L, ii = e % G::L;
        double s, c;
        sincospi(2.0 * (double)(ii * b) / (double)G::M, &s, &c);
        tw1[e] = cmk((float)c, (float)s);
    }
    __syncthreads();
    const int wave = xcd_remap(blockIdx.x, gridDim.x);
    const int cs = lane / G::L;
    const int64_t first = (int64_t)wave * G::CPW;
    const int64_t ci = first + cs;
    LaneCell c;
    const cse_cell_t* cp = a.cells + (ci < a.n_cells ? ci : first);
    c.algo = cp->algo;
    c.valid = (ci < a.n_cells) && c.algo >= 0;
    if (!c.valid) c.algo = CSE_ALGO_NONE;
    c.Y = a.Y + cp->y_offset;
    c.N = a.noise + cp->noise_offset;
    c.nstride = cp->noise_stride;
    c.clean = (c.valid && cp->clean_offset >= 0 && a.clean) ? a.clean + cp->clean_offset : nullptr;
    c.out = (c.valid && cp->out_offset >= 0 && a.y_out) ? a.y_out + cp->out_offset : nullptr;
    c.gout = (c.valid && cp->gain_offset >= 0 && a.g_out) ? a.g_out + cp->gain_offset : nullptr;
#pragma unroll
    for (int k = 0; k < 8; ++k) c.p[k] = cp->param[k];
    // hop and algorithm are the first slot's (the host packs equal hop/algo per
    // wave); a slot that disagrees is skipped (finite = 0 never written: host
    // validates packing before launch).
    const int hop = __builtin_amdgcn_readfirstlane(a.cells[first].hop);
    const int algo = __builtin_amdgcn_readfirstlane(a.cells[first].algo);
    if (c.valid && (cp->hop != hop || c.algo != algo)) c.valid = false;
    if (hop == 128)
        run_cells<NFFT, 128>(a, c, algo, lds, tw1, ci);
    else if (hop == 256)
        run_cells<NFFT, 256>(a, c, algo, lds, tw1, ci);
}

}  // namespace cse

using namespace cse;

extern "C" int cse_enhance_cells(int n_fft, int64_t len, const cse_cell_t* cells, int64_t n_cells,
                                 const float* Y, const float* noise, const double* clean,
                                 const float* inv_wss128, const float* inv_wss256, float* y_out,
                                 float* g_out, double* sse, uint8_t* finite,
                                 cse_stream_t stream) {
    CSE_CHECK_ARG(n_fft == 512 || n_fft == 1024, "cse_enhance_cells: n_fft=%d (512|1024)", n_fft);
    CSE_CHECK_ARG(cells && Y && noise, "cse_enhance_cells: NULL cells/Y/noise");
    CSE_CHECK_ARG(len >= 1 && n_cells >= 0, "cse_enhance_cells: len=%lld n_cells=%lld",
                  (long long)len, (long long)n_cells);
    if (n_cells == 0) return CSE_OK;
    Args a;
    a.len = len;
    a.cells = cells;
    a.n_cells = n_cells;
    a.Y = (const float2*)Y;
    a.noise = noise;
    a.clean = clean;
    a.inv_wss128 = inv_wss128;
    a.inv_wss256 = inv_wss256;
    a.y_out = y_out;
    a.g_out = g_out;
    a.sse = sse;
    a.finite = finite;
    const int cpw = CSE_CELLS_PER_WAVE(n_fft);
    const int64_t waves = (n_cells + cpw - 1) / cpw;
    CSE_CHECK_ARG(waves < (1ll << 31), "cse_enhance_cells: too many cells");
    if (n_fft == 512)
        hipLaunchKernelGGL(enhance_kernel<512>, dim3((unsigned)waves), dim3(64), 0,
                           (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(enhance_kernel<1024>, dim3((unsigned)waves), dim3(64), 0,
                           (hipStream_t)stream, a);
    CSE_CHECK_LAUNCH("cse_enhance_cells");
    return CSE_OK;
}
