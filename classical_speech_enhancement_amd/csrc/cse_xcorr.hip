// Alignment lag of finalize_enhanced (speech_enhancement_comparison.py:38-69,
// 92-106): for every cell, the cross-correlation of the mean-removed first
// n = min(len, 2 s) samples of the clean reference and of the enhanced output,
//   c(l) = sum_m r0[m + l] s0[m],   |l| <= max_lag (0.1 s),
// scipy.signal.correlate(r0, s0, 'full') restricted to the kept lags (:50-58),
// and lag = the first l of maximal c (np.argmax over ascending lags, :60).
//
// Blocked FFT correlation.  The output head e[0, n) is cut into blocks of
// XB = 4992 samples (7 blocks for 2 s at 16 kHz); block b correlates with the
// clean window r0[bXB - max_lag, bXB + XB + max_lag) (<= XN = 8192 samples, so the
// circular correlation of length XN has no wrap-around in the kept lags):
//   C(f) = sum_b R_b(f) conj(S_b(f)),   c_raw = irfft(C) on lags 0..2 max_lag,
// one inverse transform per cell.  R_b (the clean side) is computed once per
// signal by xcorr_prep_kernel.  The mean of e enters as
//   c(l) = c_raw(l) - mean(e) * W(l),  W(l) = sum of r0 over the overlap of l.
// Real transforms of XN points are complex 4096-point FFTs (radix-16
// Stockham, three passes through 32 KiB of LDS) with the usual even/odd
// packing.
//
// Exactness: the fp32 FFT value of every lag is within a small multiple of
// 1e-6 ||r0|| ||e|| of the exact one (e the raw head, mean included: the FFT
// sees it before the mean correction), so every lag within
// delta = 2e-5 ||r0|| ||e|| of the fp32 maximum is re-evaluated by a direct
// fp64 sum and the lag is chosen among those (ties -> smallest lag, like
// np.argmax).  The candidates are marked in an LDS bitmap over the lags and
// re-evaluated in ascending lag order, however many there are: up to XCAND
// one block sum each, more (a flat correlation, status CSE_XCORR_FLAT) XG
// lags per pass over the head.  An all-zero head is lag -max_lag directly
// (every correlation value is 0: np.argmax's first index).
#include "cse_common.hpp"

#include <type_traits>

namespace cse {

constexpr int XN = 8192;      // real transform length of one block correlation
constexpr int XH = XN / 2;    // complex FFT length
constexpr int XB = XN - 2 * 1600;  // output samples per block: the 0.1-s lags of 16 kHz fill XN
constexpr int XT = 256;       // threads per workgroup
constexpr int XCAND = 64;     // more fp64 candidates than this: status FLAT
constexpr int XLAGS = 2 * ((XN - XB) / 2) + 1;  // most lags a cell has (max_lag <= 1600)
constexpr int XWORDS = (XLAGS + 31) / 32;        // candidate bitmap words
constexpr int XHP = XH + XH / 16;  // LDS FFT buffer (room for the 1-in-16 padded layout)
// Two padded LDS layouts of the 4096 points.  px16 (one pad slot after every
// 16 points) is what the first Stockham pass stores: 16 consecutive points per
// lane, lane stride 17 x 8 B, so the 16 lanes of a ds_write_b64 group hit
// distinct banks (unpadded: a 32-way conflict).  Every other access runs over
// consecutive points, 32 lanes per ds_read_b64 group, and there px16's pad
// wraps the group's last lane onto its first lane's banks (a 2-way conflict on
// every read: r03's 1.16 conflict cycles per LDS instruction); px32 (one pad
// slot per 32 points) keeps such a group contiguous.  The passes convert: the
// first pass reads px32 and writes px16, the second reads px16 and writes
// px32, everything else is px32.
template <int PAD>
__device__ __forceinline__ int pxl(int p) { return p + (PAD == 16 ? (p >> 4) : (p >> 5)); }
__device__ __forceinline__ int px(int p) { return pxl<32>(p); }
constexpr int XR = XH / 16 + XH / 16 / 32;  // px32 stride of 256 points: 264
// __launch_bounds__' second argument is waves per SIMD; with XT = 256 (one wave
// per SIMD per workgroup) that equals workgroups per CU
#ifndef CSE_XC_WG_PER_CU
#define CSE_XC_WG_PER_CU 3   // 168 VGPRs + 72 B spill: 4% faster than 2 (192, no spill); 4 spills 240 B
#endif

// one radix-16 Stockham pass of stride NS (compile-time, so every padded
// address is a constant offset from one per-lane base), reading layout PI and
// writing layout PO
template <int DIR, int NS, int PI, int PO>
__device__ __forceinline__ void fft4096_pass(cf* buf) {
    const int j = threadIdx.x;
    cf v[16];
    const int pj = pxl<PI>(j);  // point j + 256 r sits at pj + (256 + 256/PI) r
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = buf[pj + r * (XH / 16 + XH / 16 / PI)];
    const int k = j % NS;
    if (NS > 1) {
        // w^r, w = e^{DIR 2πi k/(16 NS)}: one accurate sincos, then a product
        // chain (|error| <= 15 ulp, far inside the candidate margin)
        // (the argument is hidden from the optimiser: hoisting the chain out of
        // the block loop would pin 2 x 30 VGPRs)
        float s, c, arg = (float)(DIR * 2 * k) / (float)(NS * 16);
        asm volatile("" : "+v"(arg));
        sincospif(arg, &s, &c);
        const cf w = cmk(c, s);
        cf wr = w;
#pragma unroll
        for (int r = 1; r < 16; ++r) {
            v[r] = cmul(v[r], wr);
            wr = cmul(wr, w);
        }
    }
    if (DIR > 0) {
        idft16(v);
    } else {  // forward = conj(inverse(conj(v)))
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r].y = -v[r].y;
        idft16(v);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r].y = -v[r].y;
    }
    __syncthreads();
    // pxl(base + r NS) = pxl(base) + r NS + (r NS) / PO: base's low part (k < NS,
    // or base = 16 j at NS = 1) never carries into the pad index
    const int base = (j / NS) * NS * 16 + k;
    const int pb = pxl<PO>(base);
#pragma unroll
    for (int r = 0; r < 16; ++r) buf[pb + r * NS + (r * NS) / PO] = v[r];
    __syncthreads();
}

// forward (DIR = -1) / inverse (DIR = +1, unnormalised) 4096-point FFT in LDS,
// radix-16 Stockham (Govindaraju et al. 2008 form): 3 passes, natural order out
template <int DIR>
__device__ __forceinline__ void fft4096(cf* buf) {
    fft4096_pass<DIR, 1, 32, 16>(buf);
    fft4096_pass<DIR, 16, 16, 32>(buf);
    fft4096_pass<DIR, 256, 32, 32>(buf);
}

// X(f), f = 0..XH, of the real sequence x[2m] + i x[2m+1] = buf[m] after fft4096<-1>:
// X(f) = E + e^{-2πi f/XN} O,  E = (Z_f + conj Z_{XH-f})/2,  O = (Z_f - conj Z_{XH-f})/(2i)
// tw = e^{-2πi f/XN} is passed in (thread-owned bins f = tid + 256 r share
// e^{-2πi tid/XN} and differ by the compile-time rotor e^{-2πi r/32})
__device__ __forceinline__ cf rfft_bin(const cf* buf, int f, cf tw) {
    if (f == XH) return cmk(buf[0].x - buf[0].y, 0.0f);  // px(0) = 0
    const cf z = buf[px(f)];
    const cf w = buf[px((XH - f) & (XH - 1))];
    const cf e = cmk(0.5f * (z.x + w.x), 0.5f * (z.y - w.y));
    const cf o = cmk(0.5f * (z.y + w.y), -0.5f * (z.x - w.x));
    return cadd(e, cmul(tw, o));
}

// the same from the two loaded points z = Z_f, w = Z_{(XH - f) mod XH}
__device__ __forceinline__ cf rfft_pair(cf z, cf w, cf tw) {
    const cf e = cmk(0.5f * (z.x + w.x), 0.5f * (z.y - w.y));
    const cf o = cmk(0.5f * (z.y + w.y), -0.5f * (z.x - w.x));
    return cadd(e, cmul(tw, o));
}

// padded LDS index of the mirror (XH - f) mod XH of the lane's bin f = t + 256 r:
// t > 0: (256 - t) + 256 (15 - r); t = 0: 256 (16 - r) mod XH.  mirror_base(t)
// + XR (15 - r) covers both, except (t, r) = (0, 0) -> 0 (see mirror_at)
__device__ __forceinline__ int mirror_base(int t) { return t == 0 ? XR : px(256 - t); }
__device__ __forceinline__ int mirror_at(int mb, int t, int r) {
    const int q = mb + XR * (15 - r);
    return r == 0 ? (t == 0 ? 0 : q) : q;
}

__device__ __forceinline__ cf bin_rotor(int f) {
    float s, c;
    sincospif(-(float)(2 * f) / (float)XN, &s, &c);
    return cmk(c, s);
}

// per-lane sum of ld(q), q = tid, tid + XT, ... < n, in ascending q, with 8 loads
// in flight (a plain strided loop waits out one memory latency per element)
template <typename Load>
__device__ __forceinline__ double strided_sum8(int n, Load ld) {
    double acc = 0.0;
    for (int q = threadIdx.x; q < n; q += 8 * XT) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = ld(min(q + u * XT, n - 1));
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (q + u * XT < n) acc += v[u];
    }
    return acc;
}

// ---------------------------------------------------------------------------
// per signal: R_b for every block (blockIdx.x < nb), and (blockIdx.x == nb)
// r0 in fp64, W(l), the zero-padding energies Z(l) and ||r0||^2
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(XT) xcorr_prep_kernel(const double* __restrict__ clean,
                                                         int64_t len, int n, int max_lag, int nb,
                                                         float2* __restrict__ R,
                                                         double* __restrict__ r0buf,
                                                         double* __restrict__ W,
                                                         double* __restrict__ Z,
                                                         double* __restrict__ rnorm) {
    __shared__ cf buf[XHP];
    __shared__ double red[XT];
    const int sig = blockIdx.y, tid = threadIdx.x;
    const double* c = clean + (int64_t)sig * len;
    // mean of clean[0, n)
    const double acc = strided_sum8(n, [&](int q) { return c[q]; });
    red[tid] = acc;
    __syncthreads();
    for (int s = XT / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double mu = red[0] / n;
    __syncthreads();
    const int b = blockIdx.x;
    if (b < nb) {
        // window r0[b XB - max_lag + v], v < XB + 2 max_lag, zero elsewhere
        // (all 32 loads of a lane issued before the first use; clamped indices)
        double xv[32];
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const int v = 2 * tid + (u & 1) + 2 * XT * (u >> 1);
            const int q = b * XB - max_lag + v;
            xv[u] = c[min(max(q, 0), n - 1)];
        }
#pragma unroll
        for (int u = 0; u < 32; u += 2) {
            float x2[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int v = 2 * tid + e + 2 * XT * (u >> 1);
                const int q = b * XB - max_lag + v;
                x2[e] = (v < XB + 2 * max_lag && q >= 0 && q < n) ? (float)(xv[u + e] - mu) : 0.0f;
            }
            buf[px(tid + XT * (u >> 1))] = cmk(x2[0], x2[1]);
        }
        __syncthreads();
        fft4096<-1>(buf);
        float2* out = R + ((int64_t)sig * nb + b) * (XH + 1);
        for (int f = tid; f <= XH; f += XT) {
            const cf x = rfft_bin(buf, f, bin_rotor(f));
            out[f] = make_float2(x.x, x.y);
        }
        return;
    }
    // block nb: fp64 tables r0, ||r0||^2, W, Z
    double* r0 = r0buf + (int64_t)sig * n;
    double sq = 0.0, tp = 0.0;  // ||r0||^2 and sum(r0) partials
    for (int q = tid; q < n; q += 8 * XT) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = c[min(q + u * XT, n - 1)] - mu;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (q + u * XT < n) {
                r0[q + u * XT] = v[u];
                sq += v[u] * v[u];
                tp += v[u];
            }
    }
    red[tid] = sq;
    __syncthreads();
    for (int s = XT / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double r2 = red[0];
    __syncthreads();
    red[tid] = tp;
    __syncthreads();
    for (int s = XT / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    const double total = red[0];
    if (tid == 0) rnorm[sig] = r2;
    // W(l) = total - sum_{q < l} r0[q], W(-l) = total - sum_{q >= n - l} r0[q] and
    // Z(+-l) = the clean energy of the l padded head / tail samples, l = 1..max_lag:
    // four prefix sums, a chunk of CH lags per lane plus a block scan of the chunk
    // sums (a single lane walking max_lag dependent steps took ~0.3 ms)
    double* sc = (double*)buf;  // 4 x XT scan slots in the idle FFT buffer
    const int CH = (max_lag + XT - 1) / XT;
    const int l0 = tid * CH + 1, l1 = min(l0 + CH - 1, max_lag);
    double p[4] = {0.0, 0.0, 0.0, 0.0};
    for (int l = l0; l <= l1; ++l) {
        p[0] += c[l - 1] - mu;  // = r0[l - 1]
        p[1] += c[n - l] - mu;
        p[2] += c[l - 1] * c[l - 1];
        p[3] += c[len - l] * c[len - l];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) sc[k * XT + tid] = p[k];
    __syncthreads();
    for (int off = 1; off < XT; off <<= 1) {  // inclusive Hillis-Steele scan
        double t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = tid >= off ? sc[k * XT + tid - off] : 0.0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k) sc[k * XT + tid] += t[k];
        __syncthreads();
    }
    double run[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) run[k] = sc[k * XT + tid] - p[k];  // exclusive
    double* w = W + (int64_t)sig * (2 * max_lag + 1) + max_lag;
    double* z = Z + (int64_t)sig * (2 * max_lag + 1) + max_lag;
    if (tid == 0) {
        w[0] = total;
        z[0] = 0.0;
    }
    for (int l = l0; l <= l1; ++l) {
        run[0] += c[l - 1] - mu;
        run[1] += c[n - l] - mu;
        run[2] += c[l - 1] * c[l - 1];
        run[3] += c[len - l] * c[len - l];
        w[l] = total - run[0];
        w[-l] = total - run[1];
        z[l] = run[2];
        z[-l] = run[3];
    }
}

// ---------------------------------------------------------------------------
// per cell: the lag (see the file comment)
// ---------------------------------------------------------------------------
struct XcArgs {
    const float* head;      // output heads, cell c's at head + head_offset[c]
    const int64_t* head_offset;
    const int* sig_of;      // [n_cells]
    const float2* R;
    const double* r0buf;
    const double* W;
    const double* Z;
    const double* rnorm;
    int n, max_lag, nb;
    int* lag;
    double* zero_energy;
    int* status;
    float* corr;            // optional [n_cells][2 max_lag + 1]
};

__device__ __forceinline__ double block_sum(double v, double* red) {
    const int tid = threadIdx.x;
    __syncthreads();
    red[tid] = v;
    __syncthreads();
    for (int s = XT / 2; s > 0; s >>= 1) {
        if (tid < s) red[tid] += red[tid + s];
        __syncthreads();
    }
    return red[0];
}

// LDS of the lag kernel
struct XcLds {
    cf buf[XHP];
    double red[XT];
    float rv[XT];
    int ri[XT];
    unsigned cbits[XWORDS];  // candidate lags k, bit k & 31 of word k >> 5
    int ncand;
};

struct XcPass {
    double s1, s2;  // sum and energy of the head as fed (pass 1: centred)
    int kmax;       // the fp32 argmax (ascending-lag first maximum)
    int nc;         // lags within the margin, marked in cbits
    int early;      // 0, or the status of a head whose correlation is the same at every lag
};

// One blocked-FFT correlation pass of one cell (see the file comment): head e,
// its signal's clean spectra Rs, W(l) row Ws and ||r0||^2 rn; corr_row is the
// cell's optional corr output row.
// CENTRED = false: the raw head, mean corrected afterwards (c = c_raw - mu W),
// fp32 error ~ ||r0|| ||e||.  CENTRED = true: the head minus its mean mu (as
// two floats: (t - hi) - lo is within 2^-23 |t - mu| of the centred sample),
// no correction, fp32 error ~ ||r0|| ||e - mu||.
template <bool CENTRED>
__device__ __forceinline__ void xcorr_pass(const float* e, const float2* Rs, const double* Ws,
                                           double rn, int n, int L, int nb, float* corr_row,
                                           XcLds& S, double mu, XcPass& o) {
    cf* buf = S.buf;
    double* red = S.red;
    float* rv = S.rv;
    int* ri = S.ri;
    unsigned* cbits = S.cbits;
    const int tid = threadIdx.x;
    const float mu_hi = CENTRED ? (float)mu : 0.0f;
    const float mu_lo = CENTRED ? (float)(mu - (double)mu_hi) : 0.0f;
    const cf rot_tid = bin_rotor(tid);
    const int pt = px(tid), mb = mirror_base(tid);
    // raw buffer over e[0, n) (CDNA buffer resource, word 3 = 0x00020000:
    // 32-bit data format, no swizzle); every offset issued lies inside it
    const __amdgpu_buffer_rsrc_t erc =
        __builtin_amdgcn_make_buffer_rsrc((void*)e, (short)0, 4 * n, 0x00020000);
    cf C[8], Cm[8];  // C(f), C(XH - f)
    cf Ch = cmk(0.0f, 0.0f);  // C(XH/2), thread 0
#pragma unroll
    for (int r = 0; r < 8; ++r) C[r] = Cm[r] = cmk(0.0f, 0.0f);
    double s1 = 0.0, s2 = 0.0;
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        // samples v = 2 tid + (u & 1) + 512 (u >> 1) of the block; v < XB needs
        // u >> 1 <= 9 (and tid < 192 at 9).  In the last block the offsets are
        // clamped to the last sample and q >= n is masked to 0 here: the buffer
        // range check is not relied on (it misses a constant part the compiler
        // folds into the instruction's immediate offset, and a fused 8-byte
        // sample pair can straddle n).  Blocks before the last lie inside
        // [0, n) and keep the fused loads.
        float x[20];
        auto load_block = [&](auto last) {
#pragma unroll
            for (int u = 0; u < 20; ++u) {
                const int v = 2 * tid + (u & 1) + 2 * XT * (u >> 1);
                const int q = b * XB + v;
                const int qc = decltype(last)::value ? min(q, n - 1) : q;
                const float t = __builtin_bit_cast(  // the builtin returns the raw 32 bits
                    float, __builtin_amdgcn_raw_buffer_load_b32(erc, 4 * qc, 0, 0));
                const float tc = CENTRED ? (t - mu_hi) - mu_lo : t;
                x[u] = ((u < 18 || v < XB) && (!decltype(last)::value || q < n)) ? tc : 0.0f;
            }
        };
        if (b + 1 < nb)
            load_block(std::false_type());
        else
            load_block(std::true_type());
#pragma unroll
        for (int u = 0; u < 20; ++u) {
            s1 += (double)x[u];
            s2 += (double)x[u] * (double)x[u];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
            buf[pt + XR * r] = r < 10 ? cmk(x[2 * r], x[2 * r + 1]) : cmk(0.0f, 0.0f);
        // R_b at the lane's bins is issued before the transform and consumed after it
        const float2* Rb = Rs + (int64_t)b * (XH + 1);
        float2 rr[8], rm[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            rr[r] = Rb[tid + XT * r];
            rm[r] = Rb[XH - tid - XT * r];  // thread 0, r = 0: the Nyquist bin
        }
        const float2 rh = Rb[XH / 2];
        __syncthreads();
        fft4096<-1>(buf);
        cf rt = rot_tid;  // hidden: the 8 derived rotors must not live across the FFT
        asm volatile("" : "+v"(rt.x), "+v"(rt.y));
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            // e^{-2πi (tid + 256 r)/8192} = rot_tid * e^{-2πi r/32}
            const cf z = buf[pt + XR * r], w = buf[mirror_at(mb, tid, r)];
            const cf e = cmk(0.5f * (z.x + w.x), 0.5f * (z.y - w.y));
            const cf o = cmk(0.5f * (z.y + w.y), -0.5f * (z.x - w.x));
            const cf wo = cmul(cmul(rt, cmk(Rot32::c[r], -Rot32::s[r])), o);
            const cf sf = cadd(e, wo);                      // X(f)
            const cf sg = cmk(e.x - wo.x, wo.y - e.y);      // X(XH - f) = conj(E - w O)
            // R conj(S)
            C[r].x += rr[r].x * sf.x + rr[r].y * sf.y;
            C[r].y += rr[r].y * sf.x - rr[r].x * sf.y;
            Cm[r].x += rm[r].x * sg.x + rm[r].y * sg.y;
            Cm[r].y += rm[r].y * sg.x - rm[r].x * sg.y;
        }
        if (tid == 0) {  // X(XH/2) = conj(Z_{XH/2})
            const cf z = buf[px(XH / 2)];
            Ch.x += rh.x * z.x - rh.y * z.y;
            Ch.y += rh.y * z.x + rh.x * z.y;
        }
        __syncthreads();
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    o.s1 = s1;
    o.s2 = s2;
    o.early = 0;
    if (!CENTRED && (!__builtin_isfinite(s1) || !__builtin_isfinite(s2) || !__builtin_isfinite(rn))) {
        o.early = CSE_XCORR_NONFINITE;
        return;
    }
    // an all-zero head (pass 0), a constant one (pass 1: the centred head is
    // 0) or a constant clean head (r0 = 0): every c(l) is 0 exactly
    if (s2 == 0.0 || rn == 0.0) {
        o.early = CSE_XCORR_FLAT;
        return;
    }
    const double mw = CENTRED ? 0.0 : s1 / n;  // the mean correction's weight
    // inverse real transform: Zi(f) = (C_f + conj C_{XH-f}) + i e^{+2πi f/XN} (C_f - conj C_{XH-f});
    // with ev, od those two terms, Zi(XH - f) = conj(ev - i t), t = e^{+2πi f/XN} od,
    // and Zi(XH/2) = 2 conj(C_{XH/2}): every point from the lane's own pairs
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const cf ev = cmk(C[r].x + Cm[r].x, C[r].y - Cm[r].y);
        const cf od = cmk(C[r].x - Cm[r].x, C[r].y + Cm[r].y);
        const cf tw = cmul(rot_tid, cmk(Rot32::c[r], -Rot32::s[r]));  // e^{-2πi f/XN}
        const cf t = cmul(cmk(tw.x, -tw.y), od);                       // e^{+2πi f/XN} od
        buf[pt + XR * r] = cmk(ev.x - t.y, ev.y + t.x);                // ev + i t
        if (r > 0 || tid > 0)  // f = 0: its mirror is XH, not an input point
            buf[mirror_at(mb, tid, r)] = cmk(ev.x + t.y, t.x - ev.y);  // conj(ev - i t)
    }
    if (tid == 0) buf[px(XH / 2)] = cmk(2.0f * Ch.x, -2.0f * Ch.y);
    __syncthreads();
    fft4096<1>(buf);

    // c(l) = c_raw(l) - mu W(l); c_raw[k] = (k even ? Re : Im) buf[k/2] / XN, k = l + L
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int k = tid; k <= 2 * L; k += XT) {
        const cf z = buf[px(k >> 1)];
        const float craw = ((k & 1) ? z.y : z.x) * (1.0f / XN);
        const float v = craw - (float)(mw * Ws[k]);
        if (corr_row) corr_row[k] = v;
        if (v > best) {  // k ascending per thread: first max kept
            best = v;
            bi = k;
        }
    }
    rv[tid] = best;
    ri[tid] = bi;
    __syncthreads();
    for (int s = XT / 2; s > 0; s >>= 1) {
        if (tid < s) {
            const float v2 = rv[tid + s];
            const int i2 = ri[tid + s];
            if (v2 > rv[tid] || (v2 == rv[tid] && i2 < ri[tid])) {
                rv[tid] = v2;
                ri[tid] = i2;
            }
        }
        __syncthreads();
    }
    const float cmax = rv[0];
    o.kmax = ri[0];
    // the fp32 FFT works on the head as it was fed (pass 0: the raw head, mean
    // included: c = c_raw - mu W), so its error scales with ||r0|| ||fed||,
    // not ||r0|| ||e - mu||: a head with a large DC and little variance (a DC
    // head: every true c(l) is 0) needs the fed energy s2 here, or fp32 noise
    // picks the lag
    const float delta = (float)(2e-5 * sqrt(rn * s2)) + 1e-30f;
    if (tid == 0) S.ncand = 0;
    for (int w = tid; w < XWORDS; w += XT) cbits[w] = 0u;
    __syncthreads();
    for (int k = tid; k <= 2 * L; k += XT) {
        const cf z = buf[px(k >> 1)];
        const float v = ((k & 1) ? z.y : z.x) * (1.0f / XN) - (float)(mw * Ws[k]);
        if (v >= cmax - delta) {
            atomicOr(&cbits[k >> 5], 1u << (k & 31));
            atomicAdd(&S.ncand, 1);
        }
    }
    __syncthreads();
    o.nc = S.ncand;
}

// the centred pass out of line: it runs only for flat cells, and inlined beside
// pass 0 it cost the common path 30-40 spilled registers
__device__ __noinline__ void xcorr_pass_centred(const float* e, const float2* Rs, const double* Ws,
                                                double rn, int n, int L, int nb, float* corr_row,
                                                XcLds& S, double mu, XcPass& o) {
    xcorr_pass<true>(e, Rs, Ws, rn, n, L, nb, corr_row, S, mu, o);
}

__global__ void __launch_bounds__(XT, CSE_XC_WG_PER_CU) xcorr_lag_kernel(XcArgs a) {
    __shared__ XcLds S;
    cf* buf = S.buf;
    double* red = S.red;
    unsigned* cbits = S.cbits;
    const int cell = blockIdx.x, tid = threadIdx.x;
    const int sig = a.sig_of[cell];
    const float* e = a.head + a.head_offset[cell];
    const int n = a.n, L = a.max_lag;
    // Pass 0 transforms the raw head (its mean is known only once every block
    // is read).  When more than XCAND lags fall inside its margin (a head with
    // a large mean and little else: a near-DC output, a flat correlation),
    // pass 1 transforms the centred head e - mu, whose margin shrinks with the
    // head's variance: the same lags, a handful of fp64 re-evaluations instead
    // of one per lag (r04 re-evaluated up to 3,201 lags in fp64 serially in
    // this workgroup: 43.6 ms for a DC-like head).
    const float2* Rs = a.R + (int64_t)sig * a.nb * (XH + 1);
    const double* Ws = a.W + (int64_t)sig * (2 * L + 1);
    const double rn = a.rnorm[sig];
    float* corr_row = a.corr ? a.corr + (int64_t)cell * (2 * L + 1) : nullptr;
    XcPass o;
    xcorr_pass<false>(e, Rs, Ws, rn, n, L, a.nb, corr_row, S, 0.0, o);
    const double mu = o.s1 / n;
    int status = CSE_XCORR_OK;
    if (!o.early && o.nc > XCAND) {
        status = CSE_XCORR_FLAT;
        __syncthreads();  // every thread has read ncand and the buffer
        xcorr_pass_centred(e, Rs, Ws, rn, n, L, a.nb, corr_row, S, mu, o);
    }
    if (o.early) {
        // the correlation is the same at every lag, so np.argmax (:60) takes
        // the first kept lag, -max_lag (max_lag < n: -max_lag is kept):
        //  - NONFINITE: a NaN or inf in either head makes the mean-removed
        //    head (:48-49) NaN (or -inf and NaN) everywhere, scipy's FFT
        //    correlation NaN at every lag, and np.argmax of an all-NaN vector
        //    0.  The cell is still shifted and length-matched; the finiteness
        //    check comes after (:100-103), so a non-finite sample that the
        //    shift drops does not skip the cell (the enhance kernel's lag-l
        //    rescoring decides);
        //  - FLAT: every c(l) is 0 (no candidate re-evaluation: all 2 L + 1 tie).
        const bool nonfinite = o.early == CSE_XCORR_NONFINITE;
        if (a.corr)
            for (int k = tid; k <= 2 * L; k += XT)
                a.corr[(int64_t)cell * (2 * L + 1) + k] = nonfinite ? __builtin_nanf("") : 0.0f;
        if (tid == 0) {
            a.lag[cell] = -L;
            a.zero_energy[cell] = a.Z[(int64_t)sig * (2 * L + 1)];
            a.status[cell] = o.early;
        }
        return;
    }
    const int nc = o.nc;
    const int kmax = o.kmax;
    int kbest = kmax;
    if (nc > XCAND) {
        // a flat correlation (up to 2 L + 1 candidates): XG lags per pass over
        // the head, each thread's samples m = tid + XT i read once for all of
        // them, the XG sums reduced together through the idle FFT buffer
        // (one pass per XG candidates instead of one pass and a block sum
        // each: r03's uncapped form took ~50 ms for 3,201 candidates)
        constexpr int XG = 8;
        const double* r0 = a.r0buf + (int64_t)sig * n;
        double* rd = (double*)buf;  // [XG][XT]
        double bestd = -INFINITY;
        kbest = 0x7fffffff;
        const int nw = (2 * L + 1 + 31) >> 5;
        int w = 0;
        unsigned bits = cbits[0];
        for (;;) {
            int ks[XG], ng = 0;
            while (ng < XG) {  // the next XG candidates in ascending lag order (uniform)
                while (!bits && ++w < nw) bits = cbits[w];
                if (!bits) break;
                ks[ng++] = 32 * w + __builtin_ctz(bits);
                bits &= bits - 1u;
            }
            if (ng == 0) break;
            double acc[XG];
#pragma unroll
            for (int g = 0; g < XG; ++g) acc[g] = 0.0;
            for (int m = tid; m < n; m += XT) {
                const double ev = (double)e[m] - mu;
#pragma unroll
                for (int g = 0; g < XG; ++g) {
                    const int q = m + (g < ng ? ks[g] : L) - L;  // r0[m + l] inside [0, n)
                    if (g < ng && q >= 0 && q < n) acc[g] += r0[q] * ev;
                }
            }
            __syncthreads();
#pragma unroll
            for (int g = 0; g < XG; ++g) rd[g * XT + tid] = acc[g];
            __syncthreads();
            for (int s = XT / 2; s > 0; s >>= 1) {
                if (tid < s)
#pragma unroll
                    for (int g = 0; g < XG; ++g) rd[g * XT + tid] += rd[g * XT + tid + s];
                __syncthreads();
            }
            for (int g = 0; g < ng; ++g) {
                const double v = rd[g * XT];
                if (v > bestd) {  // ascending lags: the first maximum is kept
                    bestd = v;
                    kbest = ks[g];
                }
            }
        }
    } else if (nc > 1) {
        // exact fp64 re-evaluation of every candidate, in ascending lag order
        // (the bitmap words are read by every thread alike: uniform control
        // flow around block_sum's barriers):
        //   c(l) = sum over the overlap of r0[m + l] (e[m] - mu)
        const double* r0 = a.r0buf + (int64_t)sig * n;
        double bestd = -INFINITY;
        kbest = 0x7fffffff;
        const int nw = (2 * L + 1 + 31) >> 5;
        for (int w = 0; w < nw; ++w) {
            unsigned bits = cbits[w];
            while (bits) {
                const int k = 32 * w + __builtin_ctz(bits);
                bits &= bits - 1u;
                const int l = k - L;
                const int m0 = l < 0 ? -l : 0, m1 = l > 0 ? n - l : n;
                double acc = 0.0;
                for (int m = m0 + tid; m < m1; m += 8 * XT) {
                    double rv8[8], ev8[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {  // issue all 8 pairs of loads first
                        const int mm = min(m + u * XT, m1 - 1);
                        rv8[u] = r0[mm + l];
                        ev8[u] = (double)e[mm];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if (m + u * XT < m1) acc += rv8[u] * (ev8[u] - mu);
                }
                acc = block_sum(acc, red);
                if (acc > bestd) {  // ascending k: the first maximum is kept
                    bestd = acc;
                    kbest = k;
                }
            }
        }
    }
    if (tid == 0) {
        const int l = kbest - L;
        a.lag[cell] = l;
        a.zero_energy[cell] = a.Z[(int64_t)sig * (2 * L + 1) + kbest];
        a.status[cell] = status;
    }
}

}  // namespace cse

using namespace cse;

extern "C" int64_t cse_xcorr_workspace_bytes(int64_t n_sig, int64_t len, int n, int max_lag) {
    if (n_sig < 0 || n < 1 || max_lag < 0) return -1;
    const int nb = (n + XB - 1) / XB;
    const int64_t w = 2 * (int64_t)max_lag + 1;
    return n_sig * nb * (XH + 1) * 8 + n_sig * (int64_t)n * 8 + 2 * n_sig * w * 8 + n_sig * 8 + 256;
}

extern "C" int cse_xcorr_prepare(const double* clean, int64_t n_sig, int64_t len, int n,
                                 int max_lag, void* workspace, cse_stream_t stream) {
    CSE_CHECK_ARG(clean && workspace, "cse_xcorr_prepare: NULL clean/workspace");
    CSE_CHECK_ARG(n >= 1 && n <= len && max_lag >= 0 && max_lag < n && max_lag <= (XN - XB) / 2,
                  "cse_xcorr_prepare: n=%d len=%lld max_lag=%d", n, (long long)len, max_lag);
    const int nb = (n + XB - 1) / XB;
    unsigned char* ws = (unsigned char*)workspace;
    float2* R = (float2*)ws;
    double* r0 = (double*)(ws + n_sig * nb * (XH + 1) * 8);
    double* W = r0 + n_sig * (int64_t)n;
    double* Z = W + n_sig * (2 * (int64_t)max_lag + 1);
    double* rn = Z + n_sig * (2 * (int64_t)max_lag + 1);
    hipLaunchKernelGGL(xcorr_prep_kernel, dim3(nb + 1, (unsigned)n_sig), dim3(XT), 0,
                       (hipStream_t)stream, clean, len, n, max_lag, nb, R, r0, W, Z, rn);
    CSE_CHECK_LAUNCH("cse_xcorr_prepare");
    return CSE_OK;
}

extern "C" int cse_xcorr_lag(const float* head, const int64_t* head_offset, const int32_t* sig_of,
                             int64_t n_cells, int64_t n_sig, int n, int max_lag,
                             const void* workspace, int32_t* lag, double* zero_energy,
                             int32_t* status, float* corr, cse_stream_t stream) {
    CSE_CHECK_ARG(head && head_offset && sig_of && workspace && lag && zero_energy && status,
                  "cse_xcorr_lag: NULL argument");
    CSE_CHECK_ARG(n >= 1 && max_lag >= 0 && max_lag < n && max_lag <= (XN - XB) / 2,
                  "cse_xcorr_lag: n=%d max_lag=%d", n, max_lag);
    if (n_cells == 0) return CSE_OK;
    const int nb = (n + XB - 1) / XB;
    const unsigned char* ws = (const unsigned char*)workspace;
    XcArgs a;
    a.head = head;
    a.head_offset = head_offset;
    a.sig_of = sig_of;
    a.R = (const float2*)ws;
    a.r0buf = (const double*)(ws + n_sig * nb * (XH + 1) * 8);
    a.W = a.r0buf + n_sig * (int64_t)n;
    a.Z = a.W + n_sig * (2 * (int64_t)max_lag + 1);
    a.rnorm = a.Z + n_sig * (2 * (int64_t)max_lag + 1);
    a.n = n;
    a.max_lag = max_lag;
    a.nb = nb;
    a.lag = lag;
    a.zero_energy = zero_energy;
    a.status = status;
    a.corr = corr;
    hipLaunchKernelGGL(xcorr_lag_kernel, dim3((unsigned)n_cells), dim3(XT), 0,
                       (hipStream_t)stream, a);
    CSE_CHECK_LAUNCH("cse_xcorr_lag");
    return CSE_OK;
}
