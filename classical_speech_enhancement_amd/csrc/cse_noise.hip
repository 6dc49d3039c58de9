// Noise-PSD estimators (Code/noise_estimation.py) on device, fp64 math.
//
//   PercentileNoiseEstimator.estimate   :20-56   -> frame_energy + select_quiet + bin_stats
//   MinTrackingNoiseEstimator.estimate  :64-95   -> bin_stats(median) + iir + min_filter
//   TrueNoiseEstimator.estimate         :115-155 -> true_fit on |STFT(noisy-clean)|^2
//   _simple_noise_estimate              :226-232 -> bin_stats(simple) when T < 5
//   noise smoothing (mmse.py:48-54, advanced_mmse.py:60-66) -> smooth_kernel
//
// These run once per (signal, n_fft, hop) group and are amortised over the
// hundreds of grid cells that share the group, so they favour exactness
// (fp64, full sorts reproducing np.percentile / np.median) over speed.
#include "cse_common.hpp"

#include <cstdlib>

#include <math.h>

namespace cse {

constexpr int kMaxSortFrames = 16384;  // LDS bitonic sort capacity: 128 KiB of doubles

__device__ __forceinline__ bool key_less(double a, int ia, double b, int ib) {
    return a < b || (a == b && ia < ib);
}

// ascending bitonic sort of n2 (power of two) keys (+ optional indices) in LDS
__device__ void bitonic_sort(double* key, int* idx, int n2) {
    for (int k = 2; k <= n2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const int ii = idx ? idx[i] : i, il = idx ? idx[l] : l;
                    const bool gt = key_less(key[l], il, key[i], ii);
                    if (gt == up) {
                        double tk = key[i];
                        key[i] = key[l];
                        key[l] = tk;
                        if (idx) {
                            int ti = idx[i];
                            idx[i] = idx[l];
                            idx[l] = ti;
                        }
                    }
                }
            }
            __syncthreads();
        }
    }
}

static int next_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

// numpy 2.x _lerp(a, b, t): a + (b - a) t, or b - (b - a)(1 - t) for t >= 0.5,
// every operation rounded on its own (-ffp-contract=fast would fuse the product
// into the sum: one rounding less than numpy)
__device__ __forceinline__ double np_lerp(double a, double b, double t) {
#pragma clang fp contract(off)
    const double diff = b - a;
    return t >= 0.5 ? b - diff * (1.0 - t) : a + diff * t;
}

// numpy 2.x _quantile's indices for method='linear' on n sorted values:
// virtual index (n - 1) q, its neighbours, and the weight gamma = virtual -
// previous (rounded operations, as np_lerp)
__device__ __forceinline__ double np_quantile_index(int n, double q, int& prev, int& next) {
#pragma clang fp contract(off)
    const double virt = (double)(n - 1) * q;
    double prev_f = floor(virt);
    if (virt >= (double)(n - 1)) {
        prev = next = n - 1;
        prev_f = -1.0;  // numpy sets previous_indexes = -1 here; gamma uses it
    } else if (virt < 0.0) {
        prev = next = 0;
        prev_f = 0.0;
    } else {
        prev = (int)prev_f;
        next = prev + 1;
    }
    return virt - prev_f;
}

// np.percentile(sorted[0:n], pct) with method='linear' (numpy 2.x _quantile/_lerp)
__device__ double lerp_percentile(const double* s, int n, double q) {
    int prev, next;
    const double gamma = np_quantile_index(n, q, prev, next);
    return np_lerp(s[prev], s[next], gamma);
}

// mean_b log(max(P[t][b], eps)) per frame: one wavefront per frame (4 per
// 256-thread block), lane sums over b = lane + 64 m, then a butterfly
// reduction (every lane ends with the same sum; no LDS, no block barrier).
// The addition order is not numpy's pairwise one (neither was the r01-r03
// block tree): the energies only rank frames, and frames with equal rows get
// equal energies in any fixed order.
__global__ void __launch_bounds__(256) frame_energy_kernel(const double* __restrict__ P, int T,
                                                           int B, double eps,
                                                           double* __restrict__ energy) {
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t sig = blockIdx.y;
    if (t >= T) return;  // whole wavefronts only
    const double* row = P + (sig * T + t) * (int64_t)B;
    double s = 0.0;
    for (int b = lane; b < B; b += 64) s += log(fmax(row[b], eps));
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
    if (lane == 0) energy[sig * T + t] = s / (double)B;
}

// the same for two eps values from one read of P: the logs differ only where
// P is below the larger eps (bit-identical to two frame_energy_kernel passes:
// same operands, same order)
__global__ void __launch_bounds__(256) frame_energy2_kernel(const double* __restrict__ P, int T,
                                                            int B, double eps0, double eps1,
                                                            double* __restrict__ energy0,
                                                            double* __restrict__ energy1) {
    const int lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t sig = blockIdx.y;
    if (t >= T) return;
    const double* row = P + (sig * T + t) * (int64_t)B;
    const double hi = fmax(eps0, eps1);
    double s0 = 0.0, s1 = 0.0;
    for (int b = lane; b < B; b += 64) {
        const double x = row[b];
        const double l0 = log(fmax(x, eps0));
        s0 += l0;
        s1 += x >= hi ? l0 : log(fmax(x, eps1));
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        s0 += __shfl_xor(s0, m, 64);
        s1 += __shfl_xor(s1, m, 64);
    }
    if (lane == 0) {
        energy0[sig * T + t] = s0 / (double)B;
        energy1[sig * T + t] = s1 / (double)B;
    }
}

// k quietest frames: argsort(energy)[:k], ties by frame index.  Only the
// energies are sorted (8 B per frame of LDS, so T <= kMaxSortFrames fits);
// the index set is then recovered exactly: every frame below the k-th
// smallest energy thr, plus the lowest-index frames equal to thr.  The output
// order is frame order (the percentile that consumes it sorts the values).
// The selection of the k quietest frames given the sorted energies key[].
__device__ void select_from_sorted(const double* __restrict__ e, const double* key, int* scan,
                                   int T, int k, int* __restrict__ sel) {
    const double thr = key[k - 1];
    // each thread a contiguous chunk of frames; two block scans give every
    // thread its share of the ties (lowest index first) and its output slot
    const int tid = threadIdx.x, nt = blockDim.x;
    const int chunk = (T + nt - 1) / nt;
    const int i0 = min(T, tid * chunk), i1 = min(T, i0 + chunk);
    int lt = 0, eq = 0;
    for (int i = i0; i < i1; ++i) {
        const double v = e[i];
        lt += v < thr;
        eq += v == thr;
    }
    auto exclusive_scan = [&](int v) {
        __syncthreads();
        scan[tid] = v;
        __syncthreads();
        for (int d = 1; d < nt; d <<= 1) {
            const int add = tid >= d ? scan[tid - d] : 0;
            __syncthreads();
            scan[tid] += add;
            __syncthreads();
        }
        const int total = scan[nt - 1];
        const int excl = scan[tid] - v;
        __syncthreads();
        return make_int2(excl, total);
    };
    const int2 eqs = exclusive_scan(eq);
    const int2 lts = exclusive_scan(lt);
    const int take_eq = max(0, min(eq, (k - lts.y) - eqs.x));  // ties still needed before mine
    const int2 outs = exclusive_scan(lt + take_eq);
    int out = outs.x, taken = 0;
    for (int i = i0; i < i1; ++i) {
        const double v = e[i];
        if (v < thr || (v == thr && taken++ < take_eq)) sel[out++] = i;
    }
}

// grid (n_sig, sets): energy set y = energy + y n_sig T; one sort of the
// signal's energies serves k0 (-> sel0) and, if sel1, k1 (-> sel1), each set's
// outputs at + y n_sig T
__global__ void select_quiet_kernel(const double* __restrict__ energy, int T, int n2, int k0,
                                    int* __restrict__ sel0, int k1, int* __restrict__ sel1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* key = (double*)smem;
    const int64_t sig = blockIdx.x;
    const int64_t set = (int64_t)blockIdx.y * gridDim.x * T;
    const double* e = energy + set + sig * T;
    for (int i = threadIdx.x; i < n2; i += blockDim.x) key[i] = i < T ? e[i] : INFINITY;
    __syncthreads();
    bitonic_sort(key, nullptr, n2);
    int* scan = (int*)(key + n2);  // blockDim.x ints after the sort buffer
    select_from_sorted(e, key, scan, T, k0, sel0 + set + sig * T);
    if (sel1) select_from_sorted(e, key, scan, T, k1, sel1 + set + sig * T);
}

enum { STATS_MEDIAN = 0, STATS_PERCENTILE = 1, STATS_SIMPLE = 2 };

// ---------------------------------------------------------------------------
// Per-wavefront bitonic sort of 64 E doubles held in registers, element
// i = lane E + e in register e: exchanges at distance j < E stay inside the
// lane (compile-time register pairs), j >= E cross lanes (lane ^ j/E, one
// 64-bit shuffle per register).  No LDS and no block barrier: a 2048-element
// column sorts in 66 stages of register min/max instead of 66 workgroup-wide
// LDS rounds.  Ascending; values only (equal keys are interchangeable).
// ---------------------------------------------------------------------------
template <int E>
__device__ __forceinline__ void wave_bitonic(double (&v)[E], int lane) {
#pragma unroll
    for (int k = 2; k <= 64 * E; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j < E) {
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    if (e & j) continue;
                    // i = lane E + e, partner i ^ j = lane E + (e ^ j) > i
                    const bool up = (k < E) ? ((e & k) == 0) : ((lane & (k / E)) == 0);
                    const double a = v[e], b = v[e | j];
                    const double lo = fmin(a, b), hi = fmax(a, b);
                    v[e] = up ? lo : hi;
                    v[e | j] = up ? hi : lo;
                }
            } else {
                const int d = j / E;
                const bool first = (lane & d) == 0;      // i < partner
                const bool up = (lane & (k / E)) == 0;  // k > j >= E
                const bool take_min = first == up;
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    const double o = __shfl_xor(v[e], d, 64);
                    v[e] = take_min ? fmin(v[e], o) : fmax(v[e], o);
                }
            }
        }
    }
}

// element idx of the wave-sorted array, broadcast to every lane
template <int E>
__device__ __forceinline__ double wave_at(const double (&v)[E], int lane, int idx) {
    double r = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) r = (lane * E + e == idx) ? v[e] : r;
    return __shfl(r, idx / E, 64);
}

// bin_stats_kernel's median / percentile modes for n2 = 64 E <= 2048 sort
// slots: one wavefront per (bin, signal), 4 bins per block, the same order
// statistics and the same arithmetic as the LDS path: bit-identical results
// for finite P.  A NaN in P is not propagated the way numpy's median /
// percentile would (fmin / fmax drop it, so the statistic of the remaining
// values comes out, and which path runs depends on T <= 2048); such a P
// comes only from a non-finite noisy signal, whose cells are non-finite in
// the reference and here alike (the finite[] output), so the estimate's value
// does not reach any score.
template <int E>
__global__ void __launch_bounds__(256) bin_stats_wave_kernel(
    const double* __restrict__ P, int T, int B, int mode, const int* __restrict__ sel, int k,
    double q, double floor_rel, double eps, double* __restrict__ med, float* __restrict__ N,
    const int* __restrict__ sel_z1, double eps_z1, float* __restrict__ N_z1) {
    if (blockIdx.z == 1) {  // the second estimate of a two-estimate launch
        sel = sel_z1;
        eps = eps_z1;
        N = N_z1;
    }
    if (mode != STATS_MEDIAN && !N) return;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t sig = blockIdx.y;
    if (b >= B) return;  // whole wavefronts only
    const double* Ps = P + sig * (int64_t)T * B + b;
    const int n = (mode == STATS_MEDIAN) ? T : k;
    const int* sl = sel ? sel + sig * (int64_t)T : nullptr;
    double v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        const int t = i < n ? (mode == STATS_MEDIAN ? i : sl[i]) : 0;
        v[e] = i < n ? Ps[(int64_t)t * B] : INFINITY;
    }
    wave_bitonic<E>(v, lane);
    if (mode == STATS_MEDIAN) {
        const double m = (T & 1) ? wave_at<E>(v, lane, T / 2)
                                 : (wave_at<E>(v, lane, T / 2 - 1) + wave_at<E>(v, lane, T / 2)) / 2.0;
        if (lane == 0) med[sig * B + b] = m;
        return;
    }
    // np.percentile(..., q, method='linear') as lerp_percentile
    int prev, next;
    const double gamma = np_quantile_index(n, q, prev, next);
    const double pc = np_lerp(wave_at<E>(v, lane, prev), wave_at<E>(v, lane, next), gamma);
    const double est = fmax(pc, floor_rel * med[sig * B + b]);
    if (lane == 0) N[sig * B + b] = (float)fmax(est, eps);
}

// the second estimate (z1): a launch with grid z = 2 when sel_z1 is given
struct StatsZ1 {
    const int* sel = nullptr;
    double eps = 0.0;
    float* N = nullptr;
};

// ---------------------------------------------------------------------------
// Median over all frames by selection instead of a full sort (r05): one
// wavefront per (bin, signal), the column's doubles as order-preserving 64-bit
// keys in E registers per lane.  A binary descent over the key bits, counting
// candidates with ballots, narrows the candidate set around rank r until at
// most 64 remain (it starts at the highest bit in which the column's keys
// differ); those are compacted into one register per lane and sorted by the
// 64-element wave bitonic, and element r is read out.  For even T the upper
// middle element is v1 itself when it repeats past rank T/2, else the smallest
// key above v1.  The order statistics are the sort's exactly, so med equals
// the bitonic path bit for bit (finite P); ~4x fewer instructions than the
// 2,048-slot register sort at T = 1,251.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long dkey(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dval(unsigned long long k) {
    return __builtin_bit_cast(double, (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}
__device__ __forceinline__ unsigned long long wave_or64(unsigned long long v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v |= __shfl_xor(v, m, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_min64(unsigned long long v) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
        const unsigned long long o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
    return v;
}

// the key of rank r (0-based) among the column's n real keys k[] (pads are
// all-ones: above every real key, never of rank < n)
template <int E>
__device__ unsigned long long wave_select(const unsigned long long (&k)[E], int n, int r, int lane,
                                          double* buf) {
    // bits above the highest differing one are common to every real key
    unsigned long long k0 = __shfl(k[0], 0, 64), dif = 0;
#pragma unroll
    for (int e = 0; e < E; ++e)
        if (lane * E + e < n) dif |= k[e] ^ k0;
    dif = wave_or64(dif);
    int bit = dif ? 63 - __builtin_clzll(dif) : -1;
    unsigned long long pre = k0;  // candidates: keys equal to pre above `bit`
    int cnt = n;
    for (; bit >= 0 && cnt > 64; --bit) {
        const unsigned long long hi = ~((2ull << bit) - 1);  // bits above `bit` (bit 63: none)
        const unsigned long long one = 1ull << bit;
        int c0 = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const bool cand0 = ((k[e] ^ pre) & hi) == 0 && (k[e] & one) == 0;
            c0 += __popcll(__ballot(cand0));
        }
        if (r < c0) {
            pre &= ~one;
            cnt = c0;
        } else {
            pre |= one;
            r -= c0;
            cnt -= c0;
        }
    }
    if (cnt > 64) return pre;  // every bit decided: the candidates are all equal to pre
    // compact the candidates (the keys equal to pre in every bit above `bit`)
    // into buf[0, cnt), then sort 64
    const unsigned long long hi = bit >= 0 ? ~((2ull << bit) - 1) : ~0ull;
    int base = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        // (a pad matches a prefix of ones: only real keys are compacted)
        const bool cand = lane * E + e < n && ((k[e] ^ pre) & hi) == 0;
        const unsigned long long m = __ballot(cand);
        if (cand) buf[base + __popcll(m & ((1ull << lane) - 1))] = dval(k[e]);
        base += __popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double v[1] = {lane < cnt ? buf[lane] : INFINITY};
    wave_bitonic<1>(v, lane);
    return dkey(wave_at<1>(v, lane, r));
}

template <int E>
__global__ void __launch_bounds__(256) median_select_kernel(const double* __restrict__ P, int T,
                                                            int B, double* __restrict__ med) {
    __shared__ double sbuf[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int b = blockIdx.x * 4 + w;
    const int64_t sig = blockIdx.y;
    if (b >= B) return;  // whole wavefronts only
    const double* Ps = P + sig * (int64_t)T * B + b;
    unsigned long long k[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int i = lane * E + e;
        k[e] = i < T ? dkey(Ps[(int64_t)i * B]) : ~0ull;
    }
    const int r = (T & 1) ? T / 2 : T / 2 - 1;
    const unsigned long long k1 = wave_select<E>(k, T, r, lane, sbuf[w]);
    double m = dval(k1);
    if (!(T & 1)) {  // upper middle: v1 again if it repeats past rank T/2, else the next key
        int le = 0;
        unsigned long long nxt = ~0ull;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            le += __popcll(__ballot(k[e] <= k1 && lane * E + e < T));
            if (k[e] > k1 && k[e] < nxt) nxt = k[e];
        }
        const unsigned long long k2 = le > T / 2 ? k1 : wave_min64(nxt);
        m = (m + dval(k2)) / 2.0;
    }
    if (lane == 0) med[sig * B + b] = m;
}

template <int E>
static void launch_stats_wave(const double* P, int64_t n_sig, int T, int B, int mode,
                              const int* sel, int k, double q, double floor_rel, double eps,
                              double* med, float* N, StatsZ1 z1, hipStream_t s) {
    hipLaunchKernelGGL(bin_stats_wave_kernel<E>,
                       dim3((B + 3) / 4, (unsigned)n_sig, z1.sel ? 2u : 1u), dim3(256), 0,
                       s, P, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1.sel, z1.eps, z1.N);
}

// the wave path for n <= 2048 sort slots; false: use the LDS path
static bool stats_wave(int n, const double* P, int64_t n_sig, int T, int B, int mode,
                       const int* sel, int k, double q, double floor_rel, double eps, double* med,
                       float* N, hipStream_t s, StatsZ1 z1 = StatsZ1()) {
    if (n > 2048 || n < 1) return false;
    const int n2 = n <= 64 ? 64 : next_pow2(n);
    switch (n2 / 64) {
        case 1: launch_stats_wave<1>(P, n_sig, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1, s); break;
        case 2: launch_stats_wave<2>(P, n_sig, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1, s); break;
        case 4: launch_stats_wave<4>(P, n_sig, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1, s); break;
        case 8: launch_stats_wave<8>(P, n_sig, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1, s); break;
        case 16: launch_stats_wave<16>(P, n_sig, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1, s); break;
        default: launch_stats_wave<32>(P, n_sig, T, B, mode, sel, k, q, floor_rel, eps, med, N, z1, s); break;
    }
    return true;
}

// per (bin, signal): median over all frames (-> med), and optionally the
// percentile over the selected quiet frames (-> N) or the T<5 simple estimate.
__global__ void bin_stats_kernel(const double* __restrict__ P, int T, int B, int n2_all,
                                 int mode, const int* __restrict__ sel, int k, int n2_sel,
                                 double q, double floor_rel, double eps,
                                 double* __restrict__ med, float* __restrict__ N,
                                 int broadcast_T) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* s = (double*)smem;
    const int b = blockIdx.x;
    const int64_t sig = blockIdx.y;
    const double* Ps = P + sig * (int64_t)T * B + b;
    double median = 0.0;
    if (mode == STATS_PERCENTILE && med) {
        median = med[sig * B + b];  // precomputed by cse_noise_median
    } else if (mode != STATS_SIMPLE) {
        for (int i = threadIdx.x; i < n2_all; i += blockDim.x)
            s[i] = i < T ? Ps[(int64_t)i * B] : INFINITY;
        __syncthreads();
        bitonic_sort(s, nullptr, n2_all);
        median = (T & 1) ? s[T / 2] : (s[T / 2 - 1] + s[T / 2]) / 2.0;
        if (threadIdx.x == 0 && med) med[sig * B + b] = median;
        __syncthreads();
    }
    if (mode == STATS_MEDIAN) return;
    double est;
    if (mode == STATS_PERCENTILE) {
        for (int i = threadIdx.x; i < n2_sel; i += blockDim.x)
            s[i] = i < k ? Ps[(int64_t)sel[sig * (int64_t)T + i] * B] : INFINITY;
        __syncthreads();
        bitonic_sort(s, nullptr, n2_sel);
        est = fmax(lerp_percentile(s, k, q), floor_rel * median);
    } else {  // simple: mean (T < 2) or 25th percentile over all frames
        for (int i = threadIdx.x; i < n2_all; i += blockDim.x)
            s[i] = i < T ? Ps[(int64_t)i * B] : INFINITY;
        __syncthreads();
        bitonic_sort(s, nullptr, n2_all);
        est = (T < 2) ? s[0] : lerp_percentile(s, T, 0.25);
    }
    const float v = (float)fmax(est, eps);
    if (broadcast_T) {
        for (int t = threadIdx.x; t < T; t += blockDim.x) N[(sig * T + t) * (int64_t)B + b] = v;
    } else if (threadIdx.x == 0) {
        N[sig * B + b] = v;
    }
}

// One smoothing step s = a s + (1 - a) x as numpy evaluates it: two rounded
// products and a rounded sum.  HIP's __dmul_rn / __dadd_rn are plain x * y /
// x + y, which -ffp-contract=fast fuses into an FMA (one rounding less: the
// compiled recurrences were not numpy's until late r04); the pragma takes the
// contract flag off these operations.
__device__ __forceinline__ double smooth_step(double a, double s, double c, double x) {
#pragma clang fp contract(off)
    return a * s + c * x;
}

// S_t = a*S_{t-1} + (1-a)*P_t (noise_estimation.py:78-82), numpy evaluation order;
// the loads one block of U frames ahead of the recurrence (finish_row's form)
__global__ void iir_kernel(const double* __restrict__ P, int T, int B, double a,
                           double* __restrict__ S) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t sig = blockIdx.y;
    if (b >= B) return;
    const double* Ps = P + sig * (int64_t)T * B + b;
    double* Ss = S + sig * (int64_t)T * B + b;
    double s = Ps[0];
    Ss[0] = s;
    const double c = 1.0 - a;
    constexpr int U = 8;
    const int full = 1 + ((T > 1 ? T - 1 : 0) / U) * U;  // frames [1, full) in whole blocks
    int t = 1;
    if (full > 1) {
        double cur[U], nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = Ps[(int64_t)(1 + u) * B];
        for (; t < full; t += U) {
            const bool more = t + U < full;  // uniform
            if (more) {
#pragma unroll
                for (int u = 0; u < U; ++u) nxt[u] = Ps[(int64_t)(t + U + u) * B];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                s = smooth_step(a, s, c, cur[u]);
                Ss[(int64_t)(t + u) * B] = s;
            }
            if (more) {
#pragma unroll
                for (int u = 0; u < U; ++u) cur[u] = nxt[u];
            }
        }
    }
    for (; t < T; ++t) {
        s = smooth_step(a, s, c, Ps[(int64_t)t * B]);
        Ss[(int64_t)t * B] = s;
    }
}

// minimum_filter1d(S, size=w, mode='nearest') then floors (noise_estimation.py:86-95)
__global__ void min_filter_kernel(const double* __restrict__ S, int T, int B, int half,
                                  const double* __restrict__ med, double eps,
                                  float* __restrict__ N, double eps_b, float* __restrict__ Nb) {
    const int t = blockIdx.x;
    const int64_t sig = blockIdx.y;
    const int lo = t - half < 0 ? 0 : t - half;
    const int hi = t + half > T - 1 ? T - 1 : t + half;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        const double* Ss = S + sig * (int64_t)T * B + b;
        double m = Ss[(int64_t)lo * B];
        for (int u = lo + 1; u <= hi; ++u) m = fmin(m, Ss[(int64_t)u * B]);
        const double f = fmax(m, 0.01 * med[sig * B + b]);
        N[(sig * T + t) * (int64_t)B + b] = (float)fmax(f, eps);
        if (Nb) Nb[(sig * T + t) * (int64_t)B + b] = (float)fmax(f, eps_b);
    }
}

// The same through an LDS tile (r03): a block owns 32 bins x 64 output frames
// and stages rows t0 - half .. t0 + 63 + half (indices clamped to [0, T):
// 'nearest' padding repeats the edge frames, which leaves the window minimum
// unchanged); log2 doubling passes turn the tile into M_p[r] = min over rows
// [r, r + p), p the largest power of two <= W = 2 half + 1, and each output is
// min(M_p[r], M_p[r + W - p]) over its window [r, r + W).  About 7 LDS
// operations per element instead of W = 51 global loads.  half <= MF_HMAX.
constexpr int MF_T = 64, MF_B = 32, MF_HMAX = 25, MF_ROWS = MF_T + 2 * MF_HMAX;
constexpr int MF_PER = (MF_ROWS + 7) / 8;  // tile rows per thread (8 row groups)
__global__ void __launch_bounds__(256) min_filter_tiled_kernel(
    const double* __restrict__ S, int T, int B, int half, const double* __restrict__ med,
    double eps, float* __restrict__ N, double eps_b, float* __restrict__ Nb) {
    __shared__ double tile[MF_ROWS][MF_B];
    const int bl = threadIdx.x & (MF_B - 1), tg = threadIdx.x / MF_B;
    const int b = blockIdx.x * MF_B + bl;
    const int t0 = blockIdx.y * MF_T;
    const int64_t sig = blockIdx.z;
    const int rows = MF_T + 2 * half;
    const double* Ss = S + sig * (int64_t)T * B;
    const int bc = b < B ? b : B - 1;
#pragma unroll
    for (int m = 0; m < MF_PER; ++m) {
        const int r = tg + 8 * m;
        if (r < rows) {
            const int t = min(max(t0 - half + r, 0), T - 1);
            tile[r][bl] = Ss[(int64_t)t * B + bc];
        }
    }
    const int W = 2 * half + 1;
    int p = 1;
    while (2 * p <= W) p *= 2;
    for (int st = 1; st < p; st *= 2) {
        __syncthreads();
        double nv[MF_PER];
#pragma unroll
        for (int m = 0; m < MF_PER; ++m) {
            const int r = tg + 8 * m;
            nv[m] = (r + st < rows) ? fmin(tile[r][bl], tile[r + st][bl]) : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MF_PER; ++m) {
            const int r = tg + 8 * m;
            if (r + st < rows) tile[r][bl] = nv[m];
        }
    }
    __syncthreads();
    if (b >= B) return;
    const double fl = 0.01 * med[sig * B + b];
#pragma unroll
    for (int m = 0; m < MF_T / 8; ++m) {
        const int r = tg + 8 * m;
        const int t = t0 + r;
        if (t >= T) break;
        const double mn = fmin(tile[r][bl], tile[r + W - p][bl]);
        const double f = fmax(mn, fl);
        N[(sig * T + t) * (int64_t)B + b] = (float)fmax(f, eps);
        if (Nb) Nb[(sig * T + t) * (int64_t)B + b] = (float)fmax(f, eps_b);
    }
}

// TrueNoise frame fit (noise_estimation.py:146-153): max(P, eps), rows past
// the source's last frame repeat it (np.pad mode='edge'), extra rows trimmed
__global__ void true_fit_kernel(const double* __restrict__ P, int T_src, int T, int B, double eps,
                                float* __restrict__ N) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y;
    const int64_t sig = blockIdx.z;
    if (b >= B) return;
    const int ts = t < T_src ? t : T_src - 1;
    N[(sig * T + t) * (int64_t)B + b] = (float)fmax(P[(sig * T_src + ts) * (int64_t)B + b], eps);
}

__global__ void smooth_kernel(const float* __restrict__ N, int T, int B, int src_frames,
                              double mu, float* __restrict__ out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t sig = blockIdx.y;
    if (b >= B) return;
    const float* Ns = N + sig * (int64_t)src_frames * B + b;
    float* Os = out + sig * (int64_t)T * B + b;
    double s = (double)Ns[0];
    Os[0] = (float)s;
    const double c = 1.0 - mu;
    for (int t = 1; t < T; ++t) {
        const double n = t < src_frames ? (double)Ns[(int64_t)t * B] : 0.0;  // fix_length pad
        s = smooth_step(mu, s, c, n);
        Os[(int64_t)t * B] = (float)s;
    }
}

__global__ void invert_kernel(const float* __restrict__ N, int64_t n, double eps,
                              float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (float)(1.0 / fmax((double)N[i], eps));
}

// batched post-processing of noise rows: smoothing over frames, zero-padding a
// static row to out_frames (librosa fix_length), optional 1/max(., eps).
// Frames t < min(src_frames, out_frames) read the source, later ones take 0
// (the zero pad): s = mu s + (1 - mu) n in fp64 in numpy's order.  The
// inversion is a template branch and the loads come in whole blocks of U
// frames, one block ahead, with no per-frame conditions: r03's form (a bounds
// check per load and per store) compiled to a branch per access and a full
// vmcnt(0) wait per block.
// correctly rounded 1/x in f32 for x in [2^-60, 2^60): v_rcp_f32 and one FMA
// Newton step; checked against IEEE 1.0f / x for every f32 in [2^-60, 2^61)
// (tools/micro/rcp_check.hip: 0 mismatches in 1.0e9), so it equals the division
// it replaces there (3 VALU for the ~10 of the division sequence).  Outside
// that range (cse_noise_finish takes any inv_eps > 0, subnormal ones
// included, which v_rcp_f32 may flush) the division itself.
__device__ __forceinline__ float rcp_rn(float x) {
    if (x >= 0x1p-60f && x < 0x1p60f) {
        const float r = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
    return 1.0f / x;
}

// One workgroup per (signal, job) row (grid n_sig x n_jobs, 256 threads):
// tiles of F frames of the row pass through LDS, so the global side is whole
// contiguous F x B blocks read and written by consecutive dword accesses of
// every wave, while each thread runs its bins' recurrence over the tile from
// LDS in numpy's order (bit-identical to the per-bin loop).  A per-bin loop
// writing one float per frame at the 4B-byte row stride (r04's form, and a
// flattened one-thread-per-bin form) ran the rows' stores at 2.5 TB/s; the
// tiled block stores at 4.7 TB/s (tools/micro/row_store.hip).
constexpr int FIN_F = 16;     // frames per tile
// bins per thread: 4 (B <= 1,024: the grid's n_fft 512 / 1024 and up to 2046)
// or 9 (B <= 2,304: n_fft up to 4096, r06), one instantiation each
constexpr int FIN_MAXU = 4, FIN_MAXU_BIG = 9;
template <int MAXU>
__global__ void __launch_bounds__(256) finish_kernel(const cse_noise_job_t* __restrict__ jobs,
                                                     int B, const float* __restrict__ src,
                                                     float* __restrict__ dst) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* tile = (float*)smem;  // [FIN_F][B]
    const cse_noise_job_t jb = jobs[blockIdx.y];
    const int64_t sig = blockIdx.x;
    const int tid = threadIdx.x;
    const float* Ns = src + jb.src_offset + sig * (int64_t)jb.src_frames * B;
    float* Os = dst + jb.dst_offset + sig * (int64_t)jb.out_frames * B;
    const int nfr = jb.out_frames, m = min(jb.src_frames, nfr);  // frames with a source row
    const double mu = jb.mu, c = 1.0 - mu;
    const bool inv = jb.inv_eps > 0.0;
    const float ief = (float)jb.inv_eps;
    double st[MAXU];
    for (int t0 = 0; t0 < nfr; t0 += FIN_F) {
        const int nf = min(FIN_F, nfr - t0);
        const int nld = max(0, min(nf, m - t0)) * B;  // source floats of the tile
        if (t0) __syncthreads();                      // the previous tile's stores have read it
        for (int i = tid; i < nld; i += 256) tile[i] = Ns[(int64_t)t0 * B + i];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MAXU; ++u) {
            const int b = tid + 256 * u;
            if (b >= B) break;
            double s = st[u];
            for (int f = 0; f < nf; ++f) {
                const int t = t0 + f;
                const double x = t < m ? (double)tile[f * B + b] : 0.0;
                s = t == 0 ? x : smooth_step(mu, s, c, x);  // the zero pad: c * 0 = +0
                tile[f * B + b] = inv ? rcp_rn(fmaxf((float)s, ief)) : (float)s;
            }
            st[u] = s;
        }
        __syncthreads();
        for (int i = tid; i < nf * B; i += 256) Os[(int64_t)t0 * B + i] = tile[i];
    }
}

struct Workspace {
    double* energy;  // [n_sig][T]
    int* sel;        // [n_sig][T]
    double* med;     // [n_sig][B]
    double* S;       // [n_sig][T][B]
    // cse_noise_percentile_quad's energies [2 eps][n_sig][T] (f64) and
    // selections [2 pct][2 eps][n_sig][T] (int): a region of its own (r06;
    // r05 borrowed S, so a min-tracking call on another stream with the same
    // workspace would have raced it)
    double* Q;
};

static int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// threads of a whole-row workgroup for the per-bin recurrences (iir, finish):
// the bins of one frame row in one workgroup, whole wavefronts, <= 1,024
static int row_threads(int B) { return B >= 1024 ? 1024 : ((B + 63) / 64) * 64; }

static Workspace carve(void* ws, int64_t n_sig, int T, int B) {
    unsigned char* p = (unsigned char*)ws;
    Workspace w;
    w.energy = (double*)p;
    p += align256(n_sig * (int64_t)T * 8);
    w.sel = (int*)p;
    p += align256(n_sig * (int64_t)T * 4);
    w.med = (double*)p;
    p += align256(n_sig * (int64_t)B * 8);
    w.S = (double*)p;
    p += align256(n_sig * (int64_t)T * B * 8);
    w.Q = (double*)p;
    return w;
}

// (k, percentile) exactly as noise_estimation.py:29-41 (constructor
// parameters :12-13: min_frames, max_fraction, adaptive_short)
static void quiet_count(int T, const cse_noise_params_t& prm, int* k_out, double* pct_out) {
    int min_frames = prm.min_frames;
    double pct = prm.percentile;
    if (prm.adaptive_short && T < 30) {
        min_frames = (T / 4 > 2) ? T / 4 : 2;
        const int target = ((int)(T * 0.15) > 3) ? (int)(T * 0.15) : 3;
        pct = 100.0 * target / T;
        if (pct > 50.0) pct = 50.0;
    }
    int k = (int)ceil((double)T * (pct / 100.0));
    if (k < min_frames) k = min_frames;
    int cap = (int)ceil((double)T * prm.max_fraction);
    if (cap < 1) cap = 1;
    if (k > cap) k = cap;
    if (k > T) k = T;
    *k_out = k;
    *pct_out = pct;
}

static int launch_median(const double* P, int64_t n_sig, int T, int B, double* med,
                         hipStream_t s) {
    static const bool sort_median = getenv("CSE_MEDIAN_SORT") != nullptr;  // A/B: the r04 sort
    if (T >= 65 && T <= 2048 && !sort_median) {  // selection (<= 64: one bitonic anyway)
        const dim3 g((B + 3) / 4, (unsigned)n_sig);
        const int e = (T + 63) / 64;
        if (e <= 8)
            hipLaunchKernelGGL(median_select_kernel<8>, g, dim3(256), 0, s, P, T, B, med);
        else if (e <= 16)
            hipLaunchKernelGGL(median_select_kernel<16>, g, dim3(256), 0, s, P, T, B, med);
        else if (e <= 24)
            hipLaunchKernelGGL(median_select_kernel<24>, g, dim3(256), 0, s, P, T, B, med);
        else
            hipLaunchKernelGGL(median_select_kernel<32>, g, dim3(256), 0, s, P, T, B, med);
        CSE_CHECK_LAUNCH("noise median");
        return CSE_OK;
    }
    if (stats_wave(T, P, n_sig, T, B, STATS_MEDIAN, nullptr, 0, 0.0, 0.0, 0.0, med, nullptr, s)) {
        CSE_CHECK_LAUNCH("noise median");
        return CSE_OK;
    }
    const int n2_all = next_pow2(T);
    hipLaunchKernelGGL(bin_stats_kernel, dim3(B, (unsigned)n_sig), dim3(256),
                       (size_t)n2_all * sizeof(double), s, P, T, B, n2_all, (int)STATS_MEDIAN,
                       (const int*)nullptr, 0, 0, 0.0, 0.0, 0.0, med, (float*)nullptr, 0);
    CSE_CHECK_LAUNCH("noise median");
    return CSE_OK;
}

static int launch_simple(const double* P, int64_t n_sig, int T, int B, double eps, float* N,
                         int broadcast, hipStream_t s) {
    const int n2_all = next_pow2(T);
    hipLaunchKernelGGL(bin_stats_kernel, dim3(B, (unsigned)n_sig), dim3(256),
                       (size_t)n2_all * sizeof(double), s, P, T, B, n2_all, (int)STATS_SIMPLE,
                       (const int*)nullptr, 0, 0, 0.0, 0.0, eps, (double*)nullptr, N, broadcast);
    CSE_CHECK_LAUNCH("noise simple");
    return CSE_OK;
}

static void launch_energy(const double* P, int64_t n_sig, int T, int B, double eps, Workspace w,
                          hipStream_t s) {
    hipLaunchKernelGGL(frame_energy_kernel, dim3((T + 3) / 4, (unsigned)n_sig), dim3(256), 0, s, P,
                       T, B, eps, w.energy);
}

// the percentile estimate from the frame energies already in w.energy
static int launch_percentile_sel(const double* P, const double* med, int64_t n_sig, int T, int B,
                                 const cse_noise_params_t& prm, double eps, float* N, Workspace w,
                                 hipStream_t s) {
    int k;
    double pct;
    quiet_count(T, prm, &k, &pct);
    const int n2_all = next_pow2(T), n2_sel = next_pow2(k);
    hipLaunchKernelGGL(select_quiet_kernel, dim3((unsigned)n_sig, 1u), dim3(1024),
                       (size_t)n2_all * 8 + 1024 * 4, s, (const double*)w.energy, T, n2_all, k,
                       w.sel, 0, (int*)nullptr);
    if (stats_wave(k, P, n_sig, T, B, STATS_PERCENTILE, (const int*)w.sel, k, pct / 100.0,
                   prm.floor_rel, eps, (double*)med, N, s)) {
        CSE_CHECK_LAUNCH("noise percentile");
        return CSE_OK;
    }
    hipLaunchKernelGGL(bin_stats_kernel, dim3(B, (unsigned)n_sig), dim3(256),
                       (size_t)n2_sel * sizeof(double), s, P, T, B, n2_all,
                       (int)STATS_PERCENTILE, (const int*)w.sel, k, n2_sel, pct / 100.0, prm.floor_rel,
                       eps, (double*)med, N, 0);
    CSE_CHECK_LAUNCH("noise percentile");
    return CSE_OK;
}

static int launch_percentile(const double* P, const double* med, int64_t n_sig, int T, int B,
                             const cse_noise_params_t& prm, double eps, float* N, Workspace w,
                             hipStream_t s) {
    launch_energy(P, n_sig, T, B, eps, w, s);
    return launch_percentile_sel(P, med, n_sig, T, B, prm, eps, N, w, s);
}

static int launch_min_tracking(const double* P, const double* med, int64_t n_sig, int T, int B,
                               const cse_noise_params_t& prm, double eps, float* N, double eps_b,
                               float* Nb, Workspace w, hipStream_t s) {
    // alpha: smoothing_factor, or max(0.8, min(0.95, 1 - 5/T)) when None (:72-75)
    const double a = (prm.smoothing_factor == prm.smoothing_factor)
                         ? prm.smoothing_factor
                         : fmax(0.8, fmin(0.95, 1.0 - 5.0 / (double)T));
    int win = prm.window_size > 3 ? prm.window_size : 3;  // min(max(3, w), T), made odd (:97-99)
    if (win > T) win = T;
    if (win % 2 == 0) win += 1;
    hipLaunchKernelGGL(iir_kernel, dim3(ceil_div(B, row_threads(B)), (unsigned)n_sig),
                       dim3(row_threads(B)), 0, s, P, T, B,
                       a, w.S);
    if (win / 2 <= MF_HMAX) {
        hipLaunchKernelGGL(min_filter_tiled_kernel,
                           dim3((B + MF_B - 1) / MF_B, (T + MF_T - 1) / MF_T, (unsigned)n_sig),
                           dim3(256), 0, s, (const double*)w.S, T, B, win / 2, med, eps, N, eps_b,
                           Nb);
    } else {
        hipLaunchKernelGGL(min_filter_kernel, dim3(T, (unsigned)n_sig), dim3(256), 0, s,
                           (const double*)w.S, T, B, win / 2, med, eps, N, eps_b, Nb);
    }
    CSE_CHECK_LAUNCH("noise min tracking");
    return CSE_OK;
}

static bool lds_ready = false;
static int reserve_lds() {
    if (!lds_ready) {
        if (hipFuncSetAttribute((const void*)select_quiet_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                kMaxSortFrames * 8 + 1024 * 4) != hipSuccess ||
            hipFuncSetAttribute((const void*)bin_stats_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                kMaxSortFrames * 8) != hipSuccess) {
            ::cse::set_error("noise kernels: cannot reserve LDS");
            return CSE_ELAUNCH;
        }
        lds_ready = true;
    }
    return CSE_OK;
}

}  // namespace cse

using namespace cse;

#define CSE_NOISE_SHAPE_CHECKS(fn)                                                            \
    CSE_CHECK_ARG(P != nullptr, fn ": P is NULL");                                            \
    CSE_CHECK_ARG(n_sig > 0 && n_sig < 65536 && T >= 1 && B >= 2,                             \
                  fn ": bad shape n_sig=%lld T=%d B=%d", (long long)n_sig, T, B);             \
    CSE_CHECK_ARG(T <= kMaxSortFrames, fn ": T=%d > %d frames unsupported", T, kMaxSortFrames)

extern "C" int64_t cse_noise_workspace_bytes(int64_t n_sig, int T, int B) {
    return align256(n_sig * (int64_t)T * 8) + align256(n_sig * (int64_t)T * 4) +
           align256(n_sig * (int64_t)B * 8) + align256(n_sig * (int64_t)T * B * 8) +
           align256(n_sig * (int64_t)T * 32);
}

extern "C" void cse_noise_default_params(cse_noise_params_t* prm) {
    if (!prm) return;
    prm->percentile = 20.0;
    prm->max_fraction = 0.30;
    prm->floor_rel = 0.02;
    prm->smoothing_factor = __builtin_nan("");
    prm->min_frames = 10;
    prm->adaptive_short = 1;
    prm->window_size = 50;
    prm->src_frames = 0;
}

extern "C" int cse_noise_estimate_ex(int method, const double* P, int64_t n_sig, int T, int B,
                                     const cse_noise_params_t* prm, double eps, float* N,
                                     void* workspace, cse_stream_t stream) {
    hipStream_t s = (hipStream_t)stream;
    CSE_NOISE_SHAPE_CHECKS("cse_noise_estimate");
    CSE_CHECK_ARG(N != nullptr && prm != nullptr, "cse_noise_estimate: N or params is NULL");
    if (method == CSE_NOISE_TRUE) {
        const int T_src = prm->src_frames > 0 ? prm->src_frames : T;
        CSE_CHECK_ARG(T_src <= (1 << 24), "cse_noise_estimate: src_frames=%d", T_src);
        hipLaunchKernelGGL(true_fit_kernel, dim3(ceil_div(B, 256), T, (unsigned)n_sig), dim3(256),
                           0, s, P, T_src, T, B, eps, N);
        CSE_CHECK_LAUNCH("cse_noise_estimate(true)");
        return CSE_OK;
    }
    CSE_CHECK_ARG(method == CSE_NOISE_PERCENTILE || method == CSE_NOISE_MIN_TRACKING,
                  "Unbekannte Methode: %d", method);
    CSE_CHECK_ARG(workspace != nullptr, "cse_noise_estimate: workspace is NULL");
    int rc = reserve_lds();
    if (rc) return rc;
    Workspace w = carve(workspace, n_sig, T, B);
    if (T < 5)  // noise_estimation.py:194-195
        return launch_simple(P, n_sig, T, B, eps, N, method == CSE_NOISE_MIN_TRACKING, s);
    rc = launch_median(P, n_sig, T, B, w.med, s);
    if (rc) return rc;
    if (method == CSE_NOISE_PERCENTILE)
        return launch_percentile(P, w.med, n_sig, T, B, *prm, eps, N, w, s);
    return launch_min_tracking(P, w.med, n_sig, T, B, *prm, eps, N, 0.0, nullptr, w, s);
}

extern "C" int cse_noise_estimate(int method, const double* P, int64_t n_sig, int T, int B,
                                  double percentile, double eps, float* N, void* workspace,
                                  cse_stream_t stream) {
    cse_noise_params_t prm;
    cse_noise_default_params(&prm);
    prm.percentile = percentile;
    return cse_noise_estimate_ex(method, P, n_sig, T, B, &prm, eps, N, workspace, stream);
}

extern "C" int cse_noise_median(const double* P, int64_t n_sig, int T, int B, double* med,
                                cse_stream_t stream) {
    CSE_NOISE_SHAPE_CHECKS("cse_noise_median");
    CSE_CHECK_ARG(med != nullptr, "cse_noise_median: med is NULL");
    int rc = reserve_lds();
    if (rc) return rc;
    return launch_median(P, n_sig, T, B, med, (hipStream_t)stream);
}

extern "C" int cse_noise_percentile_med(const double* P, const double* med, int64_t n_sig, int T,
                                        int B, double percentile, double eps, float* N,
                                        void* workspace, cse_stream_t stream) {
    CSE_NOISE_SHAPE_CHECKS("cse_noise_percentile_med");
    CSE_CHECK_ARG(med && N && workspace, "cse_noise_percentile_med: NULL pointer");
    CSE_CHECK_ARG(T >= 5, "cse_noise_percentile_med: T=%d < 5 (use the simple estimate)", T);
    int rc = reserve_lds();
    if (rc) return rc;
    cse_noise_params_t prm;
    cse_noise_default_params(&prm);
    prm.percentile = percentile;
    return launch_percentile(P, med, n_sig, T, B, prm, eps, N, carve(workspace, n_sig, T, B),
                             (hipStream_t)stream);
}

extern "C" int cse_noise_percentile_med2(const double* P, const double* med, int64_t n_sig,
                                         int T, int B, double percentile_a, double percentile_b,
                                         double eps, float* N_a, float* N_b, void* workspace,
                                         cse_stream_t stream) {
    CSE_NOISE_SHAPE_CHECKS("cse_noise_percentile_med2");
    CSE_CHECK_ARG(med && N_a && workspace, "cse_noise_percentile_med2: NULL pointer");
    CSE_CHECK_ARG(T >= 5, "cse_noise_percentile_med2: T=%d < 5 (use the simple estimate)", T);
    int rc = reserve_lds();
    if (rc) return rc;
    const Workspace w = carve(workspace, n_sig, T, B);
    const hipStream_t s = (hipStream_t)stream;
    cse_noise_params_t prm;
    cse_noise_default_params(&prm);
    launch_energy(P, n_sig, T, B, eps, w, s);  // depends on eps only
    prm.percentile = percentile_a;
    rc = launch_percentile_sel(P, med, n_sig, T, B, prm, eps, N_a, w, s);
    if (rc || !N_b) return rc;
    prm.percentile = percentile_b;
    return launch_percentile_sel(P, med, n_sig, T, B, prm, eps, N_b, w, s);
}

// Two percentiles x two eps values (noise_estimation.py:16-52 for each of the
// four (percentile, eps) estimates of a hop) in four launches: one frame-energy
// pass for both eps, one sort of each eps's energies for both percentiles, and
// one order-statistic launch per percentile covering both eps.  Outputs equal
// four cse_noise_percentile_med calls bit for bit.  N[p][e]: N_pe, NULL = skip.
extern "C" int cse_noise_percentile_quad(const double* P, const double* med, int64_t n_sig, int T,
                                         int B, double percentile_a, double percentile_b,
                                         double eps_a, double eps_b, float* N_aa, float* N_ab,
                                         float* N_ba, float* N_bb, void* workspace,
                                         cse_stream_t stream) {
    CSE_NOISE_SHAPE_CHECKS("cse_noise_percentile_quad");
    CSE_CHECK_ARG(med && workspace, "cse_noise_percentile_quad: NULL pointer");
    CSE_CHECK_ARG(T >= 5, "cse_noise_percentile_quad: T=%d < 5 (use the simple estimate)", T);
    int rc = reserve_lds();
    if (rc) return rc;
    const hipStream_t s = (hipStream_t)stream;
    cse_noise_params_t prm;
    cse_noise_default_params(&prm);
    const double pct_in[2] = {percentile_a, percentile_b};
    int k[2];
    double pct[2];
    for (int p = 0; p < 2; ++p) {
        prm.percentile = pct_in[p];
        quiet_count(T, prm, &k[p], &pct[p]);
    }
    const Workspace w = carve(workspace, n_sig, T, B);
    if (k[0] > 2048 || k[1] > 2048 || B < 16) {  // the LDS order-statistic path: one at a time
        const double eps[2] = {eps_a, eps_b};
        float* const N[2][2] = {{N_aa, N_ab}, {N_ba, N_bb}};
        for (int e = 0; e < 2; ++e) {
            launch_energy(P, n_sig, T, B, eps[e], w, s);
            for (int p = 0; p < 2; ++p) {
                if (!N[p][e]) continue;
                prm.percentile = pct_in[p];
                rc = launch_percentile_sel(P, med, n_sig, T, B, prm, eps[e], N[p][e], w, s);
                if (rc) return rc;
            }
        }
        return CSE_OK;
    }
    // the workspace's quad region holds the two energy rows and the four
    // selections (2 x 8 + 4 x 4 = 32 bytes per (signal, frame))
    double* en = w.Q;                         // [2 eps][n_sig][T]
    int* sel = (int*)(en + 2 * n_sig * T);    // [2 pct][2 eps][n_sig][T]
    const int64_t ST = n_sig * (int64_t)T;
    hipLaunchKernelGGL(frame_energy2_kernel, dim3((T + 3) / 4, (unsigned)n_sig), dim3(256), 0, s, P,
                       T, B, eps_a, eps_b, en, en + ST);
    const int n2_all = next_pow2(T);
    hipLaunchKernelGGL(select_quiet_kernel, dim3((unsigned)n_sig, 2u), dim3(1024),
                       (size_t)n2_all * 8 + 1024 * 4, s, (const double*)en, T, n2_all, k[0], sel,
                       k[1], sel + 2 * ST);
    float* const Ne[2][2] = {{N_aa, N_ab}, {N_ba, N_bb}};
    for (int p = 0; p < 2; ++p) {
        const int* sp = sel + 2 * p * ST;  // [eps][n_sig][T] of percentile p
        StatsZ1 z1;
        z1.sel = sp + ST;
        z1.eps = eps_b;
        z1.N = Ne[p][1];
        if (!Ne[p][0] && !Ne[p][1]) continue;
        stats_wave(k[p], P, n_sig, T, B, STATS_PERCENTILE, sp, k[p], pct[p] / 100.0, prm.floor_rel,
                   eps_a, (double*)med, Ne[p][0], s, z1);
    }
    CSE_CHECK_LAUNCH("cse_noise_percentile_quad");
    return CSE_OK;
}

extern "C" int cse_noise_min_tracking_med(const double* P, const double* med, int64_t n_sig,
                                          int T, int B, double eps, float* N, double eps_b,
                                          float* N_b, void* workspace, cse_stream_t stream) {
    CSE_NOISE_SHAPE_CHECKS("cse_noise_min_tracking_med");
    CSE_CHECK_ARG(med && N && workspace, "cse_noise_min_tracking_med: NULL pointer");
    CSE_CHECK_ARG(T >= 5, "cse_noise_min_tracking_med: T=%d < 5 (use the simple estimate)", T);
    cse_noise_params_t prm;
    cse_noise_default_params(&prm);
    return launch_min_tracking(P, med, n_sig, T, B, prm, eps, N, eps_b, N_b,
                               carve(workspace, n_sig, T, B), (hipStream_t)stream);
}

extern "C" int cse_noise_finish(const cse_noise_job_t* jobs, int n_jobs, int64_t n_sig, int B,
                                const float* src, float* dst, cse_stream_t stream) {
    CSE_CHECK_ARG(jobs && src && dst && n_jobs >= 0 && n_jobs < 65536,
                  "cse_noise_finish: bad arguments");
    CSE_CHECK_ARG(n_sig > 0 && n_sig < 65536 && B >= 1, "cse_noise_finish: bad shape");
    if (n_jobs == 0) return CSE_OK;
    CSE_CHECK_ARG(B <= 256 * FIN_MAXU_BIG, "cse_noise_finish: B=%d > %d", B, 256 * FIN_MAXU_BIG);
    const dim3 grid((unsigned)n_sig, (unsigned)n_jobs);
    const size_t lds = (size_t)FIN_F * B * 4;
    const void* fn = B <= 256 * FIN_MAXU ? (const void*)finish_kernel<FIN_MAXU>
                                         : (const void*)finish_kernel<FIN_MAXU_BIG>;
    if (lds > 65536 && hipFuncSetAttribute(fn,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds) != hipSuccess) {
        ::cse::set_error("cse_noise_finish: cannot reserve %zu bytes of LDS", lds);
        return CSE_ELAUNCH;
    }
    void* args[] = {&jobs, &B, &src, &dst};
    if (hipLaunchKernel(fn, grid, dim3(256), args, lds, (hipStream_t)stream) != hipSuccess) {
        ::cse::set_error("cse_noise_finish: launch failed");
        return CSE_ELAUNCH;
    }
    CSE_CHECK_LAUNCH("cse_noise_finish");
    return CSE_OK;
}

extern "C" int cse_noise_smooth(const float* N, int64_t n_sig, int T, int B, int src_frames,
                                double mu, float* out, cse_stream_t stream) {
    CSE_CHECK_ARG(N && out, "cse_noise_smooth: NULL pointer");
    CSE_CHECK_ARG(n_sig > 0 && n_sig < 65536 && T >= 1 && B >= 1, "cse_noise_smooth: bad shape");
    CSE_CHECK_ARG(src_frames == 1 || src_frames == T, "cse_noise_smooth: src_frames=%d (1|T)",
                  src_frames);
    const double m = fmin(fmax(mu, 0.0), 0.9999);
    hipLaunchKernelGGL(smooth_kernel, dim3(ceil_div(B, 64), (unsigned)n_sig), dim3(64), 0,
                       (hipStream_t)stream, N, T, B, src_frames, m, out);
    CSE_CHECK_LAUNCH("cse_noise_smooth");
    return CSE_OK;
}

extern "C" int cse_noise_invert(const float* N, int64_t n, double eps, float* out,
                                cse_stream_t stream) {
    CSE_CHECK_ARG(N && out && n >= 0 && eps > 0.0, "cse_noise_invert: bad arguments");
    if (n == 0) return CSE_OK;
    hipLaunchKernelGGL(invert_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, N,
                       n, eps, out);
    CSE_CHECK_LAUNCH("cse_noise_invert");
    return CSE_OK;
}
