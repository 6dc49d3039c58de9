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
// through.  Per frame the cell's bins pass through a half-spectrum LDS buffer
// twice (mirror pairing for the real-IFFT packing, own bins stay in registers)
// and a half transpose block twice (16 x L transpose in two 8-row rounds); the
// two length-16 DFT passes run in registers.  The inverse FFT's outputs land
// on lanes so that every lane owns output samples with fixed residues mod 32
// (mod 64 @1024): the overlap-add accumulator never leaves registers, and
// each frame retires its HOP finished samples straight into the SNR sums.
// Nothing per-frame touches HBM except the (L2-shared) Y/N rows.
#include "cse_common.hpp"
#include "cse_special.hpp"

#ifndef CSE_PK
#define CSE_PK 1  // n_fft 512: packed f32 (v_pk_*) gain pairs, packing and DFTs
#endif

namespace cse {

template <int NFFT>
struct Geo {
    static constexpr int M = NFFT / 2;        // complex IFFT length
    static constexpr int B = M + 1;           // bins
    static constexpr int L = M / 16;          // lanes per cell
    static constexpr int CPW = 64 / L;        // cells per wave
    static constexpr int SP = NFFT / 16;      // spacing of a lane's output samples
};

struct Args {
    int64_t len;
    const cse_cell_t* cells;
    int64_t n_cells;
    const float2* Y;
    const float* noise;
    const double* clean;
    float* y_out;
    int64_t out_len;
    float* g_out;
    double* sse;
    uint8_t* finite;
};

#ifdef CSE_MARKS  // static instruction-count analysis builds only (tools/isa_sections.py)
#define CSE_MARK(name) asm volatile(";#MARK " name)
#elif defined(CSE_ENH_STAMPS)
// Per-stage timing (analysis builds only, tools/enhance_stages.py): at each
// stage marker, the shader cycles (s_memtime) since the previous marker go to
// the stage that just ended; wave 0 of every workgroup stores its sums, the
// (hop, algorithm) of the group beside them, into the buffer
// cse_enhance_stamp_buffer() installs
//   0 barrier + loop top   1 gain   2 mirror exchange   3 row staging
//   4 pass-1 DFT           5 transpose + pass-2 DFT      6 window    7 retire
static __device__ unsigned long long* g_enh_stamps;  // per translation unit
struct EnhStamps {
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long last = 0;
    __device__ void start() { last = __builtin_amdgcn_s_memtime(); }
    // the scheduling barriers keep each stage's instructions on their side of
    // the stamp (without them the compiler moved pass-1 arithmetic above the
    // pass-1 marker); the stamps still cost the waits they force
    __device__ void mark(int ended) {
        __builtin_amdgcn_sched_barrier(0);
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        acc[ended] += now - last;
        last = now;
    }
};
// the stage that ends at marker `name` (the markers are string literals)
__device__ constexpr int enh_stage_before(const char* n) {
    return n[0] == 'g' ? 0 : n[0] == 'x' ? 1 : (n[0] == 'r' && n[1] == 'o') ? 2
         : (n[0] == 'p' && n[4] == '1') ? 3 : n[0] == 'p' ? 4 : n[0] == 'w' ? 5
         : n[0] == 'r' ? 6 : 7;
}
#define CSE_MARK(name) est.mark(enh_stage_before(name))
#else
#define CSE_MARK(name)
#endif

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

// exp(-v/2)[(1+v)I0(v/2) + v I1(v/2)] for v in [1e-12, 80]
__device__ __forceinline__ float mmse_bracket(float v, float sqrtv) {
    // v<=4 -> PA(t); v>4 -> sqrt(v)*PB(t(1/v))
    const float ta = (v - 2.0f) * 0.5f;
    const float u = fast_rcp(v);
    const float tb = (2.0f * u - (CSE_HB_U0 + CSE_HB_U1)) * (1.0f / (CSE_HB_U1 - CSE_HB_U0));
    const float pa = horner(CSE_HA, ta);
    const float pb = horner(CSE_HB, tb);
    return v <= 4.0f ? pa : sqrtv * pb;
}

// ---------------------------------------------------------------------------
// per-bin gains.  The a-posteriori SNR gamma = max(P/max(N, eps), eps) depends
// only on the frame's spectrum row and noise row, which every cell of a
// workgroup shares: the row stager computes it once per bin and frame
// (P * inv with inv = 1/max(N, eps) from cse_noise_invert), and the cells read
// it from LDS.  The decision-directed recursion only ever uses
// prev_gain**2 * prev_gamma (wiener_filter.py:69, mmse.py:82,
// advanced_mmse.py:95): the carried state is rr = (G*G)*gamma.
// ---------------------------------------------------------------------------
// d = max(gamma - 1, 0) (the ML estimate of the DD rule) is per bin too: the
// n_fft = 512 stager stores the row (gamma, d) (cells compute d themselves at
// 1024, whose rows do not fit the LDS budget twice as wide).
// First frame: the reference uses xi = d (Wiener) / max(gamma-1, ksi_min)
// (MMSE, OMLSA); with rr = 0 and alpha_t = 0 on frame 0 the general DD
// expression alpha_t*rr + (1-alpha_t)*d gives exactly that (for ksi_min >= 0),
// so there is no per-bin branch to split the scheduling region.
// dd = (1 - alpha_t) d, the ML term's share (gain_bin forms it with the per-bin row)
__device__ __forceinline__ float gain_wiener(float gam, float dd, float& rr, float alpha_t,
                                             float gfloor) {
    const float xi = fmaxf(fmaf(alpha_t, rr, dd), 1e-10f);
    // np.clip as one v_med3; gfloor arrives as min(gain_floor, 1), numpy's
    // result when the bounds cross
    const float g = __builtin_amdgcn_fmed3f(xi * fast_rcp(1.0f + xi), gfloor, 1.0f);
    rr = (g * g) * gam;
    return g;
}

// cig = (sqrt(pi)/2) / (gamma + 1e-12), per bin from the row stager
__device__ __forceinline__ float gain_mmse(float gam, float dd, float cig, float& rr, float alpha_t,
                                           float ksi_min, float gmin, float gmax) {
    const float xi = fmaxf(fmaf(alpha_t, rr, dd), ksi_min);
    const float v = __builtin_amdgcn_fmed3f(xi * gam * fast_rcp(1.0f + xi), 1e-12f, 80.0f);
    const float sv = __builtin_amdgcn_sqrtf(v);
    const float h = mmse_bracket(v, sv);
    float g = (sv * cig) * h;
    // nan_to_num(nan -> gmin, +inf -> gmax, -inf -> gmin) + clip (mmse.py:98-104):
    // g is finite for finite input (v is clipped, cig finite), so the clip is
    // one v_med3 (gmin arrives as min(gain_min, gain_max): numpy's clip gives
    // gain_max when the bounds cross)
    g = __builtin_amdgcn_fmed3f(g, gmin, gmax);
    rr = (g * g) * gam;
    return g;
}

// Log-MMSE x speech-presence gain (advanced_mmse.py:100-121), in the log2 domain:
//   log2 g_lsa = log2(xi/(1+xi)) + 0.5 log2(e) E1(v)
//             = log2(xi r / sqrt(vc)) + Q(vc),  vc = min(v, 11.5)
//   with Q = 0.5 log2(e) (Ein - gamma_E) = Pn(vc)/Dn(vc), a (4, 3) rational
//   (tools/gen_special.py); for v >= 11.5 this differs from the exact form by
//   0.5 log2(e)(E1(11.5) - E1(v)) < 6e-7, no branch.
//   p = 1/(1 + (1-q)/(q Lambda + eps)) = A / (A + 1 - q),  A = q Lambda + eps
//   G = clip(g_lsa^p gf^(1-p), gf, 1) = clip(exp2(lgf + p (lg - lgf)), gf, 1)
//   p (lg - lgf) = A ((L - lgf) Dn + Pn) / ((A + 1 - q) Dn),  L = log2(xi r / sqrt(vc)):
//   the rational's quotient and p share one reciprocal (8 VALU for Q where a
//   degree-11 polynomial took 12).  Dn lies in [0.045, 1] and A <= e^80, so
//   neither (A + 1 - q) Dn nor A ((L - lgf) Dn + Pn) overflows.
// The bin works on v' = v log2(e), the exp2 argument of Lambda: gam2 = gamma
// log2(e) (the stager stores it so at both n_fft), the decision-directed state
// rr = G^2 gam2 (so its weight is alpha ln 2), the rational in v' and
// L' = log2(xr rsq(v')) = L - 0.5 log2(log2 e), the constant folded into lgf_c.
constexpr float kLn2 = 0.69314718055994531f;
constexpr float kLsaC = 0.26438318647244886f;  // 0.5 log2(log2 e)
// nan_to_num of g_lsa (advanced_mmse.py:106) needs no code: for finite input
// 0 <= X <= 1e6, so lg is finite or -inf (xi = 0 with ksi_min = 0), and -inf
// gives g = exp2(-inf) = 0 -> clip -> gain_floor, the reference's 0**p * gf**(1-p)
// clipped (p >= 1e-10 > 0).  Non-finite input makes the cell non-finite either way.
// gclip = min(gain_floor, 1): the lower bound of the final np.clip
__device__ __forceinline__ float gain_omlsa(float gam2, float dd, float& rr, float a_rr,
                                            float ksi_min, float gclip, float lg2_floor,
                                            float lgf_c, float eq, float cq, float vmax2) {
    const float xi = fmaxf(fmaf(a_rr, rr, dd), ksi_min);
    const float r = fast_rcp(1.0f + xi);
    const float xr = xi * r;
    const float v2 = __builtin_amdgcn_fmed3f(xr * gam2, 1e-12f * kLog2e, vmax2);
    const float vc2 = fminf(v2, CSE_LSA_VMAX2);
    const float pn = horner(CSE_LSAP, vc2);
    const float dn = horner(CSE_LSAD, vc2);
    const float L = fast_log2(xr * __builtin_amdgcn_rsqf(vc2));
    const float ev = fast_exp2(v2);
    // A = q Lambda + 1e-10 divided by q: A' = Lambda + eq (eq = 1e-10 / q), and
    // p = A / (A + 1 - q) = A' / (A' + cq) (cq = (1 - q) / q): one multiply less.
    // A' > 0 and cq > 0: p lies in (0, 1) up to a rounding, so the reference's
    // clip (advanced_mmse.py:116) needs no instruction
    const float A = fmaf(r, ev, eq);
    const float num = fmaf(L - lgf_c, dn, pn);
    const float den = (A + cq) * dn;
    const float g = fast_exp2(fmaf(A * num, fast_rcp(den), lg2_floor));
    const float G = __builtin_amdgcn_fmed3f(g, gclip, 1.0f);  // g >= 0, never NaN
    rr = (G * G) * gam2;
    return G;
}

// The reference's skip of a cell (speech_enhancement_comparison.py:102-103) as
// this kernel reports it: a slot that breaks the slot-group contract (cse.h)
__device__ __forceinline__ void reject_cell(const Args& a, int64_t c) {
    if (a.sse) a.sse[c] = __builtin_nan("");
    if (a.finite) a.finite[c] = 0;
}

// ---------------------------------------------------------------------------
// Block -> slot-group order.  Blocks are dealt round-robin over the 8 XCDs
// (block b runs on XCD b % 8, as its (b/8)-th block there), and the host sorts
// slot groups longest-first with groups that share rows adjacent.  Runs of
// RUN consecutive groups go to one XCD (L2 reuse of the shared Y/N rows inside
// a run) and the runs are dealt round-robin, which keeps the XCDs balanced
// (one contiguous slice per XCD gave XCD 0 all the longest groups:
// 46.7 -> 33.3 ms at 13 pairs, r01).  The tail that does not fill 8 runs keeps
// the identity order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcd_remap(int b, int nb) {
    constexpr int RUN = 4;
    const int xcd = b % 8, idx = b / 8;
    const int g = ((idx / RUN) * 8 + xcd) * RUN + idx % RUN;
    const int full = (nb / (8 * RUN)) * (8 * RUN);
    return b < full ? g : b;
}

// ---------------------------------------------------------------------------
// Workgroup = CSE_WG_WAVES waves = CPWG cells that share hop, algorithm,
// spectrum Y, noise row and clean reference (the host packs them so).  Per
// frame the workgroup stages the shared rows (Y[t][:], gamma[t][:] (N[t][:] for
// SS), clean[retired samples]) into LDS once, cooperatively, one frame ahead
// (a few VGPRs per thread).
// ---------------------------------------------------------------------------
template <int NFFT, bool OUT = false>
struct WG {
    using G = Geo<NFFT>;
    static constexpr int WAVES = NFFT == 512 ? CSE_WG_WAVES : CSE_WG_WAVES_1024;
    static constexpr int THREADS = 64 * WAVES;
    static constexpr int CPWG = WAVES * G::CPW;                   // cells per workgroup
    static constexpr int HMAX = 256;                              // largest hop
    // shared rows (double-buffered): Y (float2 [B]); G (float [B], or the
    // (gamma, d) / (N, P) float2 [B] at 512); A (float [B], 512: MMSE's
    // c/(gamma + 1e-12), SS's 1/|Y|); clean (float [HMAX])
    static constexpr bool R2 = (NFFT == 512);
    // packed pairs (CSE_PK, n_fft 512; packing the 1024 kernel measured slower,
    // DESIGN.md §3.1): the rows in mirror-pair order, 16-B records
    static constexpr bool PK = R2 && CSE_PK;
    // per-cell LDS region: the mirror-exchange slots (9 complex per lane,
    // stride 72 B: the 16 lanes of a ds_write_b64 group hit disjoint banks)
    // aliased with the transpose block (16 rows x TS = L + 1 complex).  Its
    // size is an odd multiple of 128 B, so the two cells of a 32-lane
    // ds_read_b64 group (n_fft 512) sit in disjoint bank halves of the
    // transposed reads.
    static constexpr int TS = G::L + 1;
    static constexpr int XB = G::L * 9 * 8;
    static constexpr int TB = 16 * TS * 8;
    static constexpr int CREG_RAW = XB > TB ? XB : TB;
    static constexpr int CREG_U = (CREG_RAW + 127) / 128;
    static constexpr int CREG = (CREG_U + (CREG_U % 2 ? 0 : 1)) * 128;
    static constexpr int YROW = ((G::B * 8 + 15) / 16) * 16;      // bytes of one Y row
    static constexpr int GROW = ((G::B * (R2 ? 8 : 4) + 15) / 16) * 16;
    static constexpr int AROW = R2 ? ((G::B * 4 + 15) / 16) * 16 : 0;
    static constexpr int OFF_Y = CPWG * CREG;                     // float2[2][B] (double buffer)
    static constexpr int OFF_G = OFF_Y + 2 * YROW;
    static constexpr int OFF_A = OFF_G + 2 * GROW;
    static constexpr int OFF_C = OFF_A + 2 * AROW;                // float[2][HMAX]
    static constexpr int CBUF = 2 * HMAX * 4;
    // n_fft 1024 keeps two tables small.  The window keeps slots q < 16, since
    // slot q + 16 is n + N/2 and w(n + N/2) = 1 - w(n) (the full 32-slot table
    // fits the LDS budget once the twiddles shrink, but measured 64.9 vs
    // 57.4 ms at 13 pairs).  The pass-1 twiddles are products of powers of
    // the lane's rotor r = e^{2πi i/M}: tw_b = r^(b mod 4) r^(4 (b div 4)), 9
    // complex products, from a per-lane row of r, r^2, r^3, r^4, r^8, r^12
    // (48 B; r02's two-rotor form, 16 B, squared and cubed them per frame: 4
    // products more).  The rotors replaced a 16-column table (keyed by b2,
    // times W32^{h2 b} and a select on the other half of the lanes): -35 VALU
    // and 7 of 8 LDS reads per frame, 58.2 -> 57.4 ms at 13 pairs.  n_fft 512
    // reads the full table (8 ds_read_b128).
    static constexpr bool HALF_TABLES = (NFFT == 1024);
    static constexpr bool ROTOR_TW = (NFFT == 1024);
    static constexpr int TWL = G::L;                              // twiddle columns (table form)
    // pass-1 twiddles (512): one row of 18 complex (144 B) per column, entry
    // b - 1: the ds_read_b128 of a 16-lane group hit disjoint banks;
    // (1024): cf[L][6] rotor powers
    static constexpr int OFF_TW = OFF_C + CBUF;
    // packing rotors e^{2πi (i + L j)/NFFT}: a row of the 8 (j < 8) per lane,
    // stride 80 B (20 dwords: the ds_read_b128 of a 16-lane group hit
    // disjoint banks), 4 ds_read_b128 per frame instead of 7 complex products
    // (n_fft 1024: base x W32^j; its 2.5-KB table pushed the workgroup past the
    // LDS budget, +11 %)
    static constexpr bool ROT_TABLE = R2;
    static constexpr int ROTSTR = 80;
    static constexpr int OFF_LC = OFF_TW + (ROTOR_TW ? G::L * 48 : TWL * 144);
    // sweep kernels (M2C, r06): bin M/2 of the slot group's cells is evaluated
    // by one wave per frame (wave t mod 4 evaluates frame t + 1 for all the
    // group's cells, one lane each) instead of by every lane of every cell.
    // Its decision-directed state and Z'[M/2] live, at 512, in the unused tail
    // of the twiddle table row of the cell's index (entries 15 and 16 / 17;
    // pass 1 reads entries 0..15 and uses 0..14), at 1024 in a region of its
    // own after the window table (160 B)
    static constexpr bool M2C = !OUT;

    static constexpr int OFF_CP = OFF_LC + G::L * (ROT_TABLE ? ROTSTR : 8);  // CellParam[CPWG]
    // synthesis window w(n)/(NFFT wss(n)) at the lane's 32 (16) sample slots,
    // wss the steady-state window-square sum of this workgroup's hop (librosa's
    // istft normalisation folded into the overlap-add); row stride 36 (20)
    // floats: the lanes of a ds_read_b128 group hit disjoint banks
    static constexpr int WSLOTS = HALF_TABLES ? 16 : 32;
    static constexpr int WSTR = HALF_TABLES ? 20 : 36;
    static constexpr int OFF_WIN = OFF_CP + CPWG * 32;
    static constexpr int OFF_M2 = OFF_WIN + G::L * WSTR * 4;
    static constexpr int BYTES = OFF_M2 + ((M2C && !R2) ? ((CPWG * 20 + 15) / 16) * 16 : 0);
    static constexpr int m2r(int c) {  // float rr of cell c
        return R2 ? OFF_TW + 144 * c + 120 : OFF_M2 + 16 * CPWG + 4 * c;
    }
    static constexpr int m2z(int c, int par) {  // f2 Z'[M/2] of cell c, frame parity par
        return R2 ? OFF_TW + 144 * c + 128 + 8 * par : OFF_M2 + 16 * c + 8 * par;
    }
    static_assert(!M2C || (WAVES == 4 && (!R2 || (CPWG <= TWL && !ROTOR_TW))), "M2C layout");
    static constexpr int YPT = (G::B + THREADS - 1) / THREADS;     // Y/N elements per thread
    static constexpr int CPT = (HMAX + THREADS - 1) / THREADS;     // clean samples per thread
};
// waves per SIMD the register allocation targets (VGPR budget 512 / w)
#ifndef CSE_WAVES_PER_SIMD
#define CSE_WAVES_PER_SIMD 3
#endif

// the registers set the occupancy: LDS must not cut it below CSE_WAVES_PER_SIMD
// (the sweep kernels) or 3 (the OUT variants) waves per SIMD
static_assert((163840 / WG<512, false>::BYTES) * WG<512, false>::WAVES >= 4 * CSE_WAVES_PER_SIMD,
              "n_fft=512 sweep workgroups must fit the register occupancy");
static_assert((163840 / WG<512, true>::BYTES) * WG<512, true>::WAVES >= 12,
              "n_fft=512 workgroups must fit 12 waves per CU");
static_assert((163840 / WG<1024>::BYTES) * WG<1024>::WAVES >= 12,
              "n_fft=1024 workgroups must fit 12 waves per CU");
static_assert(WG<512>::CPWG == CSE_CELLS_PER_GROUP(512) &&
              WG<1024>::CPWG == CSE_CELLS_PER_GROUP(1024), "cse.h slot-group size");


// Ordering of LDS accesses between the lanes of ONE wave: the LDS executes a
// wave's DS instructions in issue order, so a compiler-level barrier is all a
// write->read or read->write hand-off inside the wave needs (no s_waitcnt).
// an LDS byte offset the compiler cannot relate to others: two reads from
// different opaque bases are never merged into one ds_read2 / wide read
__device__ __forceinline__ int opaque_off(int off) {
    asm volatile("" : "+v"(off));
    return off;
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// per-cell parameters as the gain stage wants them
struct CellParam {
    // OMLSA: q_spp = 1e-10 / q and p3 = (1 - q) / q (q clamped to [1e-3, 1 - 1e-3]),
    // gclip = min(gain_floor, 1)
    float p0, p1, p2, p3, p4, lg2_floor, q_spp, gclip;
};
static_assert(sizeof(CellParam) == 32, "CellParam layout");

// One bin's shared row values (staged once per workgroup and frame):
//   Wiener/MMSE/OMLSA: g = gamma (OMLSA: gamma log2(e)), d = max(gamma - 1, 0) (512; 1024 computes d
//     here), a = (sqrt(pi)/2)/(gamma + 1e-12) (MMSE at 512);
//   SS at 512: g = N, d = P = |Y|^2, a = 1/|Y| (gain output only), and the Y
//     row holds the unit phasor of Y instead of Y ((1, 0) where Y = 0);
//   SS at 1024: g = N with Y itself.
struct RowV {
    float g, d, a;
};

// Returns the real factor s with S = y s (y possibly replaced: SS at 1024 with
// Y = 0); the packing forms the products inside its sums and differences.
template <int NFFT, int ALGO>
__device__ __forceinline__ float gain_bin(float2& y, RowV rv, float& rr, float alpha_t,
                                          const CellParam& cp, float& g) {
    constexpr bool R2 = (NFFT == 512);
    if (ALGO == CSE_ALGO_SS) {
        // Ps = max(P - a N, b N); |S| = sqrt(Ps) with the noisy phase
        // (spectral_subtractor.py:44-53).  No eps floor: the reference floors
        // BEFORE fix_length (engine.noise_key).
        // The raw v_sqrt/v_rsq treat denormal inputs as 0, and a near-silent
        // clip (fix_length zero-pads N, so Ps = P) reaches them: sqrt is
        // taken of a rescaled Ps below 2^-96, and the noisy phase y/|y| of a
        // rescaled y below 2^-50 (by the stager at 512).
        const float N = rv.g;
        const float P = R2 ? rv.d : y.x * y.x + y.y * y.y;
        const float ps = fmaxf(P - cp.p0 * N, cp.p1 * N);
        const bool tiny_ps = ps < 0x1p-96f;
        const float sp = __builtin_amdgcn_sqrtf(tiny_ps ? ps * 0x1p64f : ps) *
                         (tiny_ps ? 0x1p-32f : 1.0f);
        if (R2) {  // y is the phasor
            g = sp * rv.a;
            return sp;
        }
        const float sc = fmaxf(fabsf(y.x), fabsf(y.y)) < 0x1p-50f ? 0x1p64f : 1.0f;
        const float yx = y.x * sc, yy = y.y * sc;
        const float pz = fmaf(yx, yx, yy * yy);
        const float u = sp * __builtin_amdgcn_rsqf(pz);
        g = (pz > 0.0f) ? u * sc : 0.0f;
        // angle(0) = 0; a NaN/inf spectrum value keeps the NaN phase np.angle gives it
        y = (pz > 0.0f) ? make_float2(yx, yy)
                        : (pz == 0.0f ? make_float2(1.0f, 0.0f) : make_float2(pz - pz, pz - pz));
        return (pz > 0.0f) ? u : sp;
    }
    // dd = (1 - alpha_t) max(gamma - 1, 0): at 512 d is the stager's row; at 1024
    // max((1 - alpha_t) gamma - (1 - alpha_t), 0), one FMA and a max (OMLSA's row
    // holds gamma log2(e) at both n_fft, so its FMA takes (1 - alpha_t) ln 2).
    // The per-frame weights are common to the bins (hoisted).
    const float a_d = 1.0f - alpha_t;
    const float dd = R2 ? a_d * rv.d
                        : fmaxf(fmaf(rv.g, ALGO == CSE_ALGO_OMLSA ? a_d * kLn2 : a_d, -a_d), 0.0f);
    if (ALGO == CSE_ALGO_WIENER) {
        g = gain_wiener(rv.g, dd, rr, alpha_t, cp.p1);
    } else if (ALGO == CSE_ALGO_MMSE) {
        const float cig = R2 ? rv.a : 0.88622692545275801f * fast_rcp(rv.g + 1e-12f);
        g = gain_mmse(rv.g, dd, cig, rr, alpha_t, cp.p1, cp.p2, cp.p3);
    } else {
        g = gain_omlsa(rv.g, dd, rr, alpha_t * kLn2, cp.p1, cp.gclip, cp.lg2_floor,
                       cp.lg2_floor - kLsaC, cp.q_spp, cp.p3, cp.p4 * kLog2e);
    }
    return g;
}

// ---------------------------------------------------------------------------
// Packed gain of one mirror pair (bins k, M - k) at n_fft 512 (CSE_PK): the
// same operations as gain_wiener / gain_mmse / gain_omlsa on the two bins at
// once, every multiply/add/FMA one v_pk_* instruction; max/med3/min and the
// transcendentals stay per bin (gfx950 has no packed forms of them).  The
// rows are in pair order (the stager's layout): gam = (gamma_k, gamma_{M-k})
// (OMLSA: times log2 e), d = (d_k, d_{M-k}), a = MMSE's (c/(gamma + 1e-12))
// pair.  Returns the pair's gains; rr is the pair's decision-directed state.
// ---------------------------------------------------------------------------
// a polynomial on both lanes, packed (coefficients from SGPR pairs; as two
// scalar chains with literal coefficients, r04: 24.1 against 23.1 ms at 13 pairs)
template <int N>
__device__ __forceinline__ f2 horner2(const float (&c)[N], f2 t) {
    f2 acc = pdup(c[N - 1]);
#pragma unroll
    for (int k = N - 2; k >= 0; --k) acc = pfma(acc, t, pdup(c[k]));
    return acc;
}
__device__ __forceinline__ f2 prcp(f2 x) { return f2{fast_rcp(x.x), fast_rcp(x.y)}; }
__device__ __forceinline__ f2 pmed3(f2 x, float lo, float hi) {
    return f2{__builtin_amdgcn_fmed3f(x.x, lo, hi), __builtin_amdgcn_fmed3f(x.y, lo, hi)};
}
__device__ __forceinline__ f2 pmax(f2 x, float lo) { return f2{fmaxf(x.x, lo), fmaxf(x.y, lo)}; }

template <int ALGO>
__device__ __forceinline__ f2 gain_pair(f2 gam, f2 d, f2 a, f2& rr, float alpha_t, const CellParam& cp) {
    // dd = (1 - alpha_t) max(gamma - 1, 0) from the stager's d row
    const f2 dd = d * pdup(1.0f - alpha_t);
    if (ALGO == CSE_ALGO_WIENER) {
        const f2 xi = pmax(pfma(pdup(alpha_t), rr, dd), 1e-10f);
        const f2 g = pmed3(xi * prcp(xi + 1.0f), cp.p1, 1.0f);
        rr = (g * g) * gam;
        return g;
    } else if (ALGO == CSE_ALGO_MMSE) {
        const f2 cig = a;  // the stager's (sqrt(pi)/2)/(gamma + 1e-12) row
        const f2 xi = pmax(pfma(pdup(alpha_t), rr, dd), cp.p1);
        const f2 v = pmed3((xi * gam) * prcp(xi + 1.0f), 1e-12f, 80.0f);
        const f2 sv = f2{__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
        // mmse_bracket on the pair
        const f2 ta = pfma(v, pdup(0.5f), pdup(-1.0f));  // (v - 2)/2
        const f2 u = prcp(v);
        const f2 tb = pfma(u, pdup(2.0f / (CSE_HB_U1 - CSE_HB_U0)),
                           pdup(-(CSE_HB_U0 + CSE_HB_U1) / (CSE_HB_U1 - CSE_HB_U0)));
        const f2 pa = horner2(CSE_HA, ta);
        const f2 pb = sv * horner2(CSE_HB, tb);
        const f2 h = f2{v.x <= 4.0f ? pa.x : pb.x, v.y <= 4.0f ? pa.y : pb.y};
        const f2 g = pmed3((sv * cig) * h, cp.p2, cp.p3);
        rr = (g * g) * gam;
        return g;
    } else {  // OMLSA, see gain_omlsa
        const f2 xi = pmax(pfma(pdup(alpha_t * kLn2), rr, dd), cp.p1);
        const f2 r = prcp(xi + 1.0f);
        const f2 xr = xi * r;
        const float vmax2 = cp.p4 * kLog2e;
        const f2 v2 = pmed3(xr * gam, 1e-12f * kLog2e, vmax2);
        const f2 vc2 = f2{fminf(v2.x, CSE_LSA_VMAX2), fminf(v2.y, CSE_LSA_VMAX2)};
        const f2 pn = horner2(CSE_LSAP, vc2);
        const f2 dn = horner2(CSE_LSAD, vc2);
        const f2 xs = xr * f2{__builtin_amdgcn_rsqf(vc2.x), __builtin_amdgcn_rsqf(vc2.y)};
        const f2 L = f2{fast_log2(xs.x), fast_log2(xs.y)};
        const f2 ev = f2{fast_exp2(v2.x), fast_exp2(v2.y)};
        const f2 A = pfma(r, ev, pdup(cp.q_spp));  // A / q, see gain_omlsa
        const f2 num = pfma(L - pdup(cp.lg2_floor - kLsaC), dn, pn);
        const f2 den = (A + pdup(cp.p3)) * dn;
        const f2 e = pfma(A * num, prcp(den), pdup(cp.lg2_floor));
        const f2 G = pmed3(f2{fast_exp2(e.x), fast_exp2(e.y)}, cp.gclip, 1.0f);
        rr = (G * G) * gam;
        return G;
    }
}

// One frame's gain stage + real-IFFT packing for one lane, packed (CSE_PK,
// pair-order rows): per mirror pair the gains of both bins (gain_pair; SS per
// bin through gain_bin), then
//   X_k = Y_k g_k,  conj(X_{M-k}) = Y_{M-k} (g', -g'),  g' = g_{M-k}
//   S = X_k + conj(X_{M-k}),  D = X_k - conj(X_{M-k}),  P = D w
//   Z'[k] = S + i P,  Z'[M - k] = conj(S) + i conj(P)
// (8 packed instructions per pair).  z[j] keeps Z'[k]; xw[j] goes to the
// mirror lane.  Bin M/2 (the 17th item) stays scalar (gain_bin).  Rows: Y
// records (Y_p, Y_{M-p}) (16 B), (g_p, g_{M-p}, d_p, d_{M-p}) (16 B) and
// MMSE's / SS's a pairs (8 B).  Packing rotors: the lane's table row.
template <int NFFT, int ALGO, bool OUT, bool M2C>
__device__ __forceinline__ void gain_pack_pk(const float4* __restrict__ y4row,
                                             const void* __restrict__ growv,
                                             const float2* __restrict__ a2row, f2 (&z)[16],
                                             f2* __restrict__ xw, f2 (&rr)[8], float& rrm,
                                             float alpha_t, const CellParam& cpar,
                                             const float4* __restrict__ rot4,
                                             float* __restrict__ gout_row, int i) {
    // (instantiated for 1024 too, where W::PK is false and the frame never calls it)
    constexpr int L = Geo<NFFT>::L, M = Geo<NFFT>::M;
    constexpr bool WANT_A = ALGO == CSE_ALGO_MMSE || (ALGO == CSE_ALGO_SS && OUT);
    const float4* y4 = y4row + i;
    const float4* g4 = (const float4*)growv + i;
    const float2* a2 = a2row + i;
    // the records through a by-value copy: reading g4[k] in place lets the
    // compiler turn bin M/2's two 4-byte reads into a ds_read_b128 and
    // reschedule the frame; this form keeps r05's measured instruction stream
    auto ldg = [&](int k) -> float4 { const float4 v = g4[k]; return v; };
    float4 yc = y4[0], gc = ldg(0);
    float2 ac = WANT_A ? a2[0] : make_float2(0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        // next pair's rows (j = 7: bin M/2, the record of pair M/2, unless
        // another wave evaluates it, M2C)
        const int nx = (j < 7) ? L * (j + 1) : M / 2 - i;
        const bool nxt = j < 7 || !M2C;
        const float4 yn = nxt ? y4[nx] : float4{}, gn = nxt ? ldg(nx) : float4{};
        const float2 an = (WANT_A && nxt) ? a2[nx] : make_float2(0.0f, 0.0f);
        f2 ya = f2{yc.x, yc.y}, yb = f2{yc.z, yc.w};
        f2 g;  // the pair's gains
        f2 s;  // the real factors of S = Y s (SS: sqrt(Ps) on the unit phasor)
        if (ALGO == CSE_ALGO_SS) {
            float2 y0 = make_float2(ya.x, ya.y), y1 = make_float2(yb.x, yb.y);
            float g0, g1, dummy = 0.0f;
            const float s0 = gain_bin<NFFT, ALGO>(y0, RowV{gc.x, gc.z, ac.x}, dummy, alpha_t, cpar, g0);
            const float s1 = gain_bin<NFFT, ALGO>(y1, RowV{gc.y, gc.w, ac.y}, dummy, alpha_t, cpar, g1);
            g = f2{g0, g1};
            s = f2{s0, s1};
        } else {
            g = gain_pair<ALGO>(f2{gc.x, gc.y}, f2{gc.z, gc.w}, f2{ac.x, ac.y}, rr[j],
                                 alpha_t, cpar);
            s = g;
        }
        if (OUT && gout_row) {
            gout_row[i + L * j] = g.x;
            gout_row[M - i - L * j] = g.y;
        }
        if (j == 0 && i == 0) {  // irfft ignores Im of DC and Nyquist
            ya.y = 0.0f;
            yb.y = 0.0f;
        }
        const f2 xk = ya * s.xx;
        const f2 S = p_fma_conj_hi(yb, s, xk), D = p_fms_conj_hi(yb, s, xk);
        const float4 q4 = rot4[j >> 1];  // two packing rotors
        const f2 w = (j & 1) ? f2{q4.z, q4.w} : f2{q4.x, q4.y};
        const f2 P = p_cmul(D, w);
        z[j] = p_addi(S, P);                      // Z'[k] = S + i P
        xw[j] = p_conj_addi(S, P);                // Z'[M - k] = conj(S) + i conj(P)
        yc = yn;
        gc = gn;
        ac = an;
    }
    // bin M/2: scalar, Z'[M/2] = 2 conj(X_{M/2}) (M2C: run_wg's m2_eval)
    if constexpr (!M2C) {
        float2 ym = make_float2(yc.x, yc.y);
        float gm;
        const float sm = 2.0f * gain_bin<NFFT, ALGO>(ym, RowV{gc.x, gc.z, ac.x}, rrm, alpha_t, cpar, gm);
        if (OUT && gout_row && i == 0) gout_row[M / 2] = gm;
        xw[8] = f2{ym.x * sm, -ym.y * sm};
    }
}

// One frame's gain stage + real-IFFT packing for one lane.
//
// Bin ownership: lane i holds the 8 mirror pairs (k, M - k), k = i + L j
// (j < 8), i.e. bins [0, M/2) and (M/2, M] once each, plus bin M/2 (its own
// mirror) as a 17th item that every lane of the cell evaluates alike (only
// lane 0's is used).  The inverse real FFT is a complex IFFT of length M of
//   Z'[k] = (X_k + X*_{M-k}) + i (X_k - X*_{M-k}) e^{2πi k/NFFT},
// and both halves of a pair come out of one lane:
//   S = X_k + X*_{M-k}, D = X_k - X*_{M-k}, P = D e^{2πi k/NFFT}
//   Z'[k] = S + i P,   Z'[M - k] = conj(S) + i conj(P)
// Z'[k] (class i, index j) stays in the lane; Z'[M - k] = Z'[(L - i) + L (15 - j)]
// goes to lane (L - i) mod L through a 9-entry LDS slot per lane.  Lane 0
// keeps the DC/Nyquist pair (Im ignored, as irfft does) and bin M/2, whose
// Z' = 2 conj(X_{M/2}).
// Rows: yrow (float2 [B]), grow (float [B], or float2 [B] at 512) and arow
// (float [B], 512: MMSE, and SS when the gain is written) of this frame.  They
// are __restrict__, so the scheduler may issue the bins' reads up front and
// interleave the independent gain chains.  The packing rotors e^{2πi (i + L j)/NFFT}
// come from the lane's LDS row (8 complex).
template <int NFFT, int ALGO, bool OUT, bool M2C>
__device__ __forceinline__ void gain_pack(const float2* __restrict__ yrow,
                                          const void* __restrict__ growv,
                                          const float* __restrict__ arow, cf (&z)[16],
                                          cf* __restrict__ xw, float (&rr)[17], float alpha_t,
                                          const CellParam& cpar, const float4* __restrict__ rot4,
                                          const cf* __restrict__ base_p, float* __restrict__ gout_row,
                                          int i) {
    constexpr int L = Geo<NFFT>::L, M = Geo<NFFT>::M;
    constexpr bool R2 = (NFFT == 512);
    constexpr bool WANT_A = R2 && (ALGO == CSE_ALGO_MMSE || (ALGO == CSE_ALGO_SS && OUT));
    // per-lane bases (lo: bin i, hi: bin M - i - 7L) so that every bin's
    // address is base + a compile-time immediate
    const float2* ylo = yrow + i;
    const float2* yhi = yrow + (M - i - 7 * L);
    const float* alo = arow + i;
    const float* ahi = arow + (M - i - 7 * L);
    const float2* g2lo = (const float2*)growv + i;
    const float2* g2hi = (const float2*)growv + (M - i - 7 * L);
    const float* g1lo = (const float*)growv + i;
    const float* g1hi = (const float*)growv + (M - i - 7 * L);
    // hi: bin M - i - L j is index L (7 - j) from its base; M/2 is index M/2 - i
    // from the lo base
    auto ld = [&](bool hi, int k, float2& y, RowV& rv) {
        y = hi ? yhi[k] : ylo[k];
        if constexpr (R2) {
            const float2 g2 = hi ? g2hi[k] : g2lo[k];
            rv.g = g2.x;
            rv.d = g2.y;
        } else {
            rv.g = hi ? g1hi[k] : g1lo[k];
            rv.d = 0.0f;
        }
        rv.a = WANT_A ? (hi ? ahi[k] : alo[k]) : 0.0f;
    };
    // lane i: bins k = i + L j (lo) and M - i - L j (hi), j < 8, then M/2.
    // The next pair's reads are issued before this pair's gains; the
    // scheduler may interleave neighbouring pairs' chains (a memory fence per
    // pair, which kept it from doing so, measured 0.3 % slower at 3 waves/SIMD).
    float2 ya, yb;
    RowV ga, gb;
    ld(false, 0, ya, ga);
    ld(true, 7 * L, yb, gb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float2 yan, ybn;
        RowV gan, gbn;
        if (j < 7) {
            ld(false, L * (j + 1), yan, gan);
            ld(true, L * (6 - j), ybn, gbn);
        } else if (M2C) {  // bin M/2: another wave evaluates it (run_wg's m2_eval)
            yan = make_float2(0.0f, 0.0f);
            gan = RowV{0.0f, 0.0f, 0.0f};
        } else {
            // bin M/2 (the same for every lane): base - i + M/2
            yan = yrow[M / 2];
            if constexpr (R2) {
                const float2 g2 = ((const float2*)growv)[M / 2];
                gan.g = g2.x;
                gan.d = g2.y;
            } else {
                gan.g = ((const float*)growv)[M / 2];
                gan.d = 0.0f;
            }
            gan.a = WANT_A ? arow[M / 2] : 0.0f;
        }
        float g0, g1;
        const float sa = gain_bin<NFFT, ALGO>(ya, ga, rr[j], alpha_t, cpar, g0);
        const float sb = gain_bin<NFFT, ALGO>(yb, gb, rr[8 + j], alpha_t, cpar, g1);
        if (OUT && gout_row) {
            gout_row[i + L * j] = g0;
            gout_row[M - i - L * j] = g1;
        }
        if (j == 0 && i == 0) {  // irfft ignores Im of DC and Nyquist
            ya.y = 0.0f;
            yb.y = 0.0f;
        }
        // S = X_k + X*_{M-k}, D = X_k - X*_{M-k} with X_k = ya sa, X_{M-k} = yb sb:
        // the X_k products ride in the FMAs (6 VALU instead of 8)
        const float bx = yb.x * sb, by = yb.y * sb;
        const float sx = fmaf(ya.x, sa, bx), sy = fmaf(ya.y, sa, -by);
        const float dx = fmaf(ya.x, sa, -bx), dy = fmaf(ya.y, sa, by);
        // packing rotor e^{2πi (i + L j)/NFFT}: the lane's table row, or base * W32^j
        cf w;
        if constexpr (WG<NFFT>::ROT_TABLE) {
            const float4 q4 = rot4[j >> 1];  // ds_read_b128: two rotors
            w = (j & 1) ? cmk(q4.z, q4.w) : cmk(q4.x, q4.y);
        } else {
            const cf base = *base_p;
            w = (j == 0) ? base : cmul(base, cmk(Rot32::c[j], Rot32::s[j]));
        }
        const float px = fmaf(dx, w.x, -dy * w.y), py = fmaf(dx, w.y, dy * w.x);
        z[j] = cmk(sx - py, sy + px);
        xw[j] = cmk(sx + py, px - sy);  // Z'[M - k] for the mirror lane
        ya = yan;
        ga = gan;
        if (j < 7) {
            yb = ybn;
            gb = gbn;
        }
    }
    if constexpr (!M2C) {
        float gm;
        const float sm = 2.0f * gain_bin<NFFT, ALGO>(ya, ga, rr[16], alpha_t, cpar, gm);
        if (OUT && gout_row && i == 0) gout_row[M / 2] = gm;
        xw[8] = cmk(ya.x * sm, -ya.y * sm);
    }
}

// Position inside a frame (relative to the lane's first sample) of the lane's
// output slot q: the pass-2 DFT16 gives lane b2 the samples 2 b2 + SP p + e
// (slot q = 2 p + e), so slot q + F lies HOP samples after slot q.
template <int SP>
__device__ __forceinline__ constexpr int slot_pos(int q) {
    return SP * (q >> 1) + (q & 1);
}

template <int NFFT, int HOP, int ALGO, bool OUT>
__device__ __forceinline__ void run_wg(const Args& a, const cse_cell_t* wcell, int n_cells_wg,
                                       unsigned char* smem) {
    using G = Geo<NFFT>;
    using W = WG<NFFT, OUT>;
    constexpr int M = G::M, L = G::L, B = G::B, SP = G::SP, MH = M / 2;
    constexpr int R = NFFT / HOP;       // frames overlapping one sample
    constexpr int F = 2 * HOP / SP;     // samples a lane retires per frame
    constexpr int PEND = 32 - F;        // overlap-add sums carried to the next frame
    static_assert(F >= 2 && F <= 32 && (F % 2) == 0, "hop/n_fft combination");
    // gamma floor of each algorithm (wiener_filter.py:61, mmse.py:74, advanced_mmse.py:90)
    constexpr float EPS = (ALGO == CSE_ALGO_MMSE) ? 1e-12f : 1e-10f;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int cs = lane / L, i = lane % L;
    const int cslot = wave * G::CPW + cs;
    const int creg = cslot * W::CREG;   // byte offset of my cell's region

    // ---- the shared rows of this workgroup (first cell's; host-validated)
    const int len = (int)a.len;
    const float2* Ybase = a.Y + wcell[0].y_offset;
    const float* Nbase = a.noise + wcell[0].noise_offset;
    const int nstride = (int)wcell[0].noise_stride;
    const int lag = wcell[0].lag;  // shared by the slot group (host-validated)
    const double* cbase = (a.clean && wcell[0].clean_offset >= 0) ? a.clean + wcell[0].clean_offset
                                                                  : nullptr;
    const int T = 1 + len / HOP;
    const int need = (len + NFFT + HOP - 1) / HOP;
    const int nf = need < T ? need : T;

    // ---- my cell.  The slot group's shared rows are slot 0's; a slot whose
    // shared fields differ from slot 0's (cse.h: algo, hop, y_offset,
    // noise_offset, noise_stride, clean_offset, lag) is not computed: it gets
    // the reference's skip (finite = 0, sse = NaN), written here, never
    // uninitialised outputs.  Padding slots (CSE_ALGO_NONE) write nothing.
    bool valid = false;
    if (cslot < n_cells_wg && wcell[cslot].algo != CSE_ALGO_NONE) {
        const cse_cell_t* me = wcell + cslot;
        valid = me->algo == ALGO && me->hop == HOP && me->y_offset == wcell[0].y_offset &&
                me->noise_offset == wcell[0].noise_offset &&
                me->noise_stride == wcell[0].noise_stride &&
                me->clean_offset == wcell[0].clean_offset && me->lag == wcell[0].lag;
        if (!valid && i == 0) reject_cell(a, (int64_t)(me - a.cells));
    }
    // waveform output (any variant) and gain output (OUT variant only)
    const bool want_y = a.y_out != nullptr;  // uniform
    const int out_len = (int)a.out_len;
    float* yout = nullptr;
    float* gout = nullptr;
    if (valid) {
        const cse_cell_t* cp = wcell + cslot;
        if (want_y && cp->out_offset >= 0) yout = a.y_out + cp->out_offset;
        if (OUT && cp->gain_offset >= 0 && a.g_out) gout = a.g_out + cp->gain_offset;
    }

    // ---- workgroup tables: pass-1 twiddles e^{2πi i b/M} [b-1][i], lane
    // constants [i], cell parameters [slot]
    if constexpr (W::ROTOR_TW) {
        // per lane r^p, p = 1, 2, 3, 4, 8, 12 (r = e^{2πi ii/M}): a 48-B row, the
        // ds_read_b128 of a 16-lane group on disjoint banks (stride 12 dwords)
        for (int e = tid; e < 6 * L; e += W::THREADS) {
            const int ii = e / 6, k = e - 6 * (e / 6);
            const int pw = k < 3 ? k + 1 : 4 * (k - 2);
            double s, c;
            sincospi(2.0 * (double)(ii * pw) / (double)M, &s, &c);
            ((cf*)(smem + W::OFF_TW))[e] = cmk((float)c, (float)s);
        }
    } else {
        for (int e = tid; e < 15 * W::TWL; e += W::THREADS) {
            const int b = 1 + e % 15, ii = e / 15;
            double s, c;
            sincospi(2.0 * (double)(ii * b) / (double)M, &s, &c);
            ((cf*)(smem + W::OFF_TW))[ii * 18 + b - 1] = cmk((float)c, (float)s);
        }
    }
    // lane tables: packing rotors e^{2πi (ii + L j)/NFFT} (512: j < 8; 1024: j = 0);
    // window w(n)/(NFFT S(n)) at the lane's sample slots q (n = SP*(q>>1) + off +
    // (q&1)), S(n) = sum over m = n mod HOP + r HOP < NFFT of w(m)^2, the
    // steady-state window-square sum librosa's istft divides by (1.5 for
    // R = 4, 3 for R = 8, 0.75 + 0.25 cos(2π n/256) for 512/256)
    for (int e = tid; e < L * 32; e += W::THREADS) {
        const int ii = e / 32, q = e % 32;
        const int bb = (L == 16) ? ii : (ii & 15), hh = (L == 16) ? 0 : (ii >> 4);
        const int n = 2 * bb + 32 * hh + slot_pos<SP>(q);
        const double w = 0.5 - 0.5 * cospi(2.0 * (double)n / (double)NFFT);
        double S = 0.0;
        for (int m = n % HOP; m < NFFT; m += HOP) {
            const double wm = 0.5 - 0.5 * cospi(2.0 * (double)m / (double)NFFT);
            S += wm * wm;
        }
        if (q < W::WSLOTS) ((float*)(smem + W::OFF_WIN))[ii * W::WSTR + q] = (float)(w / (NFFT * S));
        if (W::ROT_TABLE ? q < 8 : q == 0) {
            double sn, cn;
            sincospi(2.0 * (double)(ii + L * q) / (double)NFFT, &sn, &cn);
            ((cf*)(smem + W::OFF_LC + (W::ROT_TABLE ? W::ROTSTR : 8) * ii))[q] =
                cmk((float)cn, (float)sn);
        }
    }
    for (int c = tid; c < W::CPWG; c += W::THREADS) {
        const cse_cell_t* cp = wcell + (c < n_cells_wg ? c : 0);
        CellParam prm;
        prm.p0 = cp->param[0];
        prm.p1 = cp->param[1];
        prm.p2 = cp->param[2];
        prm.p3 = cp->param[3];
        prm.p4 = cp->param[4];
        prm.lg2_floor = (ALGO == CSE_ALGO_OMLSA) ? fast_log2(prm.p2) : 0.0f;
        prm.q_spp = 0.0f;
        if (ALGO == CSE_ALGO_OMLSA) {  // see gain_omlsa: A and p divided by q
            const double q = fmin(fmax((double)prm.p3, 1e-3), 1.0 - 1e-3);
            prm.q_spp = (float)(1e-10 / q);
            prm.p3 = (float)((1.0 - q) / q);
        }
        prm.gclip = 0.0f;
        // clip bounds for one v_med3: the lower bound capped at the upper one
        // (numpy's clip returns the upper bound when they cross)
        if (ALGO == CSE_ALGO_WIENER) prm.p1 = fminf(prm.p1, 1.0f);
        if (ALGO == CSE_ALGO_MMSE) prm.p2 = fminf(prm.p2, prm.p3);
        if (ALGO == CSE_ALGO_OMLSA) prm.gclip = fminf(prm.p2, 1.0f);
        // v enters the OMLSA gain only through e^v (the E1 term takes min(v, 11.5)),
        // and at v = 80 the speech-presence p = A/(A + 1 - q) is already 1 in fp32
        // (A >= 1e-3 e^80 / (1 + 1e16)): v_max beyond 80 changes nothing but
        // would overflow e^v (fp32 max e^88.7), so it is capped here
        if (ALGO == CSE_ALGO_OMLSA) prm.p4 = fminf(prm.p4, 80.0f);
        ((CellParam*)(smem + W::OFF_CP))[c] = prm;
    }

    // ---- row staging: thread tid owns Y/N elements tid + u*THREADS, clean tid + u*THREADS
    float2 py[W::YPT];
    float pn[W::YPT];  // N (SS) or 1/max(N, eps); a static row stays here for the whole cell
    // clean samples stay f64 in flight: converting at load time made the
    // compiler wait (vmcnt(0)) for every row load right after issuing them
    double pc[W::CPT];
    // n_fft 512: the row loads through buffer resources, branch-free (r05, 13
    // pairs, three alternating rounds: 22.50 / 22.51 / 22.51 -> 22.06 / 22.09 /
    // 22.10 ms; at 1024 55.5 / 55.3 against 54.9 / 55.3 ms, so 1024 keeps the
    // masked loads)
    constexpr bool ROWS_BUF = NFFT == 512;
    // ROWS_BUF: the row loads through buffer resources (r05): an index past a
    // row's end returns 0 instead of taking a per-lane branch.  Y: the
    // workgroup's nf frames; N: the same for a time-varying row, the static row
    // itself re-read every frame when nstride = 0; clean: [0, len), so the
    // clean samples outside the signal read 0 without the range test
    // (negative offsets wrap to huge unsigned values; a NULL clean has no
    // records).  Offsets go through opaque_off: a constant folded into the
    // instruction's immediate field would escape the range check.  One
    // resource per array, not per row and frame (per-frame resources measured
    // 22.46 against 22.58 ms, per-array 22.08 against 22.51; per-array with a
    // workgroup-uniform fallback to the masked loads for rows past 2 GiB
    // 23.24 against 22.53).  Byte offsets are 32-bit: the entry point takes
    // n_fft 512 signals whose spectrum rows stay below 2 GiB (cse.h).
    const __amdgpu_buffer_rsrc_t yrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)Ybase, (short)0, ROWS_BUF ? nf * B * 8 : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t nrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)Nbase, (short)0, ROWS_BUF ? ((nstride ? (nf - 1) * nstride : 0) + B) * 4 : 0,
        0x00020000);
    const __amdgpu_buffer_rsrc_t crc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)cbase, (short)0, ROWS_BUF && cbase ? len * 8 : 0, 0x00020000);
    auto load_rows = [&](int t) {  // issue loads of frame t's rows into registers
      if constexpr (ROWS_BUF) {
        if (t < nf) {
#pragma unroll
            for (int u = 0; u < W::YPT; ++u) {
                const int k = tid + u * W::THREADS;  // k >= B: not stored (store_rows)
                py[u] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                    yrc, opaque_off(8 * (t * B + k)), 0, 0));
                pn[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    nrc, opaque_off(4 * (t * nstride + k)), 0, 0));
            }
        }
#pragma unroll
        for (int u = 0; u < W::CPT; ++u) {
            const int j = tid + u * W::THREADS;
            const int o = t * HOP - NFFT / 2 + j + lag;  // clean sample scored against y[o - lag]
            if (j < HOP)  // uniform per wave
                pc[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                    crc, opaque_off(8 * o), 0, 0));
        }
      } else {
        if (t < nf) {
#pragma unroll
            for (int u = 0; u < W::YPT; ++u) {
                const int k = tid + u * W::THREADS;
                if (k < B) {
                    py[u] = Ybase[t * B + k];
                    if (nstride) pn[u] = Nbase[t * nstride + k];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < W::CPT; ++u) {
            const int j = tid + u * W::THREADS;
            const int o = t * HOP - NFFT / 2 + j + lag;  // clean sample scored against y[o - lag]
            pc[u] = (j < HOP && cbase && o >= 0 && o < len) ? cbase[o] : 0.0;
        }
      }
    };
    // rows of frame t live in buffer t&1: Y and gamma = max(|Y|^2 inv, eps)
    // (the noise row itself for SS); at 512 also d = max(gamma - 1, 0) and
    // MMSE's (sqrt(pi)/2)/(gamma + 1e-12), or for SS P = |Y|^2, the unit
    // phasor of Y in place of Y and 1/|Y| (gain output) — computed once here
    // for the workgroup's cells instead of by each of them
    auto store_rows = [&](int t) {  // registers -> LDS rows of frame t
        if (t < nf) {
            float2* yrow = (float2*)(smem + W::OFF_Y + (t & 1) * W::YROW);
            float* grow = (float*)(smem + W::OFF_G + (t & 1) * W::GROW);
            float2* grow2 = (float2*)grow;
            float* arow = (float*)(smem + W::OFF_A + (t & 1) * W::AROW);
#pragma unroll
            for (int u = 0; u < W::YPT; ++u) {
                const int k = tid + u * W::THREADS;
                if (k < B) {
                    const float2 y = py[u];
                    const float P = y.x * y.x + y.y * y.y;
                    // pair order (CSE_PK): bin k goes to half h of mirror pair p,
                    // the 16-B records (Y_p, Y_{M-p}) and (g_p, g_{M-p}, d_p, d_{M-p})
                    const int pp = k <= M / 2 ? k : M - k, hh = k <= M / 2 ? 0 : 1;
                    auto put = [&](float2 yv, float gv, float dv) {
                        if constexpr (W::PK) {
                                yrow[2 * pp + hh] = yv;
                            grow[4 * pp + hh] = gv;
                            grow[4 * pp + 2 + hh] = dv;
                        } else {
                            yrow[k] = yv;
                            grow2[k] = make_float2(gv, dv);
                        }
                    };
                    const int ai = W::PK ? 2 * pp + hh : k;
                    if (!W::R2) {
                        const float gam = fmaxf(P * pn[u], EPS);
                        const float gv = (ALGO == CSE_ALGO_SS) ? pn[u] : (ALGO == CSE_ALGO_OMLSA ? gam * kLog2e : gam);
                        yrow[k] = y;
                        grow[k] = gv;
                    } else if (ALGO == CSE_ALGO_SS) {
                        // phasor y/|y| of the y rescaled by 2^64 below 2^-50
                        // (v_rsq flushes denormals); (1, 0) where y = 0
                        const float sc = fmaxf(fabsf(y.x), fabsf(y.y)) < 0x1p-50f ? 0x1p64f : 1.0f;
                        const float yx = y.x * sc, yy = y.y * sc;
                        const float pz = fmaf(yx, yx, yy * yy);
                        const float r = __builtin_amdgcn_rsqf(pz);
                        // (1, 0) where y = 0 (angle(0) = 0); NaN where y is not
                        // finite (np.angle(NaN) / of an inf is NaN or a value the
                        // NaN |Y|^2 poisons anyway: S = sqrt(Ps) e^{i angle} is NaN)
                        put(pz > 0.0f ? make_float2(yx * r, yy * r)
                                      : (pz == 0.0f ? make_float2(1.0f, 0.0f)
                                                    : make_float2(pz - pz, pz - pz)),
                            pn[u], P);
                        if (OUT) arow[ai] = pz > 0.0f ? r * sc : 0.0f;
                    } else {
                        const float gam = fmaxf(P * pn[u], EPS);
                        // OMLSA's bins take gamma log2(e) (gain_omlsa), d from gamma
                        put(y, ALGO == CSE_ALGO_OMLSA ? gam * kLog2e : gam,
                            fmaxf(gam - 1.0f, 0.0f));
                        if (ALGO == CSE_ALGO_MMSE)
                            arow[ai] = 0.88622692545275801f * fast_rcp(gam + 1e-12f);
                    }
                }
            }
        }
        float* crow = (float*)(smem + W::OFF_C + (t & 1) * W::HMAX * 4);
#pragma unroll
        for (int u = 0; u < W::CPT; ++u) {
            const int j = tid + u * W::THREADS;
            if (j < HOP) crow[j] = pc[u];
        }
    };
    if (!nstride) {
#pragma unroll
        for (int u = 0; u < W::YPT; ++u) {
            const int k = tid + u * W::THREADS;
            if (k < B) pn[u] = Nbase[k];
        }
    }
    load_rows(0);
    store_rows(0);
    load_rows(1);

    // M2C: bin M/2 of frame tt for the workgroup's cells (lane c < CPWG: cell
    // c) from that bin's Y and noise-row value, with the stager's and
    // gain_pack_pk's arithmetic; writes Z'[M/2] and the state to the cell's
    // table-row tail (read by the cell's lane 0 / the next frame's wave)
    float2 m2y = make_float2(0.0f, 0.0f);
    float m2n = 0.0f;
    // (the same ranges as the row loads' resources, which are empty at 1024)
    const __amdgpu_buffer_rsrc_t m2yrc = ROWS_BUF ? yrc : __builtin_amdgcn_make_buffer_rsrc(
        (void*)Ybase, (short)0, W::M2C ? nf * B * 8 : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t m2nrc = ROWS_BUF ? nrc : __builtin_amdgcn_make_buffer_rsrc(
        (void*)Nbase, (short)0, W::M2C ? ((nstride ? (nf - 1) * nstride : 0) + B) * 4 : 0, 0x00020000);
    auto m2_load = [&](int tt) {  // bin M/2 of frame tt (0 past the rows' end)
        m2y = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
            m2yrc, opaque_off(8 * (tt * B + M / 2)), 0, 0));
        m2n = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
            m2nrc, opaque_off(4 * (tt * nstride + M / 2)), 0, 0));
    };
    auto m2_eval = [&](int tt) {
        const int c = lane < W::CPWG ? lane : 0;
        const float2 y = m2y;
        const float P = y.x * y.x + y.y * y.y;
        float2 yv = y;
        RowV rv{0.0f, 0.0f, 0.0f};
        if (!W::R2) {  // store_rows at 1024: Y itself and gamma (N for SS)
            const float gam = fmaxf(P * m2n, EPS);
            rv.g = (ALGO == CSE_ALGO_SS) ? m2n : (ALGO == CSE_ALGO_OMLSA ? gam * kLog2e : gam);
        } else if (ALGO == CSE_ALGO_SS) {  // store_rows: the phasor, (N, P)
            const float sc = fmaxf(fabsf(y.x), fabsf(y.y)) < 0x1p-50f ? 0x1p64f : 1.0f;
            const float yx = y.x * sc, yy = y.y * sc;
            const float pz = fmaf(yx, yx, yy * yy);
            const float r = __builtin_amdgcn_rsqf(pz);
            yv = pz > 0.0f ? make_float2(yx * r, yy * r)
                           : (pz == 0.0f ? make_float2(1.0f, 0.0f) : make_float2(pz - pz, pz - pz));
            rv.g = m2n;
            rv.d = P;
        } else {
            const float gam = fmaxf(P * m2n, EPS);
            rv.g = ALGO == CSE_ALGO_OMLSA ? gam * kLog2e : gam;
            rv.d = fmaxf(gam - 1.0f, 0.0f);
            if (ALGO == CSE_ALGO_MMSE) rv.a = 0.88622692545275801f * fast_rcp(gam + 1e-12f);
        }
        const CellParam cp = *(const CellParam*)(smem + W::OFF_CP + 32 * c);
        float rr = tt == 0 ? 0.0f : *(const float*)(smem + W::m2r(c));
        float gm;
        const float sm = 2.0f * gain_bin<NFFT, ALGO>(yv, rv, rr, tt == 0 ? 0.0f : cp.p0, cp, gm);
        if (lane < W::CPWG) {
            *(f2*)(smem + W::m2z(c, tt & 1)) = f2{yv.x * sm, -yv.y * sm};
            *(float*)(smem + W::m2r(c)) = rr;
        }
    };
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    if constexpr (W::M2C) {
        if (wave_u == 0) {  // frame 0 (visible at the loop's first barrier)
            m2_load(0);
            m2_eval(0);
        }
        m2_load(wave_u + 1);  // wave w's first turn is frame w: it evaluates frame w + 1
    }

    const int b2 = (L == 16) ? i : (i & 15);
    const int h2 = (L == 16) ? 0 : (i >> 4);
    // lane's first sample offset inside a frame
    const int off = 2 * b2 + 32 * h2;

    float rr[17];  // prev_gain**2 * prev_gamma per bin (read from frame 1 on)
#pragma unroll
    for (int j = 0; j < 17; ++j) rr[j] = 0.0f;
    f2 rr2[8];       // CSE_PK: the same state per mirror pair (k, M - k) ...
    float rrm = 0.0f;  // ... and of bin M/2
#pragma unroll
    for (int j = 0; j < 8; ++j) rr2[j] = f2{0.0f, 0.0f};
    float acc[PEND];  // overlap-add sums of the positions frame t's slots q < PEND cover
#pragma unroll
    for (int q = 0; q < PEND; ++q) acc[q] = 0.0f;
    f2 acc2[PEND / 2];  // CSE_PK: the same sums in slot pairs (q, q + 1)
#pragma unroll
    for (int q = 0; q < PEND / 2; ++q) acc2[q] = f2{0.0f, 0.0f};
    double sse = 0.0;
    float chk = 0.0f;  // sum of y*0 over retired samples: NaN iff some y is not finite

#ifdef CSE_ENH_STAMPS
    EnhStamps est;
    est.start();
#endif
    for (int t = 0; t < nf + R - 1; ++t) {
        float x[32];  // this frame's windowed IFFT samples (0 in flush frames)
        f2 xp[16];    // CSE_PK: the same as pairs (x[2p], x[2p + 1])
        // the lane's window slots: ds_read_b128 from its 16-B aligned table row
        // (issued before the pass-2 DFT instead: +0.7 % at 512, the 32 VGPRs
        // held through it cost more than the latency they hide)
        float wv[W::WSLOTS];
        auto load_win = [&]() {
            const float4* w4 = (const float4*)(smem + W::OFF_WIN + 4 * W::WSTR * i);
#pragma unroll
            for (int k = 0; k < W::WSLOTS / 4; ++k) {
                const float4 q4 = w4[k];
                wv[4 * k] = q4.x;
                wv[4 * k + 1] = q4.y;
                wv[4 * k + 2] = q4.z;
                wv[4 * k + 3] = q4.w;
            }
        };

        if (W::PK && t < nf) {
            // the frame in packed pairs (CSE_PK; same stages as the branch below)
            __syncthreads();
            CSE_MARK("gain");
            __builtin_amdgcn_s_setprio(1);
            f2 z[16];
            {
                const CellParam cpar = *(const CellParam*)(smem + W::OFF_CP + 32 * cslot);
                const float alpha_t = (t == 0) ? 0.0f : cpar.p0;
                const int yb = W::OFF_Y + (t & 1) * W::YROW, gb = W::OFF_G + (t & 1) * W::GROW;
                const int ab = W::OFF_A + (t & 1) * W::AROW;
                gain_pack_pk<NFFT, ALGO, OUT, W::M2C>((const float4*)(smem + yb), (const void*)(smem + gb),
                                              (const float2*)(smem + ab), z, (f2*)(smem + creg + 72 * i),
                                              rr2, rrm, alpha_t, cpar,
                                              (const float4*)(smem + W::OFF_LC + W::ROTSTR * i),
                                              (OUT && gout) ? gout + t * B : nullptr, i);
            }
            __builtin_amdgcn_s_setprio(0);
            CSE_MARK("xchg");
            wave_sync();
            {
                const int partner = (L - i) & (L - 1);
                const int xo = creg + 72 * partner + (i == 0 ? 8 : 0);
                // entries 7, 5, 3, 1 and 6, 4, 2, 0 from two unrelated bases:
                // 8 ds_read_b64 (2 LDS cycles each), not 4 ds_read2_b64 (8)
                const f2* xe = (const f2*)(smem + opaque_off(xo));
                const f2* xd = (const f2*)(smem + opaque_off(xo + 8));
#pragma unroll
                for (int s = 8; s < 16; ++s) z[s] = ((15 - s) & 1) ? xd[14 - s] : xe[15 - s];
                if constexpr (W::M2C) {  // lane 0: Z'[M/2] from the frame's evaluating wave
                    const f2 zm = *(const f2*)(smem + W::m2z(cslot, t & 1));
                    if (i == 0) z[8] = zm;
                }
            }
            CSE_MARK("rows");
            store_rows(t + 1);
            if constexpr (W::M2C) {
                // this frame's wave evaluates bin M/2 of frame t + 1 for every
                // cell (before load_rows: its operands' wait covers no new load)
                // and fetches the operands of its next turn, frame t + 5
                if (wave_u == (t & 3)) {
                    if (t + 1 < nf) m2_eval(t + 1);
                    m2_load(t + 5);
                }
            }
            load_rows(t + 2);
            CSE_MARK("pass1");
            {  // pass-1 twiddles from the lane's table row (8 ds_read_b128), issued ahead of the DFT
                const float4* twr = (const float4*)(smem + W::OFF_TW + 144 * i);
                float4 t4[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) t4[k] = twr[k];
                idft16_pk(z);
#pragma unroll
                for (int b = 1; b < 16; ++b) {
                    const float4 q4 = t4[(b - 1) >> 1];
                    z[b] = p_cmul(z[b], ((b - 1) & 1) ? f2{q4.z, q4.w} : f2{q4.x, q4.y});
                }
            }
            CSE_MARK("pass2");
            f2 v[16];
            {
                // lane i writes row i of the block (z[b] at column b), lane b2
                // reads column b2: 16 ds_read_b64 at the row stride (the
                // row-wise read merged into 8 ds_read2_b64, 8 LDS cycles per
                // pair against 2 + 2); the even and odd columns' writes from
                // unrelated bases stay ds_write_b64
                constexpr int TS = W::TS;
                wave_sync();
                f2* we = (f2*)(smem + opaque_off(creg + 8 * TS * i));
                f2* wd = (f2*)(smem + opaque_off(creg + 8 * TS * i + 8));
#pragma unroll
                for (int b = 0; b < 16; b += 2) {
                    we[b] = z[b];
                    wd[b] = z[b + 1];
                }
                wave_sync();
                const f2* tc = (const f2*)(smem + creg + 8 * b2);
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = tc[r * TS];
            }
            idft16_pk(v);
            CSE_MARK("window");
#pragma unroll
            for (int p = 0; p < 16; ++p) xp[p] = v[p];
        } else if (t < nf) {
            // the one workgroup barrier per frame: rows(t) (stored during frame
            // t-1) are visible, and nobody still reads buffer (t+1)&1
            __syncthreads();
            CSE_MARK("gain");
            // the VALU-dense gain stage issues ahead of other waves' LDS-bound
            // IFFT stages, whose latency then overlaps it (r01: 33.3 -> 31.5 ms)
            __builtin_amdgcn_s_setprio(1);
            cf z[16];
            {
                const CellParam cpar = *(const CellParam*)(smem + W::OFF_CP + 32 * cslot);
                const float alpha_t = (t == 0) ? 0.0f : cpar.p0;  // see gain_wiener
                const int yb = W::OFF_Y + (t & 1) * W::YROW, gb = W::OFF_G + (t & 1) * W::GROW;
                const int ab = W::OFF_A + (t & 1) * W::AROW;
                // mirror halves: lane i's slot e (9 entries, 72 B) receives
                // Z'[M - i - L e] (e < 8) and Z'[M/2] (e = 8); lane q takes
                // z[s] (s >= 8) = Z'[q + L s] from lane (L - q) mod L, entry 15 - s
                // (lane 0: its own entry 16 - s, entry 8 = Z'[M/2] for s = 8)
                gain_pack<NFFT, ALGO, OUT, W::M2C>(
                    (const float2*)(smem + yb), (const void*)(smem + gb),
                    (const float*)(smem + ab), z, (cf*)(smem + creg + 72 * i), rr, alpha_t, cpar,
                    (const float4*)(smem + W::OFF_LC + W::ROTSTR * i),
                    (const cf*)(smem + W::OFF_LC + 8 * i),
                    (OUT && gout) ? gout + t * B : nullptr, i);
            }
            __builtin_amdgcn_s_setprio(0);
            CSE_MARK("xchg");
            wave_sync();  // my wave's mirror entries written
            {
                const int partner = (L - i) & (L - 1);
                const cf* xr = (const cf*)(smem + creg + 72 * partner + (i == 0 ? 8 : 0));
#pragma unroll
                for (int s = 8; s < 16; ++s) z[s] = xr[15 - s];
                if constexpr (W::M2C) {  // lane 0: Z'[M/2] from the frame's evaluating wave
                    const f2 zm = *(const f2*)(smem + W::m2z(cslot, t & 1));
                    if (i == 0) z[8] = cmk(zm.x, zm.y);
                }
            }
            CSE_MARK("rows");
            store_rows(t + 1);  // other buffer: its last readers passed this frame's barrier
            if constexpr (W::M2C) {  // see the packed branch
                if (wave_u == (t & 3)) {
                    if (t + 1 < nf) m2_eval(t + 1);
                    m2_load(t + 5);
                }
            }
            load_rows(t + 2);

            CSE_MARK("pass1");
            {
                if constexpr (W::ROTOR_TW) {
                    // twiddles e^{2πi i b/M} = r^(b mod 4) r^(4 (b div 4)) from the
                    // lane's table of r, r^2, r^3, r^4, r^8, r^12 (three ds_read_b128;
                    // one rounding per table entry, one product at most)
                    const float4* q4 = (const float4*)(smem + W::OFF_TW + 48 * i);
                    const float4 qa = q4[0], qb = q4[1], qc = q4[2];
                    idft16(z);
                    const cf lo[4] = {cmk(1.0f, 0.0f), cmk(qa.x, qa.y), cmk(qa.z, qa.w), cmk(qb.x, qb.y)};
                    const cf hi[4] = {cmk(1.0f, 0.0f), cmk(qb.z, qb.w), cmk(qc.x, qc.y), cmk(qc.z, qc.w)};
#pragma unroll
                    for (int b = 1; b < 16; ++b) {
                        const cf t = (b & 3) == 0 ? hi[b >> 2] : (b < 4 ? lo[b] : cmul(lo[b & 3], hi[b >> 2]));
                        z[b] = cmul(z[b], t);
                    }
                } else {
                // pass-1 twiddles e^{2πi i' b/M}, b = 1..15, of my column (per-lane
                // row of 18 complex: 8 ds_read_b128), issued ahead of the DFT
                const float4* twr = (const float4*)(smem + W::OFF_TW + 144 * i);
                float4 t4[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) t4[k] = twr[k];
                idft16(z);
#pragma unroll
                for (int b = 1; b < 16; ++b) {
                    const float4 q4 = t4[(b - 1) >> 1];
                    const cf t = ((b - 1) & 1) ? cmk(q4.z, q4.w) : cmk(q4.x, q4.y);
                    z[b] = cmul(z[b], t);
                }
                }
            }
            CSE_MARK("pass2");
            // ---------------- pass 2: transpose, DFT over lanes
            // Lane (b2, h2) needs row b2 of V[b][i]: the DFT16 (512) / DFT32
            // (1024) input over the pass-1 lane index.  Block: 16 rows x TS
            // complex, entry (b, i); row stride TS = L + 1: the transposed reads
            // of a 16-lane group hit distinct bank pairs.
            cf v[16];
            {
                constexpr int TS = W::TS;
                wave_sync();  // my wave's mirror reads are issued before the transpose overwrites
                cf* tw_ = (cf*)(smem + creg + 8 * i);              // + 8 TS b
                const cf* tr = (const cf*)(smem + creg + 8 * TS * b2);  // + 8 r
#pragma unroll
                for (int b = 0; b < 16; ++b) tw_[b * TS] = z[b];
                wave_sync();
                if constexpr (L == 32) {
                    // DFT32 over i = i' + 16 h: radix-2 decimation in frequency on
                    // the read side, lane (b2, h2) takes lo = V[b2][i'], hi =
                    // V[b2][i' + 16]: U_h2[i'] = (lo + (-1)^h2 hi) W32^{i' h2},
                    // then a DFT16 over i'
                    // branch-free on the lane's half: u = lo -/+ hi by a signed
                    // FMA (exact), rotor (1, 0) on h2 = 0 lanes (an exact
                    // product), so no per-element selects of whole complexes
                    const float sg = h2 ? -1.0f : 1.0f;
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const cf lo = tr[r], hi = tr[r + 16];
                        const cf u = cmk(fmaf(sg, hi.x, lo.x), fmaf(sg, hi.y, lo.y));
                        v[r] = h2 ? cmul(u, cmk(Rot32::c[r], Rot32::s[r])) : u;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) v[r] = tr[r];
                }
            }
            idft16(v);
            CSE_MARK("window");
            // the synthesis window (/n_fft) is applied by the overlap-add FMAs below
#pragma unroll
            for (int q = 0; q < 32; ++q) x[q] = (q & 1) ? v[q >> 1].y : v[q >> 1].x;
        } else {
            __syncthreads();  // flush frames: clean row t visible, row t-1 reads done
            store_rows(t + 1);
            load_rows(t + 2);
#pragma unroll
            for (int q = 0; q < 32; ++q) x[q] = 0.0f;
#pragma unroll
            for (int p = 0; p < 16; ++p) xp[p] = f2{0.0f, 0.0f};
        }

        CSE_MARK("retire");
        // ---------------- overlap-add + retire HOP finished samples ---------
        // slot q < F of this frame completes output position t*HOP + n(q):
        // y = (ola) / wss (librosa istft normalisation), then the SNR error
        // sum of the clipped sample (evaluation_metrics.py:52-56).  Steady
        // frames divide by S(n) through the window table; the first R-1 and
        // the flush frames by the covering frames' window-square sum.
        // windowed overlap-add: x * w(n)/(n_fft S(n)) folded into the
        // accumulating FMAs (x = 0 in flush frames: the sums stay unchanged)
        // w(n)/(NFFT S(n)) at slot q (compile-time after unrolling); at 1024 S is
        // constant and slot q + 16 is w(n + N/2)/(N S) = 1/(N S) - w(n)/(N S)
        load_win();
        constexpr float KHALF = (float)(1.0 / (NFFT * (0.375 * R)));  // S = 3R/8 (R >= 4)
        auto win = [&](int q) {
            return (W::HALF_TABLES && q >= 16) ? KHALF - wv[q - 16] : wv[q];
        };
        float done[F];
        f2 done2[F / 2];
        if constexpr (W::PK) {  // slot pairs (q, q + 1) = (Re, Im) of one IFFT output
            // (applying the window one ds_read_b128 at a time, fenced, to keep
            // 4 of its 32 values live instead of 32: 13-pair A/B 26.3 against
            // 22.8 ms, r05; the compiler's own schedule stays)
#pragma unroll
            for (int p = 0; p < F / 2; ++p) {
                done2[p] = pfma(xp[p], f2{win(2 * p), win(2 * p + 1)}, acc2[p]);
                done[2 * p] = done2[p].x;
                done[2 * p + 1] = done2[p].y;
            }
#pragma unroll
            for (int p = 0; p < PEND / 2; ++p) {
                const int q = 2 * p + F;
                acc2[p] = pfma(xp[q / 2], f2{win(q), win(q + 1)},
                               q < PEND ? acc2[p + F / 2] : f2{0.0f, 0.0f});
            }
        } else {
#pragma unroll
            for (int q = 0; q < F; ++q) done[q] = fmaf(x[q], win(q), acc[q]);
#pragma unroll
            for (int q = 0; q < PEND; ++q) acc[q] = fmaf(x[q + F], win(q + F), q + F < PEND ? acc[q + F] : 0.0f);
        }
        if (valid) {
            const int o0 = t * HOP + off - NFFT / 2;  // output index of q = 0
            const float* crow_t = (const float*)__builtin_assume_aligned(
                smem + W::OFF_C + (t & 1) * W::HMAX * 4 + 4 * off, 8);
            // frame t retires output positions [t*HOP - NFFT/2, (t+1)*HOP - NFFT/2)
            // interior: every slot o and its scored clean index o + lag lie in [0, len)
            const bool edge = (t < R - 1) || (t >= nf);
            const int lo = t * HOP - NFFT / 2;
            const bool interior = !edge && lo + (lag < 0 ? lag : 0) >= 0 &&
                                  lo + HOP + (lag > 0 ? lag : 0) <= len;  // uniform
            const bool head = want_y && lo < out_len;                      // uniform
            float part = 0.0f;
            if (interior) {
                // steady state: every slot is inside [0, len) and the window
                // already carries 1/wss; the finiteness check rides along as
                // chk += y*0 (NaN for a NaN or inf y).  Two accumulator chains
                // each (even / odd slots): the frame's last dependent chain
                // (one chain each: 24.51 -> two: 24.15 ms at 13 pairs)
                float2 cl2[F / 2];  // the clean samples of slots q, q + 1
#pragma unroll
                for (int k = 0; k < F / 2; ++k)
                    cl2[k] = *(const float2*)(crow_t + slot_pos<SP>(2 * k));
                float pa = 0.0f, pb = 0.0f, ca = 0.0f, cb = 0.0f;
                if constexpr (W::PK) {  // the two chains as one pair
                    f2 pp = f2{0.0f, 0.0f}, cc = f2{0.0f, 0.0f};
#pragma unroll
                    for (int p = 0; p < F / 2; ++p) {
                        const f2 y = done2[p];
                        const int n = slot_pos<SP>(2 * p);
                        if (head && yout && o0 + n < out_len) yout[o0 + n] = y.x;
                        if (head && yout && o0 + n + 1 < out_len) yout[o0 + n + 1] = y.y;
                        const f2 d = f2{cl2[p].x, cl2[p].y} - pmed3(y, -1.0f, 1.0f);
                        cc = pfma(y, pdup(0.0f), cc);
                        pp = pfma(d, d, pp);
                    }
                    pa = pp.x;
                    pb = pp.y;
                    ca = cc.x;
                    cb = cc.y;
                }
#pragma unroll
                for (int q = 0; q < (W::PK ? 0 : F); ++q) {
                    const int n = slot_pos<SP>(q);
                    const float y = done[q];
                    if (head && yout && o0 + n < out_len) yout[o0 + n] = y;
                    // np.clip as one v_med3 (fminf(fmaxf()) of a value carried
                    // across the loop got a canonicalising v_max in front)
                    const float d = ((q & 1) ? cl2[q >> 1].y : cl2[q >> 1].x) -
                                    __builtin_amdgcn_fmed3f(y, -1.0f, 1.0f);
                    if (q & 1) {
                        cb = fmaf(y, 0.0f, cb);
                        pb = fmaf(d, d, pb);
                    } else {
                        ca = fmaf(y, 0.0f, ca);
                        pa = fmaf(d, d, pa);
                    }
                }
                part = pa + pb;
                chk += ca + cb;
            } else {
#pragma unroll
                for (int q = 0; q < F; ++q) {
                    const int n = slot_pos<SP>(q);  // + off: position inside frame t
                    const int o = o0 + n;
                    float iv = 1.0f;
                    if (edge) {
                        // fewer than R frames cover this sample: librosa divides by
                        // the covering frames' window-square sum, not S(n).  With
                        // T_r = w_r/(N S) the table entries of the R frames,
                        // S / sum_cov w_r^2 = sum_all T_r^2 / sum_cov T_r^2.
                        float all = 0.0f, cov = 0.0f;
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const float w = win(q + 2 * r * (HOP / SP));
                            all = fmaf(w, w, all);
                            const int tr = t - r;
                            if (tr >= 0 && tr < nf) cov = fmaf(w, w, cov);
                        }
                        iv = cov > 0.0f ? all * __builtin_amdgcn_rcpf(cov) : 1.0f;
                    }
                    if (o >= 0 && o < len) {
                        const float y = done[q] * iv;
                        if (head && yout && o < out_len) yout[o] = y;
                        if (o + lag >= 0 && o + lag < len) {  // dropped by the alignment otherwise
                            chk = fmaf(y, 0.0f, chk);
                            const float d = crow_t[n] - __builtin_amdgcn_fmed3f(y, -1.0f, 1.0f);
                            part = fmaf(d, d, part);
                        }
                    }
                }
            }
            sse += (double)part;
        }
        CSE_MARK("end");
    }

    // ---------------- per-cell reductions over the cell's L lanes ----------
#pragma unroll
    for (int m = L / 2; m > 0; m >>= 1) sse += __shfl_xor(sse, m, 64);
    const unsigned long long bad = __ballot(chk != 0.0f);  // NaN != 0
    const unsigned long long my = (bad >> (cs * L)) & ((1ull << L) - 1);
    const int64_t cell_idx = (int64_t)(wcell - a.cells) + cslot;
#ifdef CSE_ENH_STAMPS
    if (tid == 0 && g_enh_stamps) {
        unsigned long long* o = g_enh_stamps + (int64_t)blockIdx.x * 10;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = est.acc[k];
        o[8] = ALGO;
        o[9] = HOP;
    }
#endif
    if (i == 0 && valid) {
        if (a.sse) a.sse[cell_idx] = sse;
        if (a.finite) a.finite[cell_idx] = my == 0 ? 1 : 0;
    }
}

template <int NFFT, int HOP, bool OUT>
__device__ __forceinline__ void dispatch_algo(const Args& a, const cse_cell_t* wcell, int n,
                                              int algo, unsigned char* smem) {
    switch (algo) {
        case CSE_ALGO_SS: run_wg<NFFT, HOP, CSE_ALGO_SS, OUT>(a, wcell, n, smem); break;
        case CSE_ALGO_WIENER: run_wg<NFFT, HOP, CSE_ALGO_WIENER, OUT>(a, wcell, n, smem); break;
        case CSE_ALGO_MMSE: run_wg<NFFT, HOP, CSE_ALGO_MMSE, OUT>(a, wcell, n, smem); break;
        case CSE_ALGO_OMLSA: run_wg<NFFT, HOP, CSE_ALGO_OMLSA, OUT>(a, wcell, n, smem); break;
        default: break;
    }
}

// One workgroup's slot group at hop H0 or H1: the short-hop kernels' entry
// (enhance_kernel below spells the same steps out for 128 / 256; routed
// through this function its code came out different, r06).
template <int NFFT, bool OUT, int H0, int H1>
__device__ __forceinline__ void enhance_group(const Args& a) {
    using W = WG<NFFT, OUT>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t first = (int64_t)wg * W::CPWG;
    const int64_t left = a.n_cells - first;
    const int n = (int)(left < W::CPWG ? left : W::CPWG);
    const cse_cell_t* wcell = a.cells + first;
    // hop and algorithm of the workgroup = its first cell's (the host packs
    // so); run_wg rejects slots that do not match them.  A group whose slot 0
    // names no algorithm or a hop outside this kernel's set rejects every
    // non-padding slot.
    const int hop = __builtin_amdgcn_readfirstlane(wcell[0].hop);
    const int algo = __builtin_amdgcn_readfirstlane(wcell[0].algo);
    if ((hop != H0 && hop != H1) || algo < CSE_ALGO_SS || algo > CSE_ALGO_OMLSA) {
        for (int c = threadIdx.x; c < n; c += W::THREADS)
            if (wcell[c].algo != CSE_ALGO_NONE) reject_cell(a, first + c);
        return;
    }
    if (H0 == H1 || hop == H0)
        dispatch_algo<NFFT, H0, OUT>(a, wcell, n, algo, smem);
    else
        dispatch_algo<NFFT, H1, OUT>(a, wcell, n, algo, smem);
}

// OUT: the g_out (gain matrix) variant for parity tests; waveform output
// (y_out, any out_len) is available in both variants at run time.
template <int NFFT, bool OUT>
// launch bounds: HIP's second argument is the minimum number of waves per SIMD
// (amdgpu_waves_per_eu), whatever the workgroup size: the register budget is
// 512 / CSE_WAVES_PER_SIMD VGPRs per lane
__global__ void __launch_bounds__(WG<NFFT>::THREADS, CSE_WAVES_PER_SIMD)
    enhance_kernel(Args a) {
    using W = WG<NFFT, OUT>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t first = (int64_t)wg * W::CPWG;
    const int64_t left = a.n_cells - first;
    const int n = (int)(left < W::CPWG ? left : W::CPWG);
    const cse_cell_t* wcell = a.cells + first;
    // hop and algorithm of the workgroup = its first cell's (the host packs
    // so); run_wg rejects slots that do not match them.  A group whose slot 0
    // names no algorithm or an unsupported hop rejects every non-padding slot.
    const int hop = __builtin_amdgcn_readfirstlane(wcell[0].hop);
    const int algo = __builtin_amdgcn_readfirstlane(wcell[0].algo);
    if ((hop != 128 && hop != 256) || algo < CSE_ALGO_SS || algo > CSE_ALGO_OMLSA) {
        for (int c = threadIdx.x; c < n; c += W::THREADS)
            if (wcell[c].algo != CSE_ALGO_NONE) reject_cell(a, first + c);
        return;
    }
    if (hop == 128)
        dispatch_algo<NFFT, 128, OUT>(a, wcell, n, algo, smem);
    else
        dispatch_algo<NFFT, 256, OUT>(a, wcell, n, algo, smem);
}

// The short hops (cse_enhance_cells_short_hop): n_fft 512 at hop 32 / 64, n_fft
// 1024 at hop 64 (a lane retires F = 2 HOP / SP >= 2 samples per frame), no
// gain-matrix variant.  Kernels of their own, so the sweep kernel above keeps
// its registers and code.
template <int NFFT>
__global__ void __launch_bounds__(WG<NFFT>::THREADS, CSE_WAVES_PER_SIMD)
    enhance_kernel_short_hop(Args a) {
    enhance_group<NFFT, false, NFFT == 512 ? 32 : 64, 64>(a);
}

// cse_enhance_generic.hip includes this file for the gain functions above
// (CSE_ENHANCE_DEVICE_ONLY): no kernel instantiations, no entry points.
#ifndef CSE_ENHANCE_DEVICE_ONLY
// The two n_fft halves can be compiled as separate translation units (with
// their own code-generation flags): cse_enhance_512.hip defines
// CSE_ENHANCE_ONLY=512 and holds the 512 kernels, cse_enhance_1024.hip the
// 1024 kernels and the C entry points.  The short-hop kernels are a unit of
// their own (cse_enhance_short.hip defines CSE_ENHANCE_SHORT): instantiated
// beside the sweep kernels they moved the compiler's inlining of the shared
// helpers, and the sweep kernels' code with it.  Compiled on its own
// (analysis tools), this file holds everything.
#if defined(CSE_ENHANCE_SHORT) || !defined(CSE_ENHANCE_ONLY)
const void* enhance_fn_512_short_hop() { return (const void*)enhance_kernel_short_hop<512>; }
const void* enhance_fn_1024_short_hop() { return (const void*)enhance_kernel_short_hop<1024>; }
#else
const void* enhance_fn_512_short_hop();   // cse_enhance_short.hip
const void* enhance_fn_1024_short_hop();
#endif
#ifndef CSE_ENHANCE_SHORT
#if !defined(CSE_ENHANCE_ONLY) || CSE_ENHANCE_ONLY == 512
const void* enhance_fn_512(bool out) {
    return out ? (const void*)enhance_kernel<512, true> : (const void*)enhance_kernel<512, false>;
}
#endif
#if !defined(CSE_ENHANCE_ONLY) || CSE_ENHANCE_ONLY == 1024
const void* enhance_fn_1024(bool out) {
    return out ? (const void*)enhance_kernel<1024, true> : (const void*)enhance_kernel<1024, false>;
}
#endif
#if defined(CSE_ENHANCE_ONLY) && CSE_ENHANCE_ONLY == 1024
const void* enhance_fn_512(bool out);  // cse_enhance_512.hip
#endif
#endif  // !CSE_ENHANCE_SHORT
#endif  // !CSE_ENHANCE_DEVICE_ONLY

}  // namespace cse

#ifndef CSE_ENHANCE_DEVICE_ONLY

#if defined(CSE_ENH_STAMPS) && !defined(CSE_ENHANCE_SHORT)
// analysis builds only: per-workgroup stage cycles into buf [n_groups][10]
// (u64: 8 stages, algorithm, hop) of this translation unit's n_fft, or off (NULL)
#if !defined(CSE_ENHANCE_ONLY) || CSE_ENHANCE_ONLY == 512
extern "C" int cse_enhance_stamp_buffer_512(void* buf) {
#else
extern "C" int cse_enhance_stamp_buffer_1024(void* buf) {
#endif
    unsigned long long* p = (unsigned long long*)buf;
    return hipMemcpyToSymbol(HIP_SYMBOL(cse::g_enh_stamps), &p, sizeof(p)) == hipSuccess ? CSE_OK
                                                                                          : CSE_ELAUNCH;
}
#endif

#if !defined(CSE_ENHANCE_SHORT) && (!defined(CSE_ENHANCE_ONLY) || CSE_ENHANCE_ONLY == 1024)
using namespace cse;

extern "C" int cse_cells_per_group(int n_fft) {
    return (n_fft == 512 || n_fft == 1024) ? CSE_CELLS_PER_GROUP(n_fft) : 0;
}

// cse_enhance_cells / cse_enhance_cells_short_hop: one launch over the cells
static int enhance_launch(const char* name, bool short_hop, int n_fft, int64_t len,
                          const cse_cell_t* cells, int64_t n_cells, const float* Y,
                          const float* noise, const double* clean, float* y_out, int64_t out_len,
                          float* g_out, double* sse, uint8_t* finite, cse_stream_t stream) {
    CSE_CHECK_ARG(n_fft == 512 || n_fft == 1024, "%s: n_fft=%d (512|1024)", name, n_fft);
    CSE_CHECK_ARG(cells && Y && noise, "%s: NULL cells/Y/noise", name);
    CSE_CHECK_ARG(len >= 1 && len < (1ll << 30) && n_cells >= 0, "%s: len=%lld n_cells=%lld", name,
                  (long long)len, (long long)n_cells);
    // n_fft 512 reads its rows through buffer resources with 32-bit byte
    // offsets (run_wg's ROWS_BUF): the signal's spectrum rows at the smallest hop
    // must stay below 2 GiB
    const int64_t min_hop = short_hop ? 32 : 128;
    CSE_CHECK_ARG(n_fft != 512 || (1 + len / min_hop) * 257 * 8 < (1ll << 31),
                  "%s: len=%lld too long for n_fft=512 (spectrum rows >= 2 GiB)", name,
                  (long long)len);
    CSE_CHECK_ARG(!short_hop || !g_out, "%s: no gain-matrix output at the short hops", name);
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
    const int per = CSE_CELLS_PER_GROUP(n_fft);
    const int64_t groups = (n_cells + per - 1) / per;
    CSE_CHECK_ARG(groups < (1ll << 31), "%s: too many cells", name);
    CSE_CHECK_ARG(!y_out || (out_len >= 0 && out_len <= len), "%s: out_len=%lld not in [0, len]",
                  name, (long long)out_len);
    const bool out = g_out != nullptr;  // the gain-writing variant
    const void* fn;
    int bytes, threads;
    if (n_fft == 512) {
        fn = short_hop ? enhance_fn_512_short_hop() : enhance_fn_512(out);
        bytes = out ? WG<512, true>::BYTES : WG<512, false>::BYTES;
        threads = WG<512>::THREADS;
    } else {
        fn = short_hop ? enhance_fn_1024_short_hop() : enhance_fn_1024(out);
        bytes = out ? WG<1024, true>::BYTES : WG<1024, false>::BYTES;
        threads = WG<1024>::THREADS;
    }
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
        ::cse::set_error("%s: cannot reserve %d bytes of LDS", name, bytes);
        return CSE_ELAUNCH;
    }
    void* args[] = {&a};
    if (hipLaunchKernel(fn, dim3((unsigned)groups), dim3(threads), args, (size_t)bytes,
                        (hipStream_t)stream) != hipSuccess) {
        ::cse::set_error("%s: launch failed", name);
        return CSE_ELAUNCH;
    }
    CSE_CHECK_LAUNCH(name);
    return CSE_OK;
}

extern "C" int cse_enhance_cells(int n_fft, int64_t len, const cse_cell_t* cells, int64_t n_cells,
                                 const float* Y, const float* noise, const double* clean,
                                 float* y_out, int64_t out_len, float* g_out, double* sse,
                                 uint8_t* finite, cse_stream_t stream) {
    return enhance_launch("cse_enhance_cells", false, n_fft, len, cells, n_cells, Y, noise, clean,
                          y_out, out_len, g_out, sse, finite, stream);
}

extern "C" int cse_enhance_cells_short_hop(int n_fft, int64_t len, const cse_cell_t* cells,
                                           int64_t n_cells, const float* Y, const float* noise,
                                           const double* clean, float* y_out, int64_t out_len,
                                           double* sse, uint8_t* finite, cse_stream_t stream) {
    return enhance_launch("cse_enhance_cells_short_hop", true, n_fft, len, cells, n_cells, Y,
                          noise, clean, y_out, out_len, nullptr, sse, finite, stream);
}
#endif  // the C entry points
#endif  // !CSE_ENHANCE_DEVICE_ONLY
