/*
 * cse.h — C ABI of libcse.so, the MI355X (gfx950) engine for the STFT
 * frame-gain path of Katja39/Classical_Speech_Enhancement.
 *
 * The reference has no FFI: its seams are Python plugins:
 *   alg_fn(noisy_audio, sr, **params) -> ndarray   registered at
 *     Code/speech_enhancement_comparison.py:395-401, called via
 *     algorithm_wrapper :282-292 from the grid loop :156-226;
 *   NoiseEstimator.estimate(power, **kw)          Code/noise_estimation.py:6-9,
 *     selected by _create_estimator :215-223.
 * Each entry point below replaces the numeric core behind one of those
 * seams; the Python package mirrors the plugin signatures on top of it
 * (see INTEGRATION.md for the ctypes binding).
 *
 * Conventions
 *   - Every pointer is CALLER-OWNED DEVICE memory (hipMalloc / torch tensor).
 *     The library allocates nothing; every call is enqueued on `stream` and
 *     returns immediately (asynchronous, reentrant per stream).
 *   - Return value: CSE_OK (0) or a negative CSE_E* code; cse_last_error()
 *     returns a thread-local message for the last failure.
 *   - Layouts are frame-major: spectra are [signal][frame][bin] with
 *     bins = n_fft/2 + 1 contiguous; complex values are interleaved
 *     (re, im) float pairs.
 *   - Per-cell numerical failure (non-finite output) is reported through the
 *     `finite` output, never as a status code — it mirrors the reference's
 *     "skip this cell" semantics (speech_enhancement_comparison.py:102-103).
 */
#ifndef CSE_H_
#define CSE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* cse_stream_t; /* == hipStream_t */

enum {
    CSE_OK = 0,
    CSE_EINVAL = -1,  /* bad argument / unsupported shape */
    CSE_ELAUNCH = -2, /* HIP launch failure */
};

/* algorithms (cse_cell_t.algo) */
enum {
    CSE_ALGO_NONE = -1, /* padding slot: computes nothing, writes nothing */
    CSE_ALGO_SS = 0,    /* spectral_subtractor.py:6-65   param: alpha, beta            */
    CSE_ALGO_WIENER = 1,/* wiener_filter.py:7-95         param: alpha, gain_floor      */
    CSE_ALGO_MMSE = 2,  /* mmse.py:6-120                 param: alpha, ksi_min, gain_min, gain_max */
    CSE_ALGO_OMLSA = 3, /* advanced_mmse.py:7-136        param: alpha, ksi_min, gain_floor, q, v_max */
};

/* noise-PSD estimators (noise_estimation.py) */
enum {
    CSE_NOISE_PERCENTILE = 0,   /* :11-56  static [B]            */
    CSE_NOISE_MIN_TRACKING = 1, /* :59-107 time-varying [T][B]   */
    CSE_NOISE_TRUE = 2,         /* :109-155 time-varying [T][B]  */
};

/*
 * One grid cell = one (signal group, noise PSD, algorithm, parameter set).
 * Cells are processed CSE_CELLS_PER_GROUP(n_fft) at a time by one workgroup of
 * CSE_WG_WAVES (n_fft 512) / CSE_WG_WAVES_1024 wavefronts that stages their shared rows in LDS, so the cells
 * of one such slot group (cells[g*G .. g*G+G-1]) MUST share algo, hop,
 * y_offset, noise_offset, noise_stride, clean_offset and lag; pad a short
 * group with CSE_ALGO_NONE slots.  Only param, out_offset and gain_offset may
 * differ.  The kernel checks it: a non-padding slot whose shared fields differ
 * from slot 0's is not computed and gets finite = 0, sse = NaN (the
 * reference's skip, speech_enhancement_comparison.py:102-103; y_out / g_out
 * untouched), and a group whose slot 0 is padding or names an unsupported
 * algorithm or hop rejects every non-padding slot the same way.
 */
typedef struct cse_cell {
    int32_t algo;          /* CSE_ALGO_* */
    int32_t hop;           /* hop length; 128 or 256 (short hops: cse_enhance_cells_short_hop) */
    int64_t y_offset;      /* offset (in complex elements) of this cell's spectrum Y[T][B] */
    int64_t noise_offset;  /* offset (floats) of this cell's noise row: the PSD N itself for
                              CSE_ALGO_SS, 1/max(N, eps) (cse_noise_invert) for the others */
    int64_t noise_stride;  /* floats between frames of the noise PSD: 0 = static [B], B = [T][B] */
    int64_t clean_offset;  /* offset (doubles) of the clean reference for the SNR, or -1 */
    int64_t out_offset;    /* offset (floats) of this cell's output waveform in y_out, or -1 */
    int64_t gain_offset;   /* offset (floats) of this cell's gain matrix G[T][B] in g_out, or -1 */
    int32_t lag;           /* alignment lag l of the SNR sum (finalize_enhanced): output sample
                              y[o] is scored against clean[o + l]; samples with o + l outside
                              [0, len) are dropped (speech_enhancement_comparison.py:61-69).
                              0 = unaligned.  |lag| < len. */
    int32_t reserved;      /* 0 */
    float param[8];        /* algorithm parameters, order as in the CSE_ALGO_* comments */
} cse_cell_t;              /* 96 bytes */

#ifndef CSE_WG_WAVES
#define CSE_WG_WAVES 4 /* wavefronts per n_fft=512 workgroup (cse_cells_per_group reports it) */
#endif
#ifndef CSE_WG_WAVES_1024
#define CSE_WG_WAVES_1024 4 /* wavefronts per n_fft=1024 workgroup */
#endif
#define CSE_CELLS_PER_GROUP(n_fft) ((n_fft) == 512 ? 4 * CSE_WG_WAVES : 2 * CSE_WG_WAVES_1024)

/* Library identity. */
int cse_version(void);
const char* cse_last_error(void);
/* CSE_CELLS_PER_GROUP(n_fft) of this build (0 for an unsupported n_fft). */
int cse_cells_per_group(int n_fft);

/*
 * Centred, reflect-padded, periodic-Hann STFT (librosa 0.11 `stft` as called
 * at spectral_subtractor.py:25, wiener_filter.py:35, mmse.py:29,
 * advanced_mmse.py:39 and noise_estimation.py:184-188, :136-144), computed in
 * fp64.  x: [n_sig][len] f64.  If x_sub != NULL the transform is taken of
 * (x - x_sub) (TrueNoise, noise_estimation.py:133).  T = 1 + len/hop.
 * n_fft even, in [64, 4096] (a power of two: radix 2; otherwise a direct
 * DFT), hop in [1, n_fft].
 * Outputs (either may be NULL): Y [n_sig][T][B] complex64, P [n_sig][T][B] f64 = |Y|^2.
 */
int cse_stft(const double* x, const double* x_sub, int64_t n_sig, int64_t len, int n_fft,
             int hop, float* Y, double* P, cse_stream_t stream);

/* Workspace bytes needed by cse_noise_estimate for one call. */
int64_t cse_noise_workspace_bytes(int64_t n_sig, int T, int B);

/*
 * Noise-PSD estimators on P [n_sig][T][B] f64 (noise_estimation.py):
 *   CSE_NOISE_PERCENTILE   -> N [n_sig][B]   (PercentileNoiseEstimator :20-56,
 *                             or _simple_noise_estimate :226-232 when T < 5)
 *   CSE_NOISE_MIN_TRACKING -> N [n_sig][T][B] (MinTrackingNoiseEstimator :64-95,
 *                             or the static T < 5 fallback, broadcast over T)
 *   CSE_NOISE_TRUE         -> N [n_sig][T][B] = max(P, eps) where P is the
 *                             power of STFT(noisy - clean) (:135-147)
 * percentile is ignored except for CSE_NOISE_PERCENTILE.  N is f32.
 * workspace: >= cse_noise_workspace_bytes(n_sig, T, B) bytes of device memory.
 */
int cse_noise_estimate(int method, const double* P, int64_t n_sig, int T, int B,
                       double percentile, double eps, float* N, void* workspace,
                       cse_stream_t stream);

/*
 * Estimator constructor parameters (noise_estimation.py:12-13, :60) and the
 * TrueNoise frame fit (:149-153), for cse_noise_estimate_ex.
 * cse_noise_default_params() fills the reference's defaults.
 */
typedef struct cse_noise_params {
    double percentile;       /* PercentileNoiseEstimator(percentile=20.0)             */
    double max_fraction;     /*   max_fraction=0.30                                   */
    double floor_rel;        /*   floor_rel=0.02                                      */
    double smoothing_factor; /* MinTrackingNoiseEstimator(smoothing_factor=None): NaN = None */
    int32_t min_frames;      /* PercentileNoiseEstimator min_frames=10                */
    int32_t adaptive_short;  /*   adaptive_short=True                                 */
    int32_t window_size;     /* MinTrackingNoiseEstimator(window_size=50)             */
    int32_t src_frames;      /* CSE_NOISE_TRUE: frames of P (STFT of the trimmed noisy - clean);
                                rows t >= src_frames repeat the last one (np.pad mode='edge'),
                                src_frames > T is trimmed.  0 = T.  Ignored otherwise. */
} cse_noise_params_t;        /* 48 bytes */

void cse_noise_default_params(cse_noise_params_t* prm);

/*
 * cse_noise_estimate with estimator parameters (host struct, read at call
 * time).  P is [n_sig][T][B] (CSE_NOISE_TRUE: [n_sig][src_frames][B]); N and
 * the T < 5 fallback (:194-195) as for cse_noise_estimate.  Parameters a
 * method does not read are ignored, as the reference's **kwargs swallow them.
 */
int cse_noise_estimate_ex(int method, const double* P, int64_t n_sig, int T, int B,
                          const cse_noise_params_t* prm, double eps, float* N, void* workspace,
                          cse_stream_t stream);

/*
 * Time-varying noise PSD for the smoothed / frame-padded cases, fp64 math:
 *   src = N [n_sig][src_frames][B] with src_frames == T, or src_frames == 1: a
 *   static estimate that librosa.util.fix_length(..., size=T, axis=1)
 *   zero-pads to T frames (spectral_subtractor.py:40-41, advanced_mmse.py:54-55);
 *   out_0 = src_0, out_t = mu*out_{t-1} + (1-mu)*src_t  (mmse.py:48-54,
 *   advanced_mmse.py:60-66) with mu = clip(mu, 0, 0.9999); mu = 0 gives the
 *   plain (padded) source.  out: [n_sig][T][B] f32.
 */
int cse_noise_smooth(const float* N, int64_t n_sig, int T, int B, int src_frames, double mu,
                     float* out, cse_stream_t stream);

/*
 * Building blocks of cse_noise_estimate for the grid planner, so work shared
 * by several estimates of one (signals, n_fft, hop) group is done once:
 *   cse_noise_median           med[n_sig][B] = np.median(P, axis=frames)
 *                              (noise_estimation.py:53, :93), f64;
 *   cse_noise_percentile_med   the percentile estimate given that median (T >= 5);
 *   cse_noise_min_tracking_med the min-tracking estimate given that median, floored
 *                              at eps into N and (if N_b != NULL) at eps_b into N_b
 *                              (the two eps the algorithms pass share the IIR + min
 *                              filter, noise_estimation.py:78-94) (T >= 5).
 * The workspace is the cse_noise_workspace_bytes() one.
 */
int cse_noise_median(const double* P, int64_t n_sig, int T, int B, double* med,
                     cse_stream_t stream);
int cse_noise_percentile_med(const double* P, const double* med, int64_t n_sig, int T, int B,
                             double percentile, double eps, float* N, void* workspace,
                             cse_stream_t stream);
/* Two percentile estimates with one eps (pct 10 and 20 of the grids,
 * parameter_ranges.py): the frame energies e_t = mean_b log(max(P, eps))
 * (noise_estimation.py:44) depend on eps only and are computed once; each
 * percentile then selects its quiet frames and takes its statistic as
 * cse_noise_percentile_med does.  N_b may be NULL. */
int cse_noise_percentile_med2(const double* P, const double* med, int64_t n_sig, int T, int B,
                              double percentile_a, double percentile_b, double eps, float* N_a,
                              float* N_b, void* workspace, cse_stream_t stream);
/* Two percentiles x two eps values of one hop's P (the HEAD grid's four
 * PercentileNoiseEstimator calls per hop, noise_estimation.py:16-52 with
 * percentile_a/_b and eps_a/_b) in four launches: the frame energies for both
 * eps from one read of P, one sort of each eps's energies for both
 * percentiles, one order-statistic launch per percentile covering both eps.
 * N_pe (p: percentile a/b, e: eps a/b) equal cse_noise_percentile_med bit for
 * bit; a NULL output is skipped.  Its scratch is a region of the workspace of
 * its own (r06: r05 borrowed the min-tracking IIR region); as for every
 * cse_noise_* call, one workspace serves one stream at a time. */
int cse_noise_percentile_quad(const double* P, const double* med, int64_t n_sig, int T, int B,
                              double percentile_a, double percentile_b, double eps_a,
                              double eps_b, float* N_aa, float* N_ab, float* N_ba, float* N_bb,
                              void* workspace, cse_stream_t stream);
int cse_noise_min_tracking_med(const double* P, const double* med, int64_t n_sig, int T, int B,
                               double eps, float* N, double eps_b, float* N_b, void* workspace,
                               cse_stream_t stream);

/*
 * Batched post-processing of noise rows into the rows the hot kernel reads.
 * Job j, signal s, bin b (fp64 math, f32 in/out):
 *   x_t  = src[src_offset + (s*src_frames + t)*B + b] for t < src_frames, else 0
 *          (src_frames = 1 for a static row that librosa fix_length zero-pads)
 *   y_0  = x_0,  y_t = mu*y_{t-1} + (1-mu)*x_t     (mu = 0: plain copy / pad)
 *   dst[dst_offset + (s*out_frames + t)*B + b] = inv_eps > 0 ? 1/max(y_t, inv_eps) : y_t
 */
typedef struct cse_noise_job {
    int64_t src_offset;
    int64_t dst_offset;
    int32_t src_frames;
    int32_t out_frames;
    double mu;
    double inv_eps;
} cse_noise_job_t; /* 40 bytes */

int cse_noise_finish(const cse_noise_job_t* jobs, int n_jobs, int64_t n_sig, int B,
                     const float* src, float* dst, cse_stream_t stream);

/*
 * out = 1 / max(N, eps) (fp64 math, f32 out), n elements: the noise row the
 * Wiener/MMSE/OMLSA cells of cse_enhance_cells read (their in-loop floors,
 * wiener_filter.py:58, mmse.py:71, advanced_mmse.py:87, folded in).
 */
int cse_noise_invert(const float* N, int64_t n, double eps, float* out, cse_stream_t stream);

/*
 * 1 / window-sum-square of the ISTFT (librosa 0.11 istft normalisation) for a
 * centred signal of `len` samples; entries where the sum is <= DBL_MIN are 1.
 * out: [len] f32.  (A reference table: cse_enhance_cells computes the same
 * normalisation analytically in-kernel.)
 */
int cse_istft_norm(int n_fft, int hop, int64_t len, float* out, cse_stream_t stream);

/*
 * THE HOT PATH.  For every cell: the per-frame gain recursion of its algorithm
 * (decision-directed a-priori SNR, serial over frames), S = Y*G (SS: noisy
 * phase), inverse real FFT, periodic-Hann synthesis window, overlap-add,
 * window-sum-square normalisation (librosa istft, length = len), and the
 * per-cell score reductions, with l = cell.lag:
 *   sse[c]    = sum over o in [0,len) with o+l in [0,len) of
 *               (clean[o + l] - clip(y[o], -1, 1))^2   (f64; clean is f64 [..][len],
 *               used if clean_offset >= 0)
 *   finite[c] = 1 if every scored y[o] is finite
 * (the samples an aligned output gets as zero padding are not included: see
 * cse_xcorr_lag's zero_energy).
 * Optional outputs: y_out (the first out_len samples of the enhanced waveform,
 * f32, at out_offset; out_len = len for the whole waveform) and g_out (the
 * gain matrix, f32 [T][B] at gain_offset).
 * n_fft in {512, 1024}; hop in {128, 256}; len < 2^30, and at n_fft 512
 * (1 + len/128) * 257 * 8 < 2^31 (len < 133.6 M samples, 2.3 h at 16 kHz:
 * its rows are read with 32-bit byte offsets).  noise_stride is 0 or B.
 */
int cse_enhance_cells(int n_fft, int64_t len, const cse_cell_t* cells, int64_t n_cells,
                      const float* Y, const float* noise, const double* clean,
                      float* y_out, int64_t out_len, float* g_out, double* sse,
                      uint8_t* finite, cse_stream_t stream);

/*
 * cse_enhance_cells at the short hops the plugins accept beside the grid's
 * 128/256 (spectral_subtractor.py:6, wiener_filter.py:7, mmse.py:6,
 * advanced_mmse.py:7 take any hop_length): n_fft 512 at hop 32 or 64, n_fft
 * 1024 at hop 64 — kernels of their own, so every slot group of `cells` must
 * name one of those hops (a group at another hop is rejected as above; the
 * 128/256 groups go to cse_enhance_cells).  Same cells, rows, outputs and
 * limits (n_fft 512: (1 + len/32) * 257 * 8 < 2^31), no gain-matrix output.
 */
int cse_enhance_cells_short_hop(int n_fft, int64_t len, const cse_cell_t* cells, int64_t n_cells,
                                const float* Y, const float* noise, const double* clean,
                                float* y_out, int64_t out_len, double* sse, uint8_t* finite,
                                cse_stream_t stream);

/*
 * cse_enhance_cells at any other STFT shape (r06): n_fft even, in
 * [64, 4096], cell.hop in [1, n_fft] (e.g. 512 / 160, 1024 / 512, 256 / 64,
 * 2048 / 512, 400 / 160) — the plugins' shapes beyond the grid's.  One workgroup per
 * cell, no slot groups (cells are independent; CSE_ALGO_NONE cells are
 * skipped), a cell whose hop lies outside [1, n_fft] gets the reference's skip
 * (finite = 0, sse = NaN).  Same rows, outputs (incl. g_out) and sums as
 * cse_enhance_cells; len < 2^30.
 */
int cse_enhance_cells_generic(int n_fft, int64_t len, const cse_cell_t* cells, int64_t n_cells,
                              const float* Y, const float* noise, const double* clean,
                              float* y_out, int64_t out_len, float* g_out, double* sse,
                              uint8_t* finite, cse_stream_t stream);

/*
 * Alignment of finalize_enhanced (speech_enhancement_comparison.py:38-69, 92-106):
 * the lag l in [-max_lag, max_lag] maximising the cross-correlation
 *   c(l) = sum_m r0[m + l] s0[m]   (scipy.signal.correlate(r0, s0, 'full'), :50-58)
 * of the mean-removed first n samples of the clean reference (r0) and of the
 * enhanced output (s0); the first maximum in ascending lag order (np.argmax,
 * :60).  The reference uses n = min(len, 2 s * sr) and max_lag = 0.1 s * sr and
 * skips alignment when n < 256 (:44-46) — the caller applies those rules.
 * Requires max_lag <= 1600 (0.1 s at 16 kHz).
 *
 * cse_xcorr_prepare: per-signal tables (FFT blocks of the clean reference,
 *   fp64 r0, overlap sums, zero-padding energies) into the workspace of
 *   cse_xcorr_workspace_bytes(n_sig, len, n, max_lag) bytes.  clean: [n_sig][len] f64.
 * cse_xcorr_lag: per cell c, the cell's output samples y[0, n) at
 *   head + head_offset[c] (f32, e.g. written by cse_enhance_cells with
 *   out_len >= n), sig_of[c] = its signal.  Outputs:
 *     lag[c]          the alignment lag; -max_lag when status is NONFINITE (a NaN
 *                     or inf in either head makes scipy's correlation NaN at
 *                     every lag, and np.argmax of it is the first kept lag).
 *                     The reference still shifts and length-matches such a
 *                     cell and only then rejects it if a non-finite sample
 *                     remains (:100-103): the lag-l sse/finite of
 *                     cse_enhance_cells decide, as for any other lag
 *     zero_energy[c]  sum of clean^2 over the samples the shifted output leaves
 *                     as zero padding (l > 0: clean[0, l); l < 0: clean[len+l, len)),
 *                     to be added to the lag-l sse of cse_enhance_cells
 *     status[c]       CSE_XCORR_*
 *     corr            optional [n_cells][2 max_lag + 1] f32 c(l) (diagnostics), or NULL
 * Lags whose fp32 FFT correlation lies within 2e-5 ||r0|| ||e|| of the maximum
 * (e the raw head, mean included: the FFT sees it before the mean correction)
 * are re-evaluated exactly in fp64, every one of them: the lag is exact in both
 * OK and FLAT status (FLAT only reports that the slow path ran; an all-zero
 * head is FLAT with lag -max_lag and corr rows of 0).
 */
enum {
    CSE_XCORR_OK = 0,
    CSE_XCORR_FLAT = 1,      /* > 64 near-maximal lags (flat correlation), all re-evaluated in fp64 */
    CSE_XCORR_NONFINITE = 2, /* non-finite head (output or clean): lag -max_lag, corr rows NaN */
};
int64_t cse_xcorr_workspace_bytes(int64_t n_sig, int64_t len, int n, int max_lag);
int cse_xcorr_prepare(const double* clean, int64_t n_sig, int64_t len, int n, int max_lag,
                      void* workspace, cse_stream_t stream);
int cse_xcorr_lag(const float* head, const int64_t* head_offset, const int32_t* sig_of,
                  int64_t n_cells, int64_t n_sig, int n, int max_lag, const void* workspace,
                  int32_t* lag, double* zero_energy, int32_t* status, float* corr,
                  cse_stream_t stream);

/*
 * STOI (pystoi 0.4.1 `stoi(clean, enhanced, sr, extended=False)`, the score of
 * evaluation_metrics.py:30-36 that the reference's sweep optimises at
 * speech_enhancement_comparison.py:180, and its noisy baseline at :115).
 * Both signals are resampled to 10 kHz with Octave's resample filter
 * (pystoi utils.resample_oct).  sr = 16000, the reference's working rate
 * (:381) and the sweep's, is resampled inside the cell kernel; any other
 * rate in [1000, 768000] (filter below 2^25 taps; 10000 = no resampling)
 * goes through a generic fp64 polyphase resampler first (r06).  Workspace
 * and scratch sizes then depend on the rate: the _sr size functions (the
 * plain ones are their sr = 16000 case).
 *
 * cse_stoi_prepare: the clean side, once per signal batch — clean [n_sig][len]
 *   f64 -> workspace of cse_stoi_workspace_bytes(n_sig, len) bytes (10-kHz clean
 *   in fp64, silent-frame mask, kept-frame list, clean band envelopes and
 *   per-segment statistics).
 * cse_stoi_cells: per cell c, the test signal e[n] = y[n - lag[c]] for
 *   n - lag[c] in [0, len), else 0 (finalize_enhanced's shift and
 *   length match, :61-69, :100), clipped to [-1, 1] if clip != 0 (:105),
 *   where y = y_base + y_offset[c] is f32 [len]; clean = signal sig_of[c].
 *   lag may be NULL (all 0).  stoi[c] = the STOI value; 1e-5 when fewer than
 *   30 frames survive the silent-frame removal (pystoi's warning path); NaN
 *   when the signals hold no 256-sample frame at 10 kHz (pystoi raises ->
 *   calculate_stoi returns None).  scratch: cse_stoi_scratch_bytes(n_cells, len)
 *   bytes of device memory (per-cell band envelopes).
 */
int64_t cse_stoi_workspace_bytes(int64_t n_sig, int64_t len);
int64_t cse_stoi_scratch_bytes(int64_t n_cells, int64_t len);
int64_t cse_stoi_workspace_bytes_sr(int64_t n_sig, int64_t len, int sr);  /* -1: rate unsupported */
int64_t cse_stoi_scratch_bytes_sr(int64_t n_cells, int64_t len, int sr);
int cse_stoi_prepare(const double* clean, int64_t n_sig, int64_t len, int sr, void* workspace,
                     cse_stream_t stream);
/* cse_stoi_cells scores signals at 16 kHz; cse_stoi_cells_sr at the rate the
 * workspace was prepared for (n_cells < 65536 per call at other rates). */
int cse_stoi_cells(const float* y, const int64_t* y_offset, const int32_t* lag,
                   const int32_t* sig_of, int64_t n_cells, int64_t n_sig, int64_t len, int clip,
                   const void* workspace, void* scratch, double* stoi, cse_stream_t stream);
int cse_stoi_cells_sr(const float* y, const int64_t* y_offset, const int32_t* lag,
                      const int32_t* sig_of, int64_t n_cells, int64_t n_sig, int64_t len, int sr,
                      int clip, const void* workspace, void* scratch, double* stoi,
                      cse_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* CSE_H_ */
