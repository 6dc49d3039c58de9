"""STOI (short-time objective intelligibility) — oracle only.

The reference scores every grid cell with ``pystoi.stoi(clean, enhanced, sr,
extended=False)`` (``Code/evaluation_metrics.py:30-36``, called from
``speech_enhancement_comparison.py:180`` and ``:115`` for the noisy baseline).
pystoi is a third-party dependency that is absent from /root/reference and
from this image.  The reference report (§3.1) pins it as **pystoi 0.4.1**;
this module restates that version's published algorithm (Taal et al., "An
algorithm for intelligibility prediction of time-frequency weighted noisy
speech", IEEE TASLP 2011), in float64:

  1. resample to 10 kHz with Octave's ``resample`` filter
     (``utils.resample_oct``: Kaiser-windowed sinc, 60 dB rejection,
     roll-off = cutoff/10, applied with ``scipy.signal.resample_poly``);
  2. drop frames (256 samples, hop 128, Hann without its zero endpoints) of the
     CLEAN signal more than 40 dB below its loudest frame, in both signals,
     and overlap-add the kept frames back (``utils.remove_silent_frames``);
  3. STFT: 256-sample Hann frames at hop 128, 512-point rfft, frames starting
     at ``range(0, len - 256, 128)`` (``utils.stft``);
  4. 15 one-third-octave bands from 150 Hz (``utils.thirdoct``): band
     envelopes sqrt(OBM @ |X|^2);
  5. segments of 30 frames: normalise y to x's segment norm, clip at
     x·(1 + 10^(15/20)), remove means, normalise, correlate, average over
     bands and segments; fewer than 30 frames returns 1e-5.

Parity: pystoi itself cannot run here, so the restatement is pinned loosely
by the reference's own outputs — ``all_results.json`` holds the STOI values
the reference computed for the two stems whose clean/noisy/enhanced WAVs are
committed under ``Document/Presentation`` (tests/golden/stoi_pins.npz, made by
tests/golden/make_stoi_pins.py).  The 48-kHz inputs pass through a resampler
stand-in (librosa's soxr is absent) and the enhanced WAVs are PCM16, so the pin
is not bit-level: the 8 recorded values are reproduced to <= 1.9e-5.
"""

import numpy as np
from scipy.signal import resample_poly

FS = 10000
N_FRAME = 256
NFFT = 512
NUMBAND = 15
MINFREQ = 150
N_SEG = 30
BETA = -15.0
DYN_RANGE = 40
EPS = np.finfo("float").eps


def resample_window_oct(p, q):
    """Octave's resample filter (pystoi utils._resample_window_oct)."""
    g = np.gcd(int(p), int(q))
    p, q = p / g, q / g
    log10_rejection = -3.0
    stopband_cutoff_f = 1.0 / (2 * max(p, q))
    roll_off_width = stopband_cutoff_f / 10
    rejection_db = -20 * log10_rejection
    L = np.ceil((rejection_db - 8) / (28.714 * roll_off_width))
    t = np.arange(-L, L + 1)
    ideal = 2 * p * stopband_cutoff_f * np.sinc(2 * stopband_cutoff_f * t)
    if 21 <= rejection_db <= 50:
        beta = 0.5842 * (rejection_db - 21) ** 0.4 + 0.07886 * (rejection_db - 21)
    elif rejection_db > 50:
        beta = 0.1102 * (rejection_db - 8.7)
    else:
        beta = 0.0
    return np.kaiser(2 * L + 1, beta) * ideal


def resample_oct(x, p, q):
    """pystoi utils.resample_oct: resample_poly with the normalised Octave window."""
    h = resample_window_oct(p, q)
    return resample_poly(x, p, q, window=h / np.sum(h))


def hann_matlab(n):
    """MATLAB hanning(n): scipy hann(n + 2) without its zero endpoints."""
    k = np.arange(1, n + 1)
    return 0.5 - 0.5 * np.cos(2 * np.pi * k / (n + 1))


def thirdoct(fs=FS, nfft=NFFT, num_bands=NUMBAND, min_freq=MINFREQ):
    """One-third-octave band matrix (pystoi utils.thirdoct); rows = bands."""
    f = np.linspace(0, fs, nfft + 1)[: nfft // 2 + 1]
    k = np.arange(num_bands, dtype=float)
    freq_low = min_freq * np.power(2.0, (2 * k - 1) / 6)
    freq_high = min_freq * np.power(2.0, (2 * k + 1) / 6)
    obm = np.zeros((num_bands, len(f)))
    for i in range(num_bands):
        lo = int(np.argmin(np.square(f - freq_low[i])))
        hi = int(np.argmin(np.square(f - freq_high[i])))
        obm[i, lo:hi] = 1
    return obm


OBM = thirdoct()


def band_edges():
    """[lo, hi) bin range of each band (the non-zero span of each OBM row)."""
    out = []
    for row in OBM:
        nz = np.nonzero(row)[0]
        out.append((int(nz[0]), int(nz[-1]) + 1))
    return out


def _overlap_and_add(frames, hop):
    n, flen = frames.shape
    out = np.zeros((n - 1) * hop + flen) if n else np.zeros(0)
    for i in range(n):
        out[i * hop:i * hop + flen] += frames[i]
    return out


def silent_mask(x, dyn_range=DYN_RANGE, framelen=N_FRAME, hop=N_FRAME // 2):
    """Kept-frame mask of remove_silent_frames (computed from x only)."""
    w = hann_matlab(framelen)
    starts = range(0, len(x) - framelen + 1, hop)
    e = np.array([20 * np.log10(np.linalg.norm(w * x[i:i + framelen]) + EPS) for i in starts])
    if e.size == 0:  # pystoi: norm(axis=1) of the empty frame array raises
        raise ValueError("no frame of framelen samples")
    return (np.max(e) - dyn_range - e) < 0


def remove_silent_frames(x, y, dyn_range=DYN_RANGE, framelen=N_FRAME, hop=N_FRAME // 2):
    """pystoi utils.remove_silent_frames."""
    w = hann_matlab(framelen)
    starts = list(range(0, len(x) - framelen + 1, hop))
    mask = silent_mask(x, dyn_range, framelen, hop)
    xf = np.array([w * x[i:i + framelen] for i in starts]).reshape(-1, framelen)[mask]
    yf = np.array([w * y[i:i + framelen] for i in starts]).reshape(-1, framelen)[mask]
    return _overlap_and_add(xf, hop), _overlap_and_add(yf, hop)


def stft(x, win_size=N_FRAME, fft_size=NFFT, overlap=2):
    """pystoi utils.stft: frames at range(0, len - win, hop) -> (frames, bins)."""
    hop = win_size // overlap
    w = hann_matlab(win_size)
    starts = range(0, len(x) - win_size, hop)
    return np.array([np.fft.rfft(w * x[i:i + win_size], n=fft_size) for i in starts]).reshape(-1, fft_size // 2 + 1)


def band_envelopes(sig_spec):
    """sqrt(OBM @ |X|^2): (bands, frames)."""
    return np.sqrt(OBM @ np.square(np.abs(sig_spec.T)))


def stoi_from_envelopes(x_tob, y_tob):
    """Intermediate intelligibility averaged over bands and segments (eqs. 3-6)."""
    M = x_tob.shape[1]
    xs = np.array([x_tob[:, m - N_SEG:m] for m in range(N_SEG, M + 1)])
    ys = np.array([y_tob[:, m - N_SEG:m] for m in range(N_SEG, M + 1)])
    norm_const = np.linalg.norm(xs, axis=2, keepdims=True) / (np.linalg.norm(ys, axis=2, keepdims=True) + EPS)
    yn = ys * norm_const
    clip_value = 10 ** (-BETA / 20)
    yp = np.minimum(yn, xs * (1 + clip_value))
    yp = yp - np.mean(yp, axis=2, keepdims=True)
    xs = xs - np.mean(xs, axis=2, keepdims=True)
    yp /= (np.linalg.norm(yp, axis=2, keepdims=True) + EPS)
    xs /= (np.linalg.norm(xs, axis=2, keepdims=True) + EPS)
    J, Mb = xs.shape[0], xs.shape[1]
    return float(np.sum(yp * xs) / (J * Mb))


def stoi(x, y, fs_sig):
    """pystoi 0.4.1 ``stoi(x, y, fs_sig, extended=False)``."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if x.shape != y.shape:
        raise Exception(f"x and y should have the same length, found {x.shape} and {y.shape}")
    if fs_sig != FS:
        x = resample_oct(x, FS, fs_sig)
        y = resample_oct(y, FS, fs_sig)
    x, y = remove_silent_frames(x, y)
    xs = stft(x)
    ys = stft(y)
    if xs.shape[0] < N_SEG:
        return 1e-5
    return stoi_from_envelopes(band_envelopes(xs), band_envelopes(ys))


def calculate_stoi(clean_reference, test_audio, sr):
    """evaluation_metrics.calculate_stoi (:30-36): trim to the common length."""
    try:
        n = min(len(clean_reference), len(test_audio))
        return stoi(clean_reference[:n], test_audio[:n], sr)
    except Exception:
        return None
