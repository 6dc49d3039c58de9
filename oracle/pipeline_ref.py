"""Grid enumeration, finalize/SNR and selection semantics — oracle only.

  GRIDS / grid_cells   <- Code/parameter_ranges.py:2-40 enumerated like
                          itertools.product at speech_enhancement_comparison.py:149-157
  to_mono, match_length, align_to_reference, finalize_enhanced
                       <- speech_enhancement_comparison.py:14-21, 29-36, 38-69, 92-106
  calculate_snr        <- evaluation_metrics.py:39-58
  combined_score       <- evaluation_metrics.py:104-115
  tolerance_scan       <- the best-so-far update of speech_enhancement_comparison.py:186-216
"""

import itertools

import numpy as np
from scipy.signal import correlate

# Restated HEAD grid (parameter_ranges.py:2-40). Key order = enumeration order.
GRIDS = {
    "spectralSubtractor": {
        "alpha": [0.5, 0.8, 1.0, 1.5, 2.0, 2.5, 3.0, 4.0, 5.0],
        "beta": [0.001, 0.005, 0.05, 0.1, 0.15],
        "n_fft": [512, 1024],
        "hop_length": [128, 256],
        "noise_percentile": [10.0, 20.0],
        "noise_method": ["percentile", "min_tracking"],
    },
    "mmse": {
        "alpha": [0.90, 0.95, 0.98, 0.99],
        "ksi_min": [0.0001, 0.001, 0.01, 0.05, 0.1, 0.15],
        "gain_min": [0.001, 0.01, 0.05, 0.1, 0.2],
        "gain_max": [1.0],
        "n_fft": [512, 1024],
        "hop_length": [128, 256],
        "noise_percentile": [10.0, 20.0],
        "noise_method": ["percentile", "min_tracking"],
    },
    "wiener": {
        "alpha": [0.90, 0.95, 0.98],
        "gain_floor": [0.01, 0.02, 0.05, 0.1],
        "n_fft": [512, 1024],
        "hop_length": [128, 256],
        "noise_percentile": [10.0, 20.0],
        "noise_method": ["percentile", "min_tracking"],
    },
    "omlsa": {
        "alpha": [0.7, 0.80, 0.9, 0.95],
        "ksi_min": [0.001, 0.005, 0.01, 0.05],
        "gain_floor": [0.05, 0.1, 0.2],
        "noise_mu": [0.92, 0.95, 0.98],
        "q": [0.3, 0.4, 0.5],
        "n_fft": [512, 1024],
        "hop_length": [128, 256],
        "noise_percentile": [10.0, 20.0],
        "noise_method": ["percentile", "min_tracking"],
    },
}


def grid_cells(ranges):
    """List of param dicts in itertools.product order (last key fastest)."""
    names = list(ranges.keys())
    return [dict(zip(names, combo)) for combo in itertools.product(*ranges.values())]


def to_mono(x):
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        return x
    return x.mean(axis=1) if x.shape[0] >= x.shape[1] else x.mean(axis=0)


def match_length(x, L):
    x = np.asarray(x, dtype=np.float64)
    if len(x) > L:
        return x[:L]
    if len(x) < L:
        return np.pad(x, (0, L - len(x)))
    return x


def align_lag(ref, sig, sr, max_shift_s=0.10, corr_seconds=2.0):
    """Cross-correlation lag used by align_to_reference (None = no shift)."""
    ref = np.asarray(ref, dtype=np.float64)
    sig = np.asarray(sig, dtype=np.float64)
    n = int(min(len(ref), len(sig), corr_seconds * sr))
    if n < 256:
        return None
    r0 = ref[:n] - np.mean(ref[:n])
    s0 = sig[:n] - np.mean(sig[:n])
    c = correlate(r0, s0, mode="full", method="auto")
    lags = np.arange(-len(s0) + 1, len(r0))
    max_lag = int(max_shift_s * sr)
    keep = (lags >= -max_lag) & (lags <= max_lag)
    if not np.any(keep):
        return None
    return int(lags[keep][np.argmax(c[keep])])


def shift_by_lag(sig, lag):
    if lag is None or lag == 0:
        return sig
    if lag > 0:
        return np.pad(sig, (lag, 0))
    return sig[-lag:]


def align_to_reference(ref, sig, sr, max_shift_s=0.10, corr_seconds=2.0):
    return shift_by_lag(np.asarray(sig, dtype=np.float64),
                        align_lag(ref, sig, sr, max_shift_s, corr_seconds))


def finalize_enhanced(enhanced, clean_ref, sr, do_align=True):
    """Align to the clean reference, length-match, reject non-finite, clip."""
    e = to_mono(enhanced)
    if do_align:
        e = align_to_reference(clean_ref, e, sr)
    e = match_length(e, len(clean_ref))
    if not np.all(np.isfinite(e)):
        return None
    return np.clip(e, -1.0, 1.0)


def calculate_snr(clean, processed):
    clean = np.asarray(clean)
    processed = np.asarray(processed)
    m = min(len(clean), len(processed))
    err = clean[:m] - processed[:m]
    ps = np.sum(clean[:m] ** 2)
    pn = np.sum(err ** 2)
    if pn == 0:
        return float("inf")
    return float(10 * np.log10(ps / (pn + 1e-10)))


def combined_score(stoi, pesq):
    stoi = 0 if stoi is None else stoi
    pesq = 0 if pesq is None else pesq
    return 0.5 * stoi + 0.5 * (max(0, pesq) / 4.5)


def tolerance_scan(scores, tol, initial=-1.0):
    """Index of the winner of the reference's sequential best-so-far update.

    A cell replaces the incumbent only if score > best + tol, scanned in grid
    order; None/NaN-skipped cells are given as None.  Returns -1 if no cell
    ever won.  (Not an argmax: ties within tol keep the EARLIER cell.)
    """
    best, idx = initial, -1
    for i, s in enumerate(scores):
        if s is None:
            continue
        if s > best + tol:
            best, idx = s, i
    return idx
