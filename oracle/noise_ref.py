"""Noise-PSD estimators restated in numpy (fp64) — oracle only.

Follows Code/noise_estimation.py of the reference:
  percentile_noise     <- PercentileNoiseEstimator.estimate   :20-56
  min_tracking_noise   <- MinTrackingNoiseEstimator.estimate  :64-95 (+ :97-99)
  true_noise           <- TrueNoiseEstimator.estimate         :115-155
  simple_noise         <- _simple_noise_estimate              :226-232
  noise_estimation     <- noise_estimation + _create_estimator :158-223
"""

import numpy as np
from scipy.ndimage import minimum_filter1d

from .stft_ref import stft


def percentile_quiet_count(n_frames, percentile=20.0, min_frames=10,
                           max_fraction=0.30, adaptive_short=True):
    """(k, percentile) exactly as noise_estimation.py:29-41 evaluates them."""
    if adaptive_short and n_frames < 30:
        min_frames = max(2, n_frames // 4)
        target = max(3, int(n_frames * 0.15))
        percentile = min(50.0, 100.0 * target / n_frames)
    k = max(min_frames, int(np.ceil(n_frames * (percentile / 100.0))))
    k = min(k, max(1, int(np.ceil(n_frames * max_fraction))))
    k = min(k, n_frames)
    return k, percentile


def percentile_noise(power, eps=1e-10, percentile=20.0, min_frames=10,
                     max_fraction=0.30, floor_rel=0.02, adaptive_short=True):
    """Static (B,1) PSD: percentile over the k quietest frames, median floor."""
    k, pct = percentile_quiet_count(power.shape[1], percentile, min_frames,
                                    max_fraction, adaptive_short)
    energy = np.log(np.maximum(power, eps)).mean(axis=0)
    quiet = np.argsort(energy)[:k]
    est = np.percentile(power[:, quiet], pct, axis=1, keepdims=True)
    floor = floor_rel * np.median(power, axis=1, keepdims=True)
    return np.maximum(np.maximum(est, floor), eps)


def min_tracking_window(n_frames, window_size=50):
    w = min(max(3, window_size), n_frames)
    return w if w % 2 == 1 else w + 1


def min_tracking_noise(power, eps=1e-10, window_size=50, smoothing_factor=None):
    """Time-varying (B,T) PSD: IIR smoothing then a centred running minimum."""
    n_bins, n_frames = power.shape
    a = smoothing_factor
    if a is None:
        a = max(0.8, min(0.95, 1 - 5 / n_frames))
    sm = np.empty_like(power)
    sm[:, 0] = power[:, 0]
    for t in range(1, n_frames):
        sm[:, t] = a * sm[:, t - 1] + (1 - a) * power[:, t]
    w = min_tracking_window(n_frames, window_size)
    mins = minimum_filter1d(sm, size=w, axis=1, mode="nearest")
    floor = 0.01 * np.median(power, axis=1, keepdims=True)
    return np.maximum(np.maximum(mins, floor), eps)


def true_noise(power, noisy, clean, n_fft, hop_length, eps=1e-12):
    """Oracle PSD |STFT(noisy - clean)|², frame-matched to ``power``."""
    if clean is None or noisy is None:
        raise ValueError("TrueNoiseEstimator requires clean_audio and noisy_audio")
    m = min(len(clean), len(noisy))
    d = np.asarray(noisy[:m], dtype=np.float64) - np.asarray(clean[:m], dtype=np.float64)
    npsd = np.maximum(np.abs(stft(d, n_fft, hop_length)) ** 2, eps)
    T = power.shape[1]
    if npsd.shape[1] > T:
        npsd = npsd[:, :T]
    elif npsd.shape[1] < T:
        npsd = np.pad(npsd, ((0, 0), (0, T - npsd.shape[1])), mode="edge")
    return npsd


def simple_noise(power, eps=1e-10):
    """T < 5 fallback: mean (T<2) or 25th percentile over frames."""
    if power.shape[1] < 2:
        est = power.mean(axis=1, keepdims=True)
    else:
        est = np.percentile(power, 25, axis=1, keepdims=True)
    return np.maximum(est, eps)


def noise_estimation(y, sr, method="percentile", n_fft=1024, hop_length=256,
                     win_length=None, estimator_params=None, window="hann",
                     center=True, pad_mode="reflect", **kwargs):
    """Dispatch of noise_estimation.py:158-212.  The estimator is constructed
    from {**estimator_params, **kwargs} (:175, :197), estimate() reads eps and
    clean_audio from **kwargs alone (:199-210); the T < 5 fallback reads eps
    from the merged dict (:191-195)."""
    params = dict(estimator_params or {})
    params.update(kwargs)
    y = np.asarray(y, dtype=np.float64)
    if y.ndim > 1:
        y = y.mean(axis=1)
    power = np.abs(stft(y, n_fft, hop_length, win_length, window, center,
                        pad_mode)) ** 2
    if power.shape[1] < 5:
        return simple_noise(power, params.get("eps", 1e-10))
    if method == "percentile":
        keys = ("percentile", "min_frames", "max_fraction", "floor_rel",
                "adaptive_short")
        return percentile_noise(power, eps=kwargs.get("eps", 1e-10),
                                **{k: params[k] for k in keys if k in params})
    if method == "min_tracking":
        keys = ("window_size", "smoothing_factor")
        return min_tracking_noise(power, eps=kwargs.get("eps", 1e-10),
                                  **{k: params[k] for k in keys if k in params})
    if method == "true_noise":
        return true_noise(power, y, kwargs.get("clean_audio"), n_fft, hop_length,
                          eps=kwargs.get("eps", 1e-12))
    raise ValueError(f"Unbekannte Methode: {method}")


def quiet_frame_order(power, eps):
    """Frame indices sorted by mean log-energy (the selection order of :44-47)."""
    return np.argsort(np.log(np.maximum(power, eps)).mean(axis=0))

