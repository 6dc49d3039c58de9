"""Drop-in mirrors of the reference's plugin functions, computed on MI355X.

Same names, argument meaning and error behaviour as
  spectral_subtraction   Code/spectral_subtractor.py:6
  wiener_filter          Code/wiener_filter.py:7
  mmse                   Code/mmse.py:6
  advanced_mmse          Code/advanced_mmse.py:7
  noise_estimation       Code/noise_estimation.py:158
Each returns a float64 numpy array like the reference; the numbers come from
libcse.so (STFT, estimator and fused gain+ISTFT kernels), computed in fp32 on
the device (fp64 analysis), within the 1e-5 relative tolerance of the
north-star.  There is no CPU fallback: without the built library or a GPU
these raise.
"""

import numpy as np
import torch

from .engine import NOISE_PARAM_KEYS, Engine, n_frames

_ENGINE = None


def engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = Engine()
    return _ENGINE


def _mono(x, rule):
    x = np.asarray(x, dtype=np.float64)
    if x.ndim > 1:
        if rule == "shorter":  # spectral_subtractor.py:12-14, advanced_mmse.py:27-29
            x = x.mean(axis=0) if x.shape[0] < x.shape[1] else x.mean(axis=1)
        else:  # wiener_filter.py:24-25, mmse.py:13-14
            x = x.mean(axis=1)
    return x


def _dev(x):
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64)).cuda().view(1, -1)


def _single(alg, noisy, clean, params, rule):
    x = _mono(noisy, rule)
    if x.size == 0:  # the reference's reflect padding of an empty signal raises
        raise ValueError("can't extend empty axis 0 using modes other than 'constant' or 'empty'")
    eng = engine()
    c, m = None, None
    if clean is not None and params.get("noise_method") == "true_noise":
        cl = np.asarray(clean, dtype=np.float64)
        # TrueNoiseEstimator trims both to the shorter (noise_estimation.py:128-130),
        # takes the STFT of the difference and edge-pads its frames to the
        # noisy signal's (:149-153): the engine's true_len
        m = min(len(cl), len(x))
        if m == 0:
            if n_frames(len(x), params["hop_length"]) >= 5:  # below 5 frames no estimator runs
                # librosa.stft of the empty difference signal raises
                raise ValueError("can't extend empty axis 0 using modes other than 'constant' or 'empty'")
        c = np.zeros_like(x)
        c[:m] = cl[:m]
        m = m or None
    res = eng.run(_dev(x), [(0, alg, params)], clean=None if c is None else _dev(c),
                  want_waveforms=True, true_len=m)
    return res["y"][0].cpu().numpy().astype(np.float64)


def spectral_subtraction(noisy_audio, sr, alpha, beta, n_fft, hop_length, noise_percentile,
                         noise_method, clean_audio=None):
    return _single("spectralSubtractor", noisy_audio, clean_audio,
                   dict(alpha=alpha, beta=beta, n_fft=n_fft, hop_length=hop_length,
                        noise_percentile=noise_percentile, noise_method=noise_method),
                   "shorter")


def wiener_filter(noisy_audio, sr, n_fft, hop_length, alpha, gain_floor, noise_percentile,
                  noise_method, clean_audio=None):
    return _single("wiener", noisy_audio, clean_audio,
                   dict(alpha=alpha, gain_floor=gain_floor, n_fft=n_fft, hop_length=hop_length,
                        noise_percentile=noise_percentile, noise_method=noise_method), "axis1")


def mmse(noisy_audio, sr, alpha, ksi_min, gain_min, gain_max, n_fft, hop_length,
         noise_percentile, noise_method, noise_mu=0.98, clean_audio=None, log=True,
         log_every=50):
    return _single("mmse", noisy_audio, clean_audio,
                   dict(alpha=alpha, ksi_min=ksi_min, gain_min=gain_min, gain_max=gain_max,
                        n_fft=n_fft, hop_length=hop_length, noise_percentile=noise_percentile,
                        noise_method=noise_method, noise_mu=noise_mu), "axis1")


def advanced_mmse(noisy_audio, sr, n_fft, hop_length, alpha, ksi_min, q, noise_mu, gain_floor,
                  noise_percentile, noise_method, clean_audio=None, v_max=80.0):
    return _single("omlsa", noisy_audio, clean_audio,
                   dict(alpha=alpha, ksi_min=ksi_min, q=q, noise_mu=noise_mu,
                        gain_floor=gain_floor, n_fft=n_fft, hop_length=hop_length,
                        noise_percentile=noise_percentile, noise_method=noise_method,
                        v_max=v_max), "shorter")


def noise_estimation(y, sr, method="percentile", n_fft=1024, hop_length=256, win_length=None,
                     estimator_params=None, window="hann", center=True, pad_mode="reflect",
                     **kwargs):
    """Noise PSD (B,1) or (B,T) float64, like noise_estimation.py:158-212.

    Argument flow as there: the estimator is constructed from
    {**estimator_params, **kwargs} (:175, :197; percentile, min_frames,
    max_fraction, floor_rel, adaptive_short, window_size, smoothing_factor),
    while estimate() reads eps and clean_audio from **kwargs only (:199-210):
    eps defaults to 1e-10 (percentile, min_tracking) / 1e-12 (true_noise), the
    T < 5 fallback reads eps from the merged dict (:191-195)."""
    if window != "hann" or not center or pad_mode != "reflect" or (win_length or n_fft) != n_fft:
        raise NotImplementedError("only hann/center/reflect/win_length=n_fft is implemented")
    full = dict(estimator_params or {})
    full.update(kwargs)
    ctor = {k: full[k] for k in NOISE_PARAM_KEYS if k in full}
    x = np.asarray(y, dtype=np.float64)
    if x.ndim > 1:
        x = x.mean(axis=1)
    if x.size == 0:  # librosa's reflect padding of an empty signal raises
        raise ValueError("can't extend empty axis 0 using modes other than 'constant' or 'empty'")
    eng = engine()
    xd = _dev(x)
    T = n_frames(len(x), hop_length)
    if T < 5:
        _, P = eng.stft(xd, n_fft, hop_length, want_y=False)
        N = eng.noise_estimate("percentile", P, 25.0, full.get("eps", 1e-10))
        return N[0].cpu().numpy().astype(np.float64)[:, None]
    if method == "percentile":
        _, P = eng.stft(xd, n_fft, hop_length, want_y=False)
        N = eng.noise_estimate("percentile", P, eps=kwargs.get("eps", 1e-10), **ctor)
        return N[0].cpu().numpy().astype(np.float64)[:, None]
    if method == "min_tracking":
        _, P = eng.stft(xd, n_fft, hop_length, want_y=False)
        N = eng.noise_estimate("min_tracking", P, eps=kwargs.get("eps", 1e-10), **ctor)
        return N[0].cpu().numpy().astype(np.float64).T
    if method == "true_noise":
        clean = kwargs.get("clean_audio")
        if clean is None:
            raise ValueError("TrueNoiseEstimator requires clean_audio and noisy_audio")
        clean = np.asarray(clean, dtype=np.float64)
        m = min(len(clean), len(x))  # :128-130
        if m == 0:
            raise ValueError("can't extend empty axis 0 using modes other than 'constant' or 'empty'")
        _, P = eng.stft(_dev(x[:m]), n_fft, hop_length, x_sub=_dev(clean[:m]), want_y=False)
        out = eng.noise_estimate("true_noise", P, eps=kwargs.get("eps", 1e-12), frames=T)
        return out[0].cpu().numpy().astype(np.float64).T
    raise ValueError(f"Unbekannte Methode: {method}")
