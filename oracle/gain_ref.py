"""The four enhancement algorithms restated in numpy (fp64) — oracle only.

Each public function has the reference's plugin signature
``alg(noisy_audio, sr, **params) -> np.ndarray`` (float64, len(noisy)):
  spectral_subtraction <- Code/spectral_subtractor.py:6-65
  wiener_filter        <- Code/wiener_filter.py:7-95   (frame loop :55-82)
  mmse                 <- Code/mmse.py:6-120           (smoothing :48-54, loop :65-106)
  advanced_mmse        <- Code/advanced_mmse.py:7-136  (smoothing :60-66, loop :82-124)

The per-frame recursions are written as explicit loops over t, vectorised over
bins, like the reference (this module doubles as the CPU baseline).
"""

import numpy as np
from scipy.special import expn, i0, i1

from .noise_ref import noise_estimation
from .stft_ref import fix_length, istft, stft


def _mono(x, mean_axis_rule):
    x = np.asarray(x, dtype=np.float64)
    if x.ndim > 1:
        if mean_axis_rule == "shorter":
            x = x.mean(axis=0) if x.shape[0] < x.shape[1] else x.mean(axis=1)
        else:
            x = x.mean(axis=1)
    return x


def analyse(noisy, sr, n_fft, hop_length, noise_percentile, noise_method,
            clean_audio, eps):
    """STFT + noise estimate shared by all four algorithms."""
    Y = stft(noisy, n_fft, hop_length)
    P = np.abs(Y) ** 2
    N = noise_estimation(noisy, sr=sr, n_fft=n_fft, hop_length=hop_length,
                         win_length=n_fft, window="hann", center=True,
                         pad_mode="reflect", percentile=noise_percentile,
                         method=noise_method, clean_audio=clean_audio, eps=eps)
    return Y, P, N


def _column(N, t):
    """The noise column of frame t: (B,T>1) arrays are time-varying."""
    return N[:, t:t + 1] if (N.ndim == 2 and N.shape[1] > 1) else N


def smooth_noise(N, mu):
    """First-order IIR over frames (mmse.py:48-54, advanced_mmse.py:60-66)."""
    mu = float(np.clip(mu, 0.0, 0.9999))
    out = np.empty_like(N)
    out[:, 0] = N[:, 0]
    for t in range(1, N.shape[1]):
        out[:, t] = mu * out[:, t - 1] + (1.0 - mu) * N[:, t]
    return out


# ----------------------------------------------------------------------------
# gains
# ----------------------------------------------------------------------------

def ss_spectrum(Y, P, N, alpha, beta):
    """Berouti subtraction with noisy phase (spectral_subtractor.py:43-53)."""
    Ps = np.maximum(P - alpha * N, beta * N)
    return np.sqrt(Ps) * np.exp(1j * np.angle(Y))


def wiener_gains(P, N, alpha, gain_floor, eps=1e-10):
    """Decision-directed Wiener gain, serial over frames (wiener_filter.py:55-82)."""
    B, T = P.shape
    G = np.zeros((B, T))
    g_prev = np.ones((B, 1))
    gam_prev = np.ones((B, 1))
    for t in range(T):
        n = np.maximum(_column(N, t), eps)
        gam = np.maximum(P[:, t:t + 1] / n, eps)
        d = np.maximum(gam - 1.0, 0.0)
        xi = d if t == 0 else alpha * ((g_prev ** 2) * gam_prev) + (1.0 - alpha) * d
        xi = np.maximum(xi, 1e-10)
        g = np.clip(xi / (1.0 + xi), gain_floor, 1.0)
        G[:, t:t + 1] = g
        g_prev, gam_prev = g, gam
    return G


def mmse_gains(P, N, alpha, ksi_min, gain_min, gain_max, eps=1e-12):
    """Ephraim–Malah MMSE-STSA gain, serial over frames (mmse.py:65-106)."""
    B, T = P.shape
    G = np.zeros((B, T))
    g_prev = np.ones((B, 1))
    gam_prev = np.ones((B, 1))
    c0 = np.sqrt(np.pi) / 2.0
    for t in range(T):
        n = np.maximum(_column(N, t), eps)
        gam = np.maximum(P[:, t:t + 1] / n, eps)
        d = np.maximum(gam - 1.0, 0.0)
        if t == 0:
            xi = np.maximum(gam - 1.0, ksi_min)
        else:
            xi = np.maximum(alpha * ((g_prev ** 2) * gam_prev) + (1.0 - alpha) * d, ksi_min)
        v = np.clip((xi * gam) / (1.0 + xi), eps, 80.0)
        x = 0.5 * v
        g = (c0 * (np.sqrt(v) / (gam + eps))) * np.exp(-x) * ((1.0 + v) * i0(x) + v * i1(x))
        g = np.nan_to_num(g, nan=gain_min, posinf=gain_max, neginf=gain_min)
        g = np.clip(g, gain_min, gain_max)
        G[:, t:t + 1] = g
        g_prev, gam_prev = g, gam
    return G


def omlsa_gains(P, N, alpha, ksi_min, q, gain_floor, eps=1e-10, v_max=80.0):
    """Log-MMSE (LSA) x speech-presence soft gain (advanced_mmse.py:82-124)."""
    B, T = P.shape
    G = np.zeros((B, T))
    qv = float(np.clip(q, 1e-3, 1 - 1e-3))
    g_prev = np.ones((B, 1)) * gain_floor
    gam_prev = np.ones((B, 1))
    for t in range(T):
        n = np.maximum(_column(N, t), eps)
        gam = np.maximum(P[:, t:t + 1] / n, eps)
        if t == 0:
            xi = np.maximum(gam - 1.0, ksi_min)
        else:
            d = np.maximum(gam - 1.0, 0.0)
            xi = np.maximum(alpha * ((g_prev ** 2) * gam_prev) + (1.0 - alpha) * d, ksi_min)
        v = np.clip((xi * gam) / (1.0 + xi), 1e-12, v_max)
        g_lsa = (xi / (1.0 + xi)) * np.exp(0.5 * expn(1, v))
        g_lsa = np.nan_to_num(g_lsa, nan=gain_floor, posinf=1.0, neginf=gain_floor)
        lam = (1.0 / (1.0 + xi)) * np.exp(v)
        p = np.clip(1.0 / (1.0 + (1.0 - qv) / (qv * lam + eps)), 0.0, 1.0)
        g = np.clip((g_lsa ** p) * (gain_floor ** (1.0 - p)), gain_floor, 1.0)
        G[:, t:t + 1] = g
        g_prev, gam_prev = g, gam
    return G


# ----------------------------------------------------------------------------
# plugin-shaped algorithms (the reference's alg_fn(noisy, sr, **params))
# ----------------------------------------------------------------------------

def spectral_subtraction(noisy_audio, sr, alpha, beta, n_fft, hop_length,
                         noise_percentile, noise_method, clean_audio=None):
    x = _mono(noisy_audio, "shorter")
    L, eps = len(x), 1e-10
    Y, P, N = analyse(x, sr, n_fft, hop_length, noise_percentile, noise_method,
                      clean_audio, eps)
    N = np.maximum(N, eps)
    if N.ndim == 2 and N.shape[1] != P.shape[1]:
        N = fix_length(N, size=P.shape[1], axis=1)
    S = ss_spectrum(Y, P, N, alpha, beta)
    return fix_length(istft(S, hop_length=hop_length, win_length=n_fft, length=L), size=L)


def wiener_filter(noisy_audio, sr, n_fft, hop_length, alpha, gain_floor,
                  noise_percentile, noise_method, clean_audio=None):
    x = _mono(noisy_audio, "axis1")
    L, eps = len(x), 1e-10
    Y, P, N = analyse(x, sr, n_fft, hop_length, noise_percentile, noise_method,
                      clean_audio, eps)
    N = np.maximum(N, eps)
    G = wiener_gains(P, N, alpha, gain_floor, eps)
    return istft(Y * G, hop_length=hop_length, win_length=n_fft, length=L)


def mmse(noisy_audio, sr, alpha, ksi_min, gain_min, gain_max, n_fft, hop_length,
         noise_percentile, noise_method, noise_mu=0.98, clean_audio=None,
         log=True, log_every=50):
    x = _mono(noisy_audio, "axis1")
    L, eps = len(x), 1e-12
    Y, P, N = analyse(x, sr, n_fft, hop_length, noise_percentile, noise_method,
                      clean_audio, eps)
    if noise_method != "true_noise" and N.ndim == 2 and N.shape[1] > 1:
        N = smooth_noise(N, noise_mu)
    G = mmse_gains(P, N, alpha, ksi_min, gain_min, gain_max, eps)
    return istft(Y * G, hop_length=hop_length, win_length=n_fft, length=L)


def advanced_mmse(noisy_audio, sr, n_fft, hop_length, alpha, ksi_min, q, noise_mu,
                  gain_floor, noise_percentile, noise_method, clean_audio=None,
                  v_max=80.0):
    x = _mono(noisy_audio, "shorter")
    L, eps = len(x), 1e-10
    Y, P, N = analyse(x, sr, n_fft, hop_length, noise_percentile, noise_method,
                      clean_audio, eps)
    N = np.maximum(N, eps)
    if N.ndim == 2 and N.shape[1] != P.shape[1]:
        N = fix_length(N, size=P.shape[1], axis=1)
    if noise_method != "true_noise" and N.ndim == 2 and N.shape[1] > 1:
        N = smooth_noise(N, noise_mu)
    G = omlsa_gains(P, N, alpha, ksi_min, q, gain_floor, eps, v_max)
    y = istft(Y * G, hop_length=hop_length, win_length=n_fft, length=L)
    return fix_length(y, size=L)


ALGORITHMS = {
    "spectralSubtractor": spectral_subtraction,
    "mmse": mmse,
    "wiener": wiener_filter,
    "omlsa": advanced_mmse,
}
