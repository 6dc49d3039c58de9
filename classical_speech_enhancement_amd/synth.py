"""Deterministic synthetic clean/noisy pairs (SURVEY §8(d) "Synthetic inputs").

There is no dataset in the image (the reference's ``Code/data`` is git-ignored),
so benches and parity tests run on speech-like synthetic clips:
  * clean: harmonic bursts (f0 ~ U[100, 250] Hz, 10 harmonics with 1/k
    amplitude, 4 Hz syllabic AM) with ~30 % silent gaps, peak 0.3;
  * noisy: clean + white (even i) or pink (odd i) noise at SNR ~ U[-5, 15] dB,
    clipped to ±1, plus 1e-6 dither so no two frame energies tie.
Pair i uses ``np.random.default_rng(1000 + i)``.
"""

import numpy as np


def _pink(rng, n):
    """1/f noise by spectral shaping of white noise."""
    w = rng.standard_normal(n)
    spec = np.fft.rfft(w)
    f = np.arange(spec.shape[0], dtype=np.float64)
    f[0] = 1.0
    spec /= np.sqrt(f)
    p = np.fft.irfft(spec, n=n)
    return p / (np.std(p) + 1e-30)


def make_pair(i, seconds=10.0, sr=16000):
    """Return (clean, noisy) float64 arrays of length round(seconds*sr)."""
    rng = np.random.default_rng(1000 + i)
    n = int(round(seconds * sr))
    t = np.arange(n) / sr
    clean = np.zeros(n)
    # syllable-length segments, ~30 % of them silent
    pos = 0
    while pos < n:
        seg = int(rng.uniform(0.12, 0.45) * sr)
        end = min(n, pos + seg)
        if rng.uniform() > 0.3:
            f0 = rng.uniform(100.0, 250.0)
            tt = t[pos:end]
            x = np.zeros(end - pos)
            for k in range(1, 11):
                x += np.sin(2 * np.pi * k * f0 * tt + rng.uniform(0, 2 * np.pi)) / k
            am = 0.5 - 0.5 * np.cos(2 * np.pi * 4.0 * (tt - tt[0]))
            ramp = np.minimum(1.0, np.minimum(np.arange(end - pos), np.arange(end - pos)[::-1]) / (0.01 * sr))
            clean[pos:end] = x * am * ramp
        pos = end
    peak = np.max(np.abs(clean))
    if peak > 0:
        clean *= 0.3 / peak
    noise = rng.standard_normal(n) if i % 2 == 0 else _pink(rng, n)
    snr_db = rng.uniform(-5.0, 15.0)
    p_s = np.mean(clean ** 2)
    p_n = np.mean(noise ** 2)
    noise *= np.sqrt(p_s / (p_n * 10 ** (snr_db / 10.0)))
    noisy = np.clip(clean + noise, -1.0, 1.0) + 1e-6 * rng.standard_normal(n)
    return clean, noisy


def make_pairs(n_pairs, seconds=10.0, sr=16000, start=0):
    return [make_pair(start + i, seconds, sr) for i in range(n_pairs)]
