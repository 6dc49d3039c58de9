"""librosa-0.11 STFT / ISTFT / fix_length restated in numpy (fp64) — oracle only.

The reference calls these with ``window="hann", center=True,
pad_mode="reflect", win_length=n_fft`` everywhere:
  stft  : spectral_subtractor.py:25, wiener_filter.py:35, mmse.py:29,
          advanced_mmse.py:39, noise_estimation.py:184-188 and :136-144
  istft : spectral_subtractor.py:55-62, wiener_filter.py:87-94,
          mmse.py:111-118, advanced_mmse.py:128-135
  fix_length : spectral_subtractor.py:41,65; advanced_mmse.py:55,136

librosa itself is not installed, so this is a restatement of its
published algorithm (librosa 0.11.0 ``core/spectrum.py``), i.e. "parity
unpinned" except for the loose end-to-end WAV fixtures.
"""

import numpy as np


def hann_periodic(n_fft):
    """scipy.signal.get_window('hann', n_fft, fftbins=True): 0.5-0.5cos(2πn/N)."""
    n = np.arange(n_fft, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * n / n_fft)


def n_frames_for(length, hop):
    """Frames of a centred STFT of an even n_fft: 1 + L // hop."""
    return 1 + int(length) // int(hop)


def _reflect_index(p, length):
    """Index map of np.pad(mode='reflect') applied repeatedly (edge excluded)."""
    if length == 1:
        return np.zeros_like(p)
    period = 2 * (length - 1)
    q = np.mod(p, period)
    return np.where(q < length, q, period - q)


def stft(y, n_fft, hop_length, win_length=None, window="hann", center=True,
         pad_mode="reflect", **_unused):
    """Complex STFT, shape (n_fft//2+1, T), fp64 in -> complex128 out."""
    if window != "hann" or not center or pad_mode != "reflect":
        raise ValueError("oracle restates only hann/center/reflect STFT")
    win_length = win_length or n_fft
    if win_length != n_fft:
        raise ValueError("oracle restates only win_length == n_fft")
    y = np.asarray(y, dtype=np.float64)
    L = y.shape[-1]
    half = n_fft // 2
    idx = _reflect_index(np.arange(-half, L + half), L)
    padded = y[idx]
    T = 1 + (padded.shape[-1] - n_fft) // hop_length
    starts = np.arange(T) * hop_length
    frames = padded[starts[:, None] + np.arange(n_fft)[None, :]]
    spec = np.fft.rfft(frames * hann_periodic(n_fft)[None, :], n=n_fft, axis=1)
    return spec.T.copy()


def window_sumsquare(n_frames, hop_length, n_fft):
    """Σ_t w²(n - t·hop) over n_frames frames, length n_fft + hop·(n_frames-1)."""
    w2 = hann_periodic(n_fft) ** 2
    out = np.zeros(n_fft + hop_length * (n_frames - 1), dtype=np.float64)
    for t in range(n_frames):
        out[t * hop_length:t * hop_length + n_fft] += w2
    return out


def istft(stft_matrix, hop_length, win_length=None, window="hann", center=True,
          length=None, **_unused):
    """Inverse STFT with librosa-0.11 semantics for a given output length.

    n_frames = min(T, ceil((length + 2*(n_fft//2)) / hop)); frames are
    irfft'd, windowed and overlap-added; the first n_fft//2 samples are dropped,
    the result is fit to ``length`` and divided by the window sum-square where
    that exceeds float64 tiny.
    """
    if window != "hann" or not center:
        raise ValueError("oracle restates only hann/center ISTFT")
    S = np.asarray(stft_matrix)
    n_fft = 2 * (S.shape[0] - 1)
    if win_length is not None and win_length != n_fft:
        raise ValueError("oracle restates only win_length == n_fft")
    half = n_fft // 2
    T = S.shape[1]
    if length is None:
        n_frames = T
        out_len = n_fft + hop_length * (n_frames - 1) - 2 * half
    else:
        n_frames = min(T, int(np.ceil((length + 2 * half) / hop_length)))
        out_len = int(length)
    w = hann_periodic(n_fft)
    frames = np.fft.irfft(S[:, :n_frames], n=n_fft, axis=0) * w[:, None]
    full = np.zeros(n_fft + hop_length * (n_frames - 1), dtype=np.float64)
    for t in range(n_frames):
        full[t * hop_length:t * hop_length + n_fft] += frames[:, t]
    wss = window_sumsquare(n_frames, hop_length, n_fft)
    y = fix_length(full[half:], size=out_len)
    wss = fix_length(wss[half:], size=out_len)
    nz = wss > np.finfo(np.float64).tiny
    y[nz] /= wss[nz]
    return y


def fix_length(data, size, axis=-1, **kwargs):
    """librosa.util.fix_length: trim, or zero-pad at the end, along ``axis``."""
    data = np.asarray(data)
    n = data.shape[axis]
    if n > size:
        sl = [slice(None)] * data.ndim
        sl[axis] = slice(0, size)
        return data[tuple(sl)]
    if n < size:
        pad = [(0, 0)] * data.ndim
        pad[axis] = (0, size - n)
        kwargs.setdefault("mode", "constant")
        return np.pad(data, pad, **kwargs)
    return data
