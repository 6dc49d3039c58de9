"""Pair preparation: prepare_pair of
speech_enhancement_comparison.py:71-90 — mono, resample to 16 kHz, coarse
length equalisation, and alignment of the noisy signal to the clean one.

  to_mono / trim / shift     indexing on the host arrays (:14-21, :79-82, :61-69)
  alignment lag              on the device: cse_xcorr_prepare + cse_xcorr_lag,
                             the same kernels as finalize_enhanced's alignment
                             (:38-69: 2 s of signal, lags within 0.1 s)
  resampling                 the reference calls librosa.resample (soxr_hq,
                             :23-27), which is not in this image: rates other
                             than the target are converted with a polyphase
                             Kaiser FIR (scipy.signal.resample_poly).  Parity
                             unpinned for that step; the reference's committed
                             Presentation WAVs pin it loosely.
"""

from fractions import Fraction

import numpy as np

from . import _lib
from .engine import ALIGN_CORR_SAMPLES, ALIGN_MAX_LAG, ALIGN_MIN_SAMPLES, _ptr, _stream


def to_mono(x):
    """Average channels along the shorter axis (:14-21)."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        return x
    return np.mean(x, axis=1) if x.shape[0] >= x.shape[1] else np.mean(x, axis=0)


def resample_to(x, sr_in, sr_out):
    """Rate conversion (:23-27); identity when the rates match."""
    if sr_in == sr_out:
        return np.asarray(x, dtype=np.float64)
    from scipy.signal import resample_poly
    fr = Fraction(int(sr_out), int(sr_in))
    return resample_poly(np.asarray(x, dtype=np.float64), fr.numerator, fr.denominator)


def match_length(x, length):
    x = np.asarray(x, dtype=np.float64)
    if len(x) > length:
        return x[:length]
    if len(x) < length:
        return np.pad(x, (0, length - len(x)))
    return x


def shift_by_lag(sig, lag):
    """shift_by_lag (:61-69): delay by lag > 0, advance by lag < 0."""
    if lag > 0:
        return np.pad(sig, (lag, 0))
    if lag < 0:
        return sig[-lag:]
    return sig


def alignment_lag(ref, sig, sr=16000, engine=None):
    """The align_to_reference lag of ``sig`` against ``ref`` computed on the
    device (None when the reference skips alignment: fewer than 256 samples)."""
    return alignment_lag_status(ref, sig, sr, engine)[0]


def alignment_lag_status(ref, sig, sr=16000, engine=None):
    """(lag, cse_xcorr_lag status) — alignment_lag plus the status word
    (_lib.XCORR_OK, XCORR_FLAT: more than 64 near-maximal lags were
    re-evaluated in fp64, XCORR_NONFINITE: a NaN/inf in a head, lag -max_lag);
    (None, None) below 256 samples."""
    import torch
    from .engine import Engine
    eng = engine or Engine()
    ref = np.asarray(ref, dtype=np.float64)
    sig = np.asarray(sig, dtype=np.float64)
    n = int(min(len(ref), len(sig), ALIGN_CORR_SAMPLES * sr // 16000))
    if n < ALIGN_MIN_SAMPLES:
        return None, None
    max_lag = min(int(0.10 * sr), n - 1, ALIGN_MAX_LAG)
    lib, dev = eng.lib, eng.device
    c = torch.as_tensor(ref[:n]).to(dev).view(1, -1)
    head = torch.as_tensor(sig[:n].astype(np.float32)).to(dev)
    ws = torch.empty(int(lib.cse_xcorr_workspace_bytes(1, n, n, max_lag)), dtype=torch.uint8,
                     device=dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    sig_of = torch.zeros(1, dtype=torch.int32, device=dev)
    lag = torch.zeros(1, dtype=torch.int32, device=dev)
    zero = torch.zeros(1, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    st = _stream()
    _lib.check(lib.cse_xcorr_prepare(_ptr(c), 1, n, n, max_lag, _ptr(ws), st),
               "cse_xcorr_prepare")
    _lib.check(lib.cse_xcorr_lag(_ptr(head), _ptr(off), _ptr(sig_of), 1, 1, n, max_lag, _ptr(ws),
                                 _ptr(lag), _ptr(zero), _ptr(status), None, st), "cse_xcorr_lag")
    # XCORR_NONFINITE: a NaN/inf in either head; the lag is -max_lag, the
    # reference's np.argmax over its all-NaN correlation, and prepare_pair
    # shifts by it like align_to_reference does (:60-69)
    return int(lag.item()), int(status.item())


def prepare_pair(clean, sr_c, noisy, sr_n, target_sr=16000, do_align=True, engine=None):
    """(clean, noisy, target_sr) like the reference's prepare_pair (:71-90)."""
    clean = resample_to(to_mono(clean), sr_c, target_sr)
    noisy = resample_to(to_mono(noisy), sr_n, target_sr)
    n = min(len(clean), len(noisy))
    clean, noisy = clean[:n], noisy[:n]
    if do_align:
        lag = alignment_lag(clean, noisy, target_sr, engine)
        if lag is not None:
            noisy = shift_by_lag(noisy, lag)
        noisy = match_length(noisy, len(clean))
    return clean, noisy, target_sr
