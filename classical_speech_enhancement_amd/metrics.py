"""Scores of the reference's sweep, on the device.

Mirrors of Code/evaluation_metrics.py:
  calculate_stoi                   :30-36   pystoi 0.4.1 stoi(..., extended=False)
                                            -> libcse.so cse_stoi_prepare / cse_stoi_cells
  calculate_snr                    :39-58
  calculate_combined_speech_score  :104-115
  calculate_pesq                   :9-27    the pesq C extension is not in this
                                            image: returns None like the
                                            reference's failure path (:25-27)
  evaluate_audio_quality           :61-101

StoiPlan is the batched form the sweep uses: the clean side (10-kHz clean,
silent-frame mask, band envelopes, segment statistics) is prepared once per
batch of equal-length signals, then any number of cell outputs are scored
against it, each shifted by its alignment lag and clipped like
finalize_enhanced (speech_enhancement_comparison.py:92-106).  The sweep runs
at the reference's working rate, 16 kHz (:381), resampled to 10 kHz inside the
cell kernel; other rates (1-768 kHz, 10 kHz unresampled) go through a generic
fp64 resampler first (cse_stoi_cells_sr).  There is no CPU fallback.
"""

import math

import numpy as np
import torch

from . import _lib
from .engine import _ptr, _stream

STOI_SR = 16000
# cells per cse_stoi_cells launch: bounds the envelope scratch (Mmax x 64 B per cell)
STOI_CHUNK = 16384


_GPU = None


def _gpu_visible():
    global _GPU
    if _GPU is None:
        _GPU = bool(torch.cuda.is_available())
    return _GPU


class StoiPlan:
    """Clean side of STOI for S equal-length signals (clean: [S, L] f64 cuda)."""

    def __init__(self, clean, sr=STOI_SR):
        if not _gpu_visible():
            raise _lib.CseError("no GPU visible: the HIP engine has no CPU fallback")
        self.lib = _lib.load()
        clean = clean.contiguous()
        if clean.dtype != torch.float64 or clean.dim() != 2 or not clean.is_cuda:
            raise ValueError("clean must be a [S, L] float64 cuda tensor")
        self.S, self.L = clean.shape
        self.clean = clean
        self.sr = int(sr)
        nbytes = int(self.lib.cse_stoi_workspace_bytes_sr(self.S, self.L, self.sr))
        if nbytes < 0:
            raise NotImplementedError(f"STOI: sample rate {sr} not supported (1000-768000 Hz)")
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=clean.device)
        _lib.check(self.lib.cse_stoi_prepare(_ptr(clean), self.S, self.L, sr, _ptr(self.ws),
                                             _stream()), "cse_stoi_prepare")
        self._scratch = None

    def _scratch_for(self, n):
        nbytes = max(int(self.lib.cse_stoi_scratch_bytes_sr(n, self.L, self.sr)), 1)
        if self._scratch is None or self._scratch.numel() < nbytes:
            self._scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.clean.device)
        return self._scratch

    def score_async(self, y, y_offset, sig_of, lag=None, clip=True, out=None):
        """Enqueue the STOI of every cell; returns the [n] f64 cuda result.

        y: flat f32 cuda tensor holding every cell's output (>= L samples from
        y_offset[c]); sig_of: clean signal of each cell; lag: alignment lag
        (None = 0).  The test signal of cell c is y[n - lag] (zero outside
        [0, L)), clipped to [-1, 1] when clip.  y_offset / sig_of / lag given
        as host arrays are validated here and uploaded on the current stream;
        given as cuda tensors (int64 / int32 / int32) they are taken as they
        are, with no host synchronisation (the caller validated them)."""
        dev = self.clean.device
        if y.dtype != torch.float32 or not y.is_cuda:
            raise ValueError("y must be a float32 cuda tensor")
        if torch.is_tensor(y_offset):
            # device indices: every check that needs no host synchronisation
            # (the value ranges are the caller's; the kernel reads int64 / int32)
            off, sig = y_offset, sig_of
            if not torch.is_tensor(sig):
                raise ValueError("sig_of must be a cuda tensor when y_offset is one")
            if off.dtype != torch.int64 or sig.dtype != torch.int32:
                raise ValueError("device y_offset / sig_of must be int64 / int32")
            if off.device != dev or sig.device != dev:
                raise ValueError("device y_offset / sig_of must live on the clean signal's GPU")
            if not (off.is_contiguous() and sig.is_contiguous()):
                raise ValueError("device y_offset / sig_of must be contiguous")
            n = int(off.numel())
            if int(sig.numel()) != n:
                raise ValueError("y_offset and sig_of differ in length")
            if torch.is_tensor(lag) and (lag.dtype != torch.int32 or lag.device != dev
                                         or not lag.is_contiguous() or int(lag.numel()) != n):
                raise ValueError("device lag must be a contiguous int32 tensor of n entries "
                                 "on the clean signal's GPU")
        else:
            off_h = np.asarray(y_offset, dtype=np.int64)
            sig_h = np.asarray(sig_of, dtype=np.int32)
            n = len(off_h)
            if len(sig_h) != n:
                raise ValueError("y_offset and sig_of differ in length")
            if n and (int(sig_h.min()) < 0 or int(sig_h.max()) >= self.S):
                raise ValueError("sig_of out of range")
            if n and (int(off_h.min()) < 0 or int(off_h.max()) + self.L > y.numel()):
                raise ValueError("a cell's output runs past the end of y")
            off = torch.as_tensor(off_h, device=dev)
            sig = torch.as_tensor(sig_h, device=dev)
        lg = None
        if lag is not None:
            if torch.is_tensor(lag):
                lg = lag.to(dev, torch.int32).contiguous()
            else:
                lag_h = np.asarray(lag, dtype=np.int32)
                if len(lag_h) != n:
                    raise ValueError("lag and y_offset differ in length")
                lg = torch.as_tensor(lag_h, device=dev)
            if int(lg.numel()) != n:
                raise ValueError("lag and y_offset differ in length")
        if out is None:
            out = torch.empty(n, dtype=torch.float64, device=dev)
        for s in range(0, n, STOI_CHUNK):
            m = min(STOI_CHUNK, n - s)
            scratch = self._scratch_for(m)
            args = (_ptr(y), _ptr(off[s:]), None if lg is None else _ptr(lg[s:]), _ptr(sig[s:]),
                    m, self.S, self.L)
            tail = (1 if clip else 0, _ptr(self.ws), _ptr(scratch), _ptr(out[s:]), _stream())
            if self.sr == STOI_SR:
                _lib.check(self.lib.cse_stoi_cells(*args, *tail), "cse_stoi_cells")
            else:
                _lib.check(self.lib.cse_stoi_cells_sr(*args, self.sr, *tail), "cse_stoi_cells_sr")
        return out

    def score(self, y, y_offset, sig_of, lag=None, clip=True):
        """score_async, synchronised; NaN entries are pystoi failures (None)."""
        return self.score_async(y, y_offset, sig_of, lag, clip).cpu().numpy()


def stoi(x, y, fs_sig):
    """pystoi ``stoi(x, y, fs_sig, extended=False)`` on the device."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    if x.shape != y.shape:
        raise Exception(f"x and y should have the same length, found {x.shape} and {y.shape}")
    if x.ndim != 1 or x.size == 0:
        raise ValueError("stoi expects non-empty 1-D signals")
    plan = StoiPlan(torch.as_tensor(x).cuda().view(1, -1), fs_sig)
    yd = torch.as_tensor(y.astype(np.float32)).cuda()
    v = float(plan.score(yd, [0], [0], clip=False)[0])
    if math.isnan(v):
        raise ValueError("no 256-sample frame at 10 kHz")  # pystoi: empty frame array
    return v


def calculate_stoi(clean_reference, test_audio, sr):
    """evaluation_metrics.calculate_stoi (:30-36): trim to the common length,
    None on failure."""
    try:
        n = min(len(clean_reference), len(test_audio))
        return stoi(np.asarray(clean_reference)[:n], np.asarray(test_audio)[:n], sr)
    except (NotImplementedError, _lib.CseError):
        raise  # no device / unsupported: not a score failure
    except Exception as e:  # the reference's catch-all
        print(f"STOI calculation failed: {e}")
        return None


def calculate_pesq(clean_reference, test_audio, sr):
    """evaluation_metrics.calculate_pesq (:9-27).  The ITU-T P.862 `pesq`
    extension is not available in this image; like the reference when the
    call fails, report and return None."""
    print("PESQ calculation failed: the pesq extension is not available")
    return None


def calculate_snr(clean, processed):
    """evaluation_metrics.calculate_snr (:39-58)."""
    try:
        clean = np.asarray(clean)
        processed = np.asarray(processed)
        m = min(len(clean), len(processed))
        clean, processed = clean[:m], processed[:m]
        noise = clean - processed
        p_signal = np.sum(clean ** 2)
        p_noise = np.sum(noise ** 2)
        if p_noise == 0:
            return float("inf")
        return float(10 * np.log10(p_signal / (p_noise + 1e-10)))
    except Exception as e:
        print(f"SNR calculation failed: {e}")
        return None


def calculate_combined_speech_score(stoi_score, pesq_score):
    """evaluation_metrics.calculate_combined_speech_score (:104-115)."""
    if stoi_score is None:
        stoi_score = 0
    if pesq_score is None:
        pesq_score = 0
    return 0.5 * stoi_score + 0.5 * (max(0, pesq_score) / 4.5)


def evaluate_audio_quality(clean_reference, noisy_audio, enhanced_audio, sr, algorithm_name=""):
    """evaluation_metrics.evaluate_audio_quality (:61-101), same keys."""
    results = {}
    s_noisy = calculate_stoi(clean_reference, noisy_audio, sr)
    s_enh = calculate_stoi(clean_reference, enhanced_audio, sr)
    if s_noisy is not None and s_enh is not None:
        results["stoi_noisy"] = s_noisy
        results["stoi_enhanced"] = s_enh
        results["stoi_improvement"] = s_enh - s_noisy
    p_noisy = calculate_pesq(clean_reference, noisy_audio, sr)
    p_enh = calculate_pesq(clean_reference, enhanced_audio, sr)
    if p_noisy is not None and p_enh is not None:
        results["pesq_noisy"] = p_noisy
        results["pesq_enhanced"] = p_enh
        results["pesq_improvement"] = p_enh - p_noisy
    snr_val = calculate_snr(clean_reference, enhanced_audio)
    if snr_val is not None:
        results["snr_enhanced"] = snr_val
    if algorithm_name:
        print(f"\n{'=' * 60}\nEvaluation: {algorithm_name}\n{'=' * 60}")
    if "stoi_noisy" in results:
        print(f"STOI: {results['stoi_noisy']:.4f} -> {results['stoi_enhanced']:.4f} "
              f"(+{results['stoi_improvement']:.4f})")
    if "snr_enhanced" in results:
        print(f"SNR (Enhanced): {results['snr_enhanced']:.2f} dB")
    return results
