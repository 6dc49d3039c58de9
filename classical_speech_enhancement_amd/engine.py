"""Device orchestration of the STFT frame-gain path on MI355X.

PyTorch-ROCm is used only as the device-memory container and stream provider;
every numeric step is a libcse.so kernel (include/cse.h):

  cse_stft            STFT of every signal at each (n_fft, hop)        [once per group]
  cse_noise_estimate  percentile / min-tracking / true-noise PSDs     [once per group]
  cse_noise_smooth    MMSE/OMLSA noise IIR (per noise_mu)             [once per group]
  cse_enhance_cells   THE HOT PATH: gain recursion + ISTFT + SNR sums [per grid cell]

A "cell spec" is (signal index, algorithm name, params dict) where params are
the reference plugin's keyword arguments (parameter_ranges.py keys).
"""

import ctypes
import os
import math
from collections import OrderedDict

import numpy as np
import torch

from . import _lib

# algorithm name (registry names of speech_enhancement_comparison.py:395-401)
# -> (code, eps the reference passes to noise_estimation, param order in cse_cell_t)
ALGOS = {
    "spectralSubtractor": ("SS", 1e-10, ("alpha", "beta")),
    "wiener": ("WIENER", 1e-10, ("alpha", "gain_floor")),
    "mmse": ("MMSE", 1e-12, ("alpha", "ksi_min", "gain_min", "gain_max")),
    "omlsa": ("OMLSA", 1e-10, ("alpha", "ksi_min", "gain_floor", "q", "v_max")),
}
ALIASES = {"ss": "spectralSubtractor", "spectral_subtraction": "spectralSubtractor",
           "wiener_filter": "wiener", "advanced_mmse": "omlsa"}
DEFAULTS = {"mmse": {"noise_mu": 0.98, "gain_max": 1.0}, "omlsa": {"v_max": 80.0}}
# finalize_enhanced alignment (speech_enhancement_comparison.py:38-69) at 16 kHz:
# correlate the first corr_seconds = 2 s, lags within max_shift_s = 0.1 s,
# no alignment below 256 samples
ALIGN_CORR_SAMPLES = 32000
ALIGN_MAX_LAG = 1600
ALIGN_MIN_SAMPLES = 256
# relative per-bin cost used to order waves (longest first)
ALGO_COST = {"SS": 1.0, "WIENER": 1.1, "MMSE": 2.0, "OMLSA": 3.0}


def canonical_algo(name):
    name = ALIASES.get(name, name)
    if name not in ALGOS:
        raise ValueError(f"unknown algorithm {name!r}")
    return name


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _at(t, k):
    """Pointer to element k of a device tensor (None stays None)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr() + k * t.element_size())


# hops of the sweep kernels (cse_enhance_cells) and the short hops of
# cse_enhance_cells_short_hop, per n_fft; every other even n_fft in
# [64, 4096] and hop in [1, n_fft] goes to cse_enhance_cells_generic
HOPS = (128, 256)
SHORT_HOPS = {512: (32, 64), 1024: (64,)}
MAIN, SHORT, GENERIC = 0, 1, 2


def route(n_fft, hop):
    """Which enhance kernel runs (n_fft, hop): MAIN, SHORT, GENERIC, or None
    (not supported)."""
    n_fft, hop = int(n_fft), int(hop)
    if n_fft in (512, 1024) and hop in HOPS:
        return MAIN
    if hop in SHORT_HOPS.get(n_fft, ()):
        return SHORT
    if 64 <= n_fft <= 4096 and n_fft % 2 == 0 and 1 <= hop <= n_fft:
        return GENERIC
    return None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def n_frames(length, hop):
    return 1 + int(length) // int(hop)


def noise_key(alg, params, T):
    """Which noise PSD array a cell reads, mirroring each algorithm's pipeline.

    Returns (method, pct, eps, expand, mu, inverse):
      - every algorithm estimates with the eps it passes (ss/wiener/omlsa 1e-10,
        mmse 1e-12: spectral_subtractor.py:17, wiener_filter.py:23, mmse.py:17,
        advanced_mmse.py:26);
      - T < 5 -> the static 'simple' estimate for ANY method
        (noise_estimation.py:194-195, before the method is even looked at);
      - expand: SS and OMLSA pass a static (B,1) estimate through
        librosa.util.fix_length(..., size=T, axis=1) (spectral_subtractor.py:40-41,
        advanced_mmse.py:54-55), which ZERO-PADS frames 1..T-1 — frame 0 sees
        the estimate, later frames see 0 (SS) or, after OMLSA's smoothing,
        mu**t times it;
      - mmse/omlsa smooth any time-varying estimate except true_noise
        (mmse.py:48-54, advanced_mmse.py:60-66); mu=None means no smoothing;
      - inverse: Wiener/MMSE/OMLSA read 1/max(N, eps) (their in-loop floor,
        wiener_filter.py:58, mmse.py:71, advanced_mmse.py:87), SS reads N.
    A key is static (one [B] row for all frames) iff expand is False and the
    method is percentile/simple.
    """
    code, eps, _ = ALGOS[alg]
    method = params["noise_method"]
    if T < 5:
        method, pct = "simple", None
    elif method == "percentile":
        pct = float(params["noise_percentile"])
    elif method in ("min_tracking", "true_noise"):
        pct = None
    else:
        raise ValueError(f"Unbekannte Methode: {method}")
    static = method in ("percentile", "simple")
    expand = static and T > 1 and code in ("SS", "OMLSA")
    mu = None
    if method != "true_noise" and (expand or not static):
        if code == "MMSE":
            mu = float(params.get("noise_mu", 0.98))
        elif code == "OMLSA":
            mu = float(params["noise_mu"])
    return (method, pct, eps, expand, mu, code != "SS")


NOISE_PARAM_KEYS = ("percentile", "min_frames", "max_fraction", "floor_rel", "adaptive_short",
                    "window_size", "smoothing_factor")


def noise_params(percentile=20.0, min_frames=10, max_fraction=0.30, floor_rel=0.02,
                 adaptive_short=True, window_size=50, smoothing_factor=None, src_frames=0):
    """cse_noise_params_t from the reference's estimator constructor arguments
    (PercentileNoiseEstimator noise_estimation.py:12-13, MinTrackingNoiseEstimator
    :60; defaults as there).  smoothing_factor None -> NaN."""
    prm = _lib.NoiseParams()
    prm.percentile = float(percentile)
    prm.max_fraction = float(max_fraction)
    prm.floor_rel = float(floor_rel)
    prm.smoothing_factor = math.nan if smoothing_factor is None else float(smoothing_factor)
    prm.min_frames = int(min_frames)
    prm.adaptive_short = 1 if adaptive_short else 0
    prm.window_size = int(window_size)
    prm.src_frames = int(src_frames)
    return prm


def key_is_static(key):
    method, _, _, expand, mu, _ = key
    return method in ("percentile", "simple") and not expand and mu is None


class Engine:
    """Runs batches of grid cells over batches of equal-length signals."""

    def __init__(self, device="cuda"):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.CseError("no GPU visible: the HIP engine has no CPU fallback")
        self.device = torch.device(device)
        # key -> ((specs, keep), MultiPlan), most recent last: see run(reuse=...)
        self._plan_cache = OrderedDict()
        self.plan_cache_size = 1
        self._side = None

    # ------------------------------------------------------------------ prep
    def stft(self, x, n_fft, hop, x_sub=None, want_y=True, want_p=True):
        """x: [S, L] float64 cuda -> (Y [S,T,B,2] f32, P [S,T,B] f64)."""
        S, L = x.shape
        T, B = n_frames(L, hop), n_fft // 2 + 1
        Y = torch.empty((S, T, B, 2), dtype=torch.float32, device=x.device) if want_y else None
        P = torch.empty((S, T, B), dtype=torch.float64, device=x.device) if want_p else None
        _lib.check(self.lib.cse_stft(_ptr(x), _ptr(x_sub), S, L, n_fft, hop, _ptr(Y), _ptr(P),
                                     _stream()), "cse_stft")
        return Y, P

    def noise_estimate(self, method, P, percentile=20.0, eps=1e-10, out=None, frames=None,
                       **params):
        """cse_noise_estimate_ex on P [S, T', B] f64.  params: estimator
        constructor parameters (min_frames, max_fraction, floor_rel,
        adaptive_short, window_size, smoothing_factor; noise_estimation.py:12-13,
        :60).  true_noise: P is the power of STFT(noisy - clean) over the
        shorter length, fit to ``frames`` (default T') frames (:149-153)."""
        S, Tp, B = P.shape
        T = Tp if frames is None else int(frames)
        code = {"percentile": 0, "min_tracking": 1, "true_noise": 2, "simple": 0}[method]
        static = method == "percentile" or (T < 5 and method != "true_noise")
        shape = (S, B) if (static and method != "min_tracking") else (S, T, B)
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=P.device)
        ws = torch.empty(int(self.lib.cse_noise_workspace_bytes(S, T, B)), dtype=torch.uint8,
                         device=P.device)
        prm = noise_params(percentile=percentile, src_frames=Tp if code == 2 else 0, **params)
        if code != 2 and Tp != T:
            raise ValueError("frames applies to true_noise only")
        _lib.check(self.lib.cse_noise_estimate_ex(code, _ptr(P), S, T, B, ctypes.byref(prm),
                                                  float(eps), _ptr(out), _ptr(ws), _stream()),
                   f"cse_noise_estimate({method})")
        return out

    def noise_smooth(self, N, T, mu, out=None):
        """[S,T,B] (or static [S,B], zero-padded to T frames) -> smoothed [S,T,B]."""
        S, B = N.shape[0], N.shape[-1]
        src_frames = 1 if N.dim() == 2 else N.shape[1]
        if out is None:
            out = torch.empty((S, T, B), dtype=torch.float32, device=N.device)
        _lib.check(self.lib.cse_noise_smooth(_ptr(N), S, T, B, src_frames, float(mu), _ptr(out),
                                             _stream()), "cse_noise_smooth")
        return out

    def istft_norm(self, n_fft, hop, length):
        out = torch.empty(int(length), dtype=torch.float32, device=self.device)
        _lib.check(self.lib.cse_istft_norm(n_fft, hop, int(length), _ptr(out), _stream()),
                   "cse_istft_norm")
        return out

    # ------------------------------------------------------------------ grid
    def plan(self, n_signals, length, specs, with_clean=True, want_waveforms=False,
             want_gains=False, align=False, true_len=None):
        """Build one GridPlan per n_fft for these specs (see GridPlan)."""
        return MultiPlan(self, n_signals, length, specs, with_clean, want_waveforms, want_gains,
                         align, true_len)

    def side_stream(self):
        """A second stream of this engine, kept for its lifetime (work queued
        on it reuses the caching allocator's blocks of earlier calls)."""
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def run(self, noisy, specs, clean=None, want_waveforms=False, want_gains=False, align=False,
            true_len=None, reuse=None, keep=None, on_plan=None):
        """Enhance every cell spec; returns a dict of per-spec results.

        noisy/clean: [S, L] float64 cuda tensors (clean may be None if no spec
        uses true_noise and no SNR is wanted).  specs: list of
        (signal_index, algorithm_name, params).  Results (spec order):
          sse [n] f64 numpy, finite [n] bool numpy, and optionally
          'y' [n, L] f32 cuda and 'G' list of [T, B] f32 cuda.
        true_len: TrueNoise estimates use the first true_len samples of noisy
        and clean (a clean reference shorter than the noisy signal,
        noise_estimation.py:128-130); default L.
        reuse: keep the plan (device buffers, cell tables) for a later call
        with the same structure (the plan_cache_size most recent ones).  True: the structure is spec_fingerprint(specs)
        — per cell the signal index, algorithm and params object identity (the
        cached specs keep the params alive; they must not be mutated in
        between).  Or a hashable key the caller derived from the structure;
        specs may then be a zero-argument callable that builds the list, called
        only when the key misses, and ``keep`` is held with the plan (the
        object the key's identities refer to).  The results' 'y' is the plan's
        buffer: the next reusing call overwrites it.
        on_plan: see MultiPlan.execute.
        """
        S, L = noisy.shape
        flags = (S, L, clean is not None, want_waveforms, want_gains, align, true_len)
        mp, key = None, None
        if reuse is not None and reuse is not False:
            if reuse is True:
                specs = specs() if callable(specs) else specs
                reuse = spec_fingerprint(specs)
            key = flags + (reuse,)
            hit = self._plan_cache.get(key)
            if hit is not None:
                mp = hit[1]
                self._plan_cache.move_to_end(key)
        if mp is None:
            specs = specs() if callable(specs) else specs
            if key is not None:  # evict before allocating the new plan's buffers
                while len(self._plan_cache) >= max(self.plan_cache_size, 1):
                    self._plan_cache.popitem(last=False)
            mp = self.plan(S, L, specs, clean is not None, want_waveforms, want_gains, align,
                           true_len)
            if key is not None:
                self._plan_cache[key] = ((specs, keep), mp)
        mp.execute(noisy, clean, on_plan)
        return mp.results()


class GridPlan:
    """Everything one n_fft's cells need, allocated once; execute() only enqueues.

    Buffers (device, resident in HBM across steps):
      Y      [hop][S][T][B] complex64        cse_stft
      P      [S][T][B] f64 per hop           cse_stft (analysis power)
      pool   flat f32: every noise PSD the cells read, at per-key offsets
      cells  packed cse_cell_t table (wave slots, longest-first)
      sse/finite per packed cell; optional y_out / g_out
    execute() issues only kernel launches on the current stream (no host
    sync, no allocation), so it can be timed or captured as a graph.
    """

    def __init__(self, eng, n_fft, S, L, items, with_clean, want_y, want_g, y_all=None,
                 align=False, true_len=None):
        # the library and device only, not the Engine: the engine's plan cache
        # holds this plan, and a back reference would make the pair a cycle
        # that only the cyclic collector frees (with the plan's device buffers)
        self.lib, self.device = eng.lib, eng.device
        self.n_fft, self.S, self.L = n_fft, S, L
        self.true_len = L if true_len is None else int(true_len)
        if not 1 <= self.true_len <= L:
            raise ValueError(f"true_len={self.true_len} not in [1, {L}]")
        self.items = items
        dev = eng.device
        B = self.B = n_fft // 2 + 1
        self.hops = sorted({p["hop_length"] for (_, _, _, p) in items})
        self.y_base, off = {}, 0
        for hop in self.hops:
            self.y_base[hop] = off
            off += S * n_frames(L, hop) * B
        self.Ybuf = torch.empty(off * 2, dtype=torch.float32, device=dev)
        self.P = {h: torch.empty((S, n_frames(L, h), B), dtype=torch.float64, device=dev)
                  for h in self.hops}
        self.Ptrue = {}
        # ---- noise keys -> pool slices.  Each key = a base estimate (method,
        # pct, eps) post-processed by one cse_noise_finish job (smoothing,
        # fix_length zero-padding, 1/max(.,eps)); base estimates are shared.
        # noise key of every item, computed once per distinct
        # (algorithm, hop, method, percentile, noise_mu)
        keys, key_cache = {}, {}
        item_key = []
        for (_, _, alg, p) in items:
            hop = p["hop_length"]
            ck = (alg, hop, p["noise_method"], p.get("noise_percentile"), p.get("noise_mu"))
            k = key_cache.get(ck)
            if k is None:
                k = key_cache[ck] = (hop, noise_key(alg, p, n_frames(L, hop)))
                keys.setdefault(k, None)
            item_key.append(k)
        # jobs grouped by hop: each hop's rows are finished by one
        # cse_noise_finish launch right after that hop's own estimates (all on
        # one stream, so in order; grouping by hop makes each launch's job list
        # one contiguous slice)
        self.keys = sorted(keys, key=lambda k: k[0])
        self.pool_off, noff = {}, 0
        self.raw_off, roff = {}, 0
        jobs = []
        for (hop, key) in self.keys:
            T = n_frames(L, hop)
            method, pct, eps, expand, mu, inverse = key
            static = key_is_static(key)
            per_sig = B if static else T * B
            self.pool_off[(hop, key)] = (noff, 0 if static else B, per_sig)
            base = (hop, method, pct, eps)
            if base not in self.raw_off:
                src_static = method in ("percentile", "simple")
                self.raw_off[base] = (roff, 1 if src_static else T)
                roff += S * (B if src_static else T * B)
            r0, src_frames = self.raw_off[base]
            jobs.append((r0, noff, src_frames, 1 if static else T, float(mu or 0.0),
                         float(eps) if inverse else 0.0))
            noff += S * per_sig
            if method == "true_noise" and hop not in self.Ptrue:
                if not with_clean:
                    raise ValueError("TrueNoiseEstimator requires clean_audio and noisy_audio")
                self.Ptrue[hop] = torch.empty((S, n_frames(self.true_len, hop), B),
                                              dtype=torch.float64, device=dev)
        self.pool = torch.empty(noff, dtype=torch.float32, device=dev)
        self.raw = torch.empty(max(roff, 1), dtype=torch.float32, device=dev)
        jt = np.zeros(len(jobs), dtype=_lib.NOISE_JOB_DTYPE)
        for j, (so, do, sf, of, mu, ie) in enumerate(jobs):
            jt[j] = (so, do, sf, of, mu, ie)
        self.n_jobs = len(jobs)
        self.jobs_d = torch.from_numpy(jt.view(np.uint8).copy()).to(dev)
        self.hop_jobs = {}  # hop -> (first job, count)
        for j, (hop, _) in enumerate(self.keys):
            first, cnt = self.hop_jobs.get(hop, (j, 0))
            self.hop_jobs[hop] = (first, cnt + 1)
        self.med = torch.empty((S, B), dtype=torch.float64, device=dev)
        Tmax = max(n_frames(L, h) for h in self.hops)
        self.ws = torch.empty(int(eng.lib.cse_noise_workspace_bytes(S, Tmax, B)),
                              dtype=torch.uint8, device=dev)
        # ---- cell table (columns gathered once, written as arrays)
        n = len(items)
        cells = np.zeros(n, dtype=_lib.CELL_DTYPE)
        self.idx = np.fromiter((it[0] for it in items), dtype=np.int64, count=n)
        sig = np.fromiter((it[1] for it in items), dtype=np.int64, count=n)
        hop = np.fromiter((it[3]["hop_length"] for it in items), dtype=np.int64, count=n)
        algo = np.fromiter((_lib.ALGO[ALGOS[it[2]][0]] for it in items), dtype=np.int32, count=n)
        kinfo = np.array([self.pool_off[k] for k in item_key], dtype=np.int64).reshape(n, 3)
        T = 1 + L // hop
        ybase = np.zeros(n, dtype=np.int64)
        for h in self.hops:
            ybase[hop == h] = self.y_base[h]
        cells["algo"] = algo
        cells["hop"] = hop
        cells["y_offset"] = ybase + sig * T * B
        cells["noise_offset"] = kinfo[:, 0] + sig * kinfo[:, 2]
        cells["noise_stride"] = kinfo[:, 1]
        cells["clean_offset"] = sig * L if with_clean else -1
        cells["out_offset"] = self.idx * L if want_y else -1
        goff = (np.concatenate([[0], np.cumsum(T * B)[:-1]]) if want_g
                else np.zeros(n, dtype=np.int64))
        cells["gain_offset"] = goff if want_g else -1
        self.g_offsets = list(zip(goff.tolist(), T.tolist()))
        g_total = int((T * B).sum()) if want_g else 0
        prm = np.zeros((n, 8), dtype=np.float32)
        for c, (_, _, alg, p) in enumerate(items):
            names = ALGOS[alg][2]
            dflt = DEFAULTS.get(alg, {})
            prm[c, :len(names)] = [p[k] if k in p else dflt[k] for k in names]
        cells["param"] = prm
        self.cells = cells
        packed, self.order = pack_waves(cells, n_fft)
        self.n_packed = len(packed)
        self.split = route_slots(packed, n_fft)
        self.cells_d = torch.from_numpy(packed.view(np.uint8).copy()).to(dev)
        self.g_out = torch.zeros(max(g_total, 1), dtype=torch.float32, device=dev) if want_g else None
        self.y_all = y_all
        self.sse_d = torch.zeros(self.n_packed, dtype=torch.float64, device=dev)
        self.fin_d = torch.zeros(self.n_packed, dtype=torch.uint8, device=dev)
        self.clean = None
        self.with_clean = with_clean
        # frame-gain evaluations (SURVEY §8(d) unit): sum over cells of frames
        self.units = int(T.sum())
        # ---- finalize_enhanced alignment (speech_enhancement_comparison.py:38-69)
        self.rerun = None
        self.xc_n = min(L, ALIGN_CORR_SAMPLES)
        self.align = bool(align) and with_clean and self.xc_n >= ALIGN_MIN_SAMPLES
        if self.align:
            self.xc_lag_max = min(ALIGN_MAX_LAG, self.xc_n - 1)
            if y_all is not None:   # whole waveforms requested: their heads are the input
                self.head = y_all
                head_off = self.cells["out_offset"].astype(np.int64)
            else:
                self.head = torch.empty(len(items) * self.xc_n, dtype=torch.float32, device=dev)
                head_off = np.arange(len(items), dtype=np.int64) * self.xc_n
                self.cells["out_offset"] = head_off
                packed, _ = pack_waves(self.cells, n_fft)
                assert route_slots(packed, n_fft) == self.split
                self.cells_d = torch.from_numpy(packed.view(np.uint8).copy()).to(dev)
            self.head_off = torch.as_tensor(head_off, device=dev)
            self.sig_of = torch.as_tensor(sig.astype(np.int32), device=dev)
            self.xc_ws = torch.empty(int(eng.lib.cse_xcorr_workspace_bytes(
                S, L, self.xc_n, self.xc_lag_max)), dtype=torch.uint8, device=dev)
            self.lag_d = torch.zeros(len(items), dtype=torch.int32, device=dev)
            self.zero_d = torch.zeros(len(items), dtype=torch.float64, device=dev)
            self.xst_d = torch.zeros(len(items), dtype=torch.int32, device=dev)

    def prepare(self, noisy, clean=None):
        """Group-level analysis: STFTs and every noise row (once per signal batch)."""
        self.prepare_stft(noisy, clean)
        self.prepare_noise(clean)

    # The analysis in two phases: every hop's STFT first, then the noise chains.
    # The STFT (80 KB of LDS per workgroup) cannot take the slot of one finished
    # enhance workgroup, so on a side stream under an enhance launch it waits
    # for the launch's drain, while the noise kernels fit freed slots.  With
    # the STFTs adjacent (TimedJob.prep: of every plan), one drain runs them all
    # and the chains follow inside the next launch; interleaved (STFT, chain,
    # STFT, chain) each STFT waited for a drain of its own and the next launch
    # for the last chain (r05: 168.6 -> 168.2 ms/step at 100 pairs).
    def prepare_stft(self, noisy, clean=None):
        S, L, B = self.S, self.L, self.B
        lib = self.lib
        st = _stream()
        for hop in self.hops:
            T = n_frames(L, hop)
            yv = self.Ybuf[2 * self.y_base[hop]:2 * (self.y_base[hop] + S * T * B)]
            _lib.check(lib.cse_stft(_ptr(noisy), None, S, L, self.n_fft, hop, _ptr(yv),
                                    _ptr(self.P[hop]), st), "cse_stft")
            if hop in self.Ptrue:
                m = self.true_len
                xn, xc = noisy, clean
                if m < L:  # the STFT of the trimmed difference (noise_estimation.py:128-133)
                    xn, xc = noisy[:, :m].contiguous(), clean[:, :m].contiguous()
                _lib.check(lib.cse_stft(_ptr(xn), _ptr(xc), S, m, self.n_fft, hop, None,
                                        _ptr(self.Ptrue[hop]), st), "cse_stft(true)")

    def prepare_noise(self, clean=None):
        S, L, B = self.S, self.L, self.B
        lib = self.lib
        st = _stream()
        for hop in self.hops:
            T = n_frames(L, hop)
            bases = [b for b in self.raw_off if b[0] == hop]
            P = self.P[hop]

            def raw(b):
                o, frames = self.raw_off[b]
                return self.raw[o:o + S * frames * B]
            if T >= 5 and any(m in ("percentile", "min_tracking") for (_, m, _, _) in bases):
                _lib.check(lib.cse_noise_median(_ptr(P), S, T, B, _ptr(self.med), st),
                           "cse_noise_median")
            mt = [b for b in bases if b[1] == "min_tracking"]
            for k in range(0, len(mt), 2):  # two eps per IIR + min-filter pass
                a_, b_ = mt[k], (mt[k + 1] if k + 1 < len(mt) else None)
                _lib.check(lib.cse_noise_min_tracking_med(
                    _ptr(P), _ptr(self.med), S, T, B, float(a_[3]), _ptr(raw(a_)),
                    float(b_[3]) if b_ else 0.0, _ptr(raw(b_)) if b_ else None, _ptr(self.ws),
                    st), "cse_noise_min_tracking_med")
            # percentile estimates in pairs sharing eps: one frame-energy pass per pair
            pc = {}
            for b in bases:
                if b[1] == "percentile":
                    pc.setdefault(float(b[3]), []).append(b)
            quad = sorted(pc) if len(pc) == 2 and not os.environ.get("CSE_NO_QUAD") else None
            if quad and all(len(pc[e]) == 2 for e in quad) and \
                    sorted(b[2] for b in pc[quad[0]]) == sorted(b[2] for b in pc[quad[1]]):
                # the HEAD grid's case: two percentiles x two eps, four launches
                # (cse_noise_percentile_quad) instead of ten
                pa, pb = sorted(float(b[2]) for b in pc[quad[0]])
                by = {(float(b[2]), float(b[3])): b for e in quad for b in pc[e]}
                _lib.check(lib.cse_noise_percentile_quad(
                    _ptr(P), _ptr(self.med), S, T, B, pa, pb, quad[0], quad[1],
                    _ptr(raw(by[(pa, quad[0])])), _ptr(raw(by[(pa, quad[1])])),
                    _ptr(raw(by[(pb, quad[0])])), _ptr(raw(by[(pb, quad[1])])), _ptr(self.ws), st),
                    "cse_noise_percentile_quad")
                pc = {}
            for eps, group in pc.items():
                for k in range(0, len(group), 2):
                    a_, b_ = group[k], (group[k + 1] if k + 1 < len(group) else None)
                    _lib.check(lib.cse_noise_percentile_med2(
                        _ptr(P), _ptr(self.med), S, T, B, float(a_[2]),
                        float(b_[2]) if b_ else 0.0, eps, _ptr(raw(a_)),
                        _ptr(raw(b_)) if b_ else None, _ptr(self.ws), st),
                        "cse_noise_percentile_med2")
            for b in bases:
                _, method, pct, eps = b
                if method == "percentile":
                    continue
                elif method == "simple":
                    _lib.check(lib.cse_noise_estimate(0, _ptr(P), S, T, B, 25.0, float(eps),
                                                      _ptr(raw(b)), _ptr(self.ws), st),
                               "cse_noise_estimate(simple)")
                elif method == "true_noise":
                    prm = noise_params(src_frames=self.Ptrue[hop].shape[1])
                    _lib.check(lib.cse_noise_estimate_ex(2, _ptr(self.Ptrue[hop]), S, T, B,
                                                         ctypes.byref(prm), float(eps),
                                                         _ptr(raw(b)), None, st),
                               "cse_noise_estimate(true)")
            j0, nj = self.hop_jobs[hop]
            jobs = ctypes.c_void_p(self.jobs_d.data_ptr() + j0 * _lib.NOISE_JOB_DTYPE.itemsize)
            _lib.check(lib.cse_noise_finish(jobs, nj, S, B, _ptr(self.raw), _ptr(self.pool), st),
                       "cse_noise_finish")
        self.clean = clean if self.with_clean else None

    def enhance(self):
        """THE HOT PATH launch: every cell of this n_fft, one kernel."""
        if self.y_all is not None:
            yo, olen = self.y_all, self.L
        elif self.align:
            yo, olen = self.head, self.xc_n
        else:
            yo, olen = None, 0
        self.launch(self.cells_d, self.split, yo, olen, self.g_out, self.sse_d, self.fin_d,
                    _stream(), "cse_enhance_cells")

    def launch(self, cells_d, split, yo, olen, g, sse, fin, st, what):
        """The enhance launches over packed cells, split = (main, short,
        generic) slot counts in that order (pack_waves): the sweep hops
        (cse_enhance_cells, one kernel), the short hops
        (cse_enhance_cells_short_hop), every other shape
        (cse_enhance_cells_generic)."""
        args = (_ptr(self.Ybuf), _ptr(self.pool), _ptr(self.clean), _ptr(yo), olen)
        n_main, n_short, n_gen = split
        k = _lib.CELL_DTYPE.itemsize
        if n_main:
            _lib.check(self.lib.cse_enhance_cells(self.n_fft, self.L, _ptr(cells_d), n_main, *args,
                                                  _ptr(g), _ptr(sse), _ptr(fin), st), what)
        if n_short:
            _lib.check(self.lib.cse_enhance_cells_short_hop(
                self.n_fft, self.L, _at(cells_d, n_main * k), n_short, *args, _at(sse, n_main),
                _at(fin, n_main), st), what + "(short hop)")
        if n_gen:
            o = n_main + n_short
            _lib.check(self.lib.cse_enhance_cells_generic(
                self.n_fft, self.L, _at(cells_d, o * k), n_gen, *args, _ptr(g), _at(sse, o),
                _at(fin, o), st), what + "(generic)")

    def execute(self, noisy, clean=None):
        self.prepare(noisy, clean)
        self.enhance()
        if self.align:
            self.finalize()

    def finalize(self):
        """finalize_enhanced on the device: per-cell cross-correlation lag
        (cse_xcorr_lag), then the cells whose lag is not 0 are scored again
        with the shifted output (cse_enhance_cells with cell.lag, plus the
        clean energy of the zero padding)."""
        lib, st = self.lib, _stream()
        _lib.check(lib.cse_xcorr_prepare(_ptr(self.clean), self.S, self.L, self.xc_n,
                                         self.xc_lag_max, _ptr(self.xc_ws), st),
                   "cse_xcorr_prepare")
        _lib.check(lib.cse_xcorr_lag(_ptr(self.head), _ptr(self.head_off), _ptr(self.sig_of),
                                     len(self.items), self.S, self.xc_n, self.xc_lag_max,
                                     _ptr(self.xc_ws), _ptr(self.lag_d), _ptr(self.zero_d),
                                     _ptr(self.xst_d), None, st), "cse_xcorr_lag")
        lag = self.lag_d.cpu().numpy()
        sel = np.nonzero(lag != 0)[0]
        self.rerun = None
        if len(sel) == 0:
            return
        cells = self.cells[sel].copy()
        cells["lag"] = lag[sel]
        cells["out_offset"] = -1
        cells["gain_offset"] = -1
        packed, order = pack_waves(cells, self.n_fft)
        cd = torch.from_numpy(packed.view(np.uint8).copy()).to(self.device)
        sse = torch.zeros(len(packed), dtype=torch.float64, device=self.device)
        fin = torch.zeros(len(packed), dtype=torch.uint8, device=self.device)
        self.launch(cd, route_slots(packed, self.n_fft), None, 0, None, sse, fin, st,
                    "cse_enhance_cells(aligned)")
        self.rerun = (sel, order, sse, fin)

    def results(self):
        sse_p = self.sse_d.cpu().numpy()
        fin_p = self.fin_d.cpu().numpy().astype(bool)
        real = self.order >= 0
        sse = np.empty(len(self.items))
        fin = np.empty(len(self.items), dtype=bool)
        sse[self.order[real]] = sse_p[real]
        fin[self.order[real]] = fin_p[real]
        self.lag = self.xstatus = None
        if self.align:
            self.lag = self.lag_d.cpu().numpy()
            self.xstatus = self.xst_d.cpu().numpy()
            # a non-finite head aligns at -max_lag (np.argmax over an all-NaN
            # correlation) and is rescored at that lag like any other: the
            # reference checks finiteness only after the shift (:100-103)
            if self.rerun is not None:
                sel, order, sse_r, fin_r = self.rerun
                sr, fr = sse_r.cpu().numpy(), fin_r.cpu().numpy().astype(bool)
                ok = order >= 0
                sse[sel[order[ok]]] = sr[ok] + self.zero_d.cpu().numpy()[sel[order[ok]]]
                fin[sel[order[ok]]] = fr[ok]
        G = None
        if self.g_out is not None:
            G = [self.g_out[g0:g0 + T * self.B].view(T, self.B) for (g0, T) in self.g_offsets]
        return sse, fin, G


class MultiPlan:
    """GridPlans for every n_fft present in a spec list (spec order preserved)."""

    def __init__(self, eng, S, L, specs, with_clean, want_y, want_g, align=False, true_len=None):
        self.n = len(specs)
        self.align = align
        self.want_g = want_g
        self.y_all = (torch.zeros((self.n, L), dtype=torch.float32, device=eng.device)
                      if want_y else None)
        by_fft = {}
        checked = set()
        for idx, (sig, alg, params) in enumerate(specs):
            alg = canonical_algo(alg)
            p = params  # defaults (DEFAULTS) are applied where a value is read
            hop, nf = p["hop_length"], p["n_fft"]
            if not 0 <= int(sig) < S:
                raise ValueError(f"signal index {sig} out of range")
            ck = (alg, hop, nf, p["noise_method"])
            if ck not in checked:  # per distinct (algorithm, hop, n_fft, method)
                r = route(nf, hop)
                if r is None:
                    raise ValueError(f"engine supports an even n_fft in [64, 4096] and "
                                     f"hop in [1, n_fft] (got n_fft={nf}, hop={hop})")
                if want_g and r == SHORT:
                    raise ValueError(f"gain matrices not at the short hops (n_fft={nf}, hop={hop})")
                noise_key(alg, p, n_frames(L, hop))  # validates the method
                if (p["noise_method"] == "true_noise" and not with_clean
                        and n_frames(L, hop) >= 5):
                    raise ValueError("TrueNoiseEstimator requires clean_audio and noisy_audio")
                checked.add(ck)
            by_fft.setdefault(int(nf), []).append((idx, int(sig), alg, p))
        self.plans = [GridPlan(eng, n_fft, S, L, items, with_clean, want_y, want_g, self.y_all,
                               align, true_len)
                      for n_fft, items in sorted(by_fft.items())]
        self.units = sum(p.units for p in self.plans)

    def execute(self, noisy, clean=None, on_plan=None):
        """Per n_fft: analysis (STFTs, noise rows), enhance, alignment.
        on_plan(plan, sse, finite, lag): called once an n_fft's cells are final
        (host-synchronised results in plan.items order; plan.idx maps them to
        spec indices), after the next n_fft's analysis is queued and before its
        enhance is, so the caller can queue work on those cells' outputs on
        another stream without starving the next analysis' small kernels."""
        if self.plans:
            self.plans[0].prepare(noisy, clean)
        for k, p in enumerate(self.plans):
            p.enhance()
            if p.align:
                p.finalize()
            if k + 1 < len(self.plans):
                self.plans[k + 1].prepare(noisy, clean)
            if on_plan is not None:
                sse, fin, _ = p.results()
                on_plan(p, sse, fin, p.lag)

    def results(self):
        sse = np.full(self.n, np.nan)
        fin = np.zeros(self.n, dtype=bool)
        gains = [None] * self.n if self.want_g else None
        lag = np.zeros(self.n, dtype=np.int64) if self.align else None
        xst = np.zeros(self.n, dtype=np.int64) if self.align else None
        for p in self.plans:
            s, f, G = p.results()
            ix = p.idx
            sse[ix], fin[ix] = s, f
            if gains is not None:
                for c, i in enumerate(ix):
                    gains[i] = G[c]
            if lag is not None and p.lag is not None:
                lag[ix], xst[ix] = p.lag, p.xstatus
        out = {"sse": sse, "finite": fin}
        if lag is not None:
            out["lag"], out["xcorr_status"] = lag, xst
        if self.y_all is not None:
            out["y"] = self.y_all
        if gains is not None:
            out["G"] = gains
        return out


def structure_digest():
    """A 128-bit hash object for plan-reuse keys: xxh3 (an order of magnitude
    faster than blake2b on the sweep's 17-MB batch descriptions) when the
    xxhash module is importable, blake2b otherwise."""
    try:
        import xxhash
        return xxhash.xxh3_128()
    except ImportError:
        import hashlib
        return hashlib.blake2b(digest_size=16)


def spec_fingerprint(specs):
    """Digest of a spec list's structure: per cell the signal index, the
    algorithm name and the identity of its params dict (Engine.run(reuse=True))."""
    n = len(specs)
    sig = np.fromiter((s for (s, _, _) in specs), dtype=np.int64, count=n)
    pid = np.fromiter((id(p) for (_, _, p) in specs), dtype=np.int64, count=n)
    algs = {}
    aid = np.fromiter((algs.setdefault(a, len(algs)) for (_, a, _) in specs), dtype=np.int64, count=n)
    h = structure_digest()
    for arr in (sig, pid, aid):
        h.update(arr)
    h.update(repr(sorted(algs.items(), key=lambda kv: kv[1])).encode())
    return h.hexdigest()


def pack_waves(cells, n_fft):
    """Group cells into workgroup slot groups (CSE_CELLS_PER_GROUP cells each).

    A slot group's cells must share (algo, hop, spectrum, noise, clean, lag) — the
    kernel stages those rows once per workgroup.  Returns (packed cells incl.
    CSE_ALGO_NONE padding, order) with order[i] = index into ``cells`` of packed
    slot i, or -1 for padding.  Groups are ordered longest-first (frames x
    algorithm cost, then by key) so the launch ends on short workgroups;
    neighbours share rows, and the kernel's XCD remap keeps neighbours on one
    XCD's L2.  Groups at the short hops (SHORT_HOPS) come after the sweep
    hops' and the groups of every other shape after those: each class goes to
    a launch of its own (GridPlan.launch, route_slots).  n_fft other than
    512 / 1024 is all generic: one cell per slot (the generic kernel runs one
    workgroup per cell), in the given order.
    Vectorised (numpy): a 100k-cell table packs in milliseconds.
    """
    n = len(cells)
    if n == 0:
        return np.zeros(0, dtype=_lib.CELL_DTYPE), np.zeros(0, dtype=np.int64)
    if int(n_fft) not in (512, 1024):
        return cells.copy(), np.arange(n, dtype=np.int64)
    per = _lib.cells_per_group(n_fft)
    keys = np.stack([cells[f].astype(np.int64) for f in
                     ("hop", "algo", "y_offset", "noise_offset", "noise_stride",
                      "clean_offset", "lag")], axis=1)
    uniq, inv = np.unique(keys, axis=0, return_inverse=True)  # rows in key order
    inv = inv.reshape(-1)
    G = len(uniq)
    counts = np.bincount(inv, minlength=G)
    nslots = (counts + per - 1) // per
    cost_of = np.zeros(8, dtype=np.float64)
    for name, code in _lib.ALGO.items():
        if code >= 0:
            cost_of[code] = ALGO_COST[name]
    cost = (1 + 16000 // uniq[:, 0]) * cost_of[uniq[:, 1]]
    cls = np.array([_cls(n_fft, h) for h in uniq[:, 0]], dtype=np.int64)
    gorder = np.lexsort((np.arange(G), -cost, cls))     # longest first, then key order
    slot_base = np.zeros(G, dtype=np.int64)
    slot_base[gorder] = np.concatenate([[0], np.cumsum(nslots[gorder])[:-1]])
    # rank of each cell inside its group, in the cells' original order
    by_group = np.argsort(inv, kind="stable")
    first = np.concatenate([[0], np.cumsum(counts)[:-1]])
    rank = np.empty(n, dtype=np.int64)
    rank[by_group] = np.arange(n) - first[inv[by_group]]
    slot = slot_base[inv] + rank // per
    total = int(nslots.sum())
    order = np.full(total * per, -1, dtype=np.int64)
    order[slot * per + rank % per] = np.arange(n)
    packed = np.zeros(len(order), dtype=_lib.CELL_DTYPE)
    real = order >= 0
    packed[real] = cells[order[real]]
    # padding: the group's shared rows, no algorithm, no outputs
    pad = np.nonzero(~real)[0]
    if len(pad):
        lead = order[(pad // per) * per]
        packed[pad] = cells[lead]
        packed["algo"][pad] = -1
        packed["out_offset"][pad] = -1
        packed["gain_offset"][pad] = -1
    return packed, order


def _cls(n_fft, hop):
    """route() for packing: shapes no kernel supports count as generic (that
    kernel's entry point refuses them)."""
    r = route(n_fft, hop)
    return GENERIC if r is None else r


def route_slots(packed, n_fft):
    """(sweep-hop, short-hop, generic) slot counts of a packed table, which
    pack_waves orders that way."""
    per = [0, 0, 0]
    hops, counts = np.unique(packed["hop"], return_counts=True)
    for h, k in zip(hops.tolist(), counts.tolist()):
        per[_cls(n_fft, h)] += int(k)
    return per[MAIN], per[SHORT], per[GENERIC]


def snr_db(sse, clean_power):
    """calculate_snr (evaluation_metrics.py:39-58) from the kernel's error energy."""
    sse = np.asarray(sse, dtype=np.float64)
    with np.errstate(divide="ignore"):
        out = 10.0 * np.log10(clean_power / (sse + 1e-10))
    return np.where(sse == 0, math.inf, out)
