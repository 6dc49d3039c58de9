"""Device orchestration of the STFT frame-gain path on MI355X.

PyTorch-ROCm is used only as the device-memory container and stream provider;
every numeric step is a libcse.so kernel (include/cse.h):

  cse_stft            STFT of every signal at each (n_fft, hop)        [once per group]
  cse_noise_estimate  percentile / min-tracking / true-noise PSDs     [once per group]
  cse_noise_smooth    MMSE/OMLSA noise IIR (per noise_mu)             [once per group]
  cse_istft_norm      1/window-sum-square per (n_fft, hop)            [once]
  cse_enhance_cells   THE HOT PATH: gain recursion + ISTFT + SNR sums [per grid cell]

A "cell spec" is (signal index, algorithm name, params dict) where params are
the reference plugin's keyword arguments (parameter_ranges.py keys).
"""

import ctypes
import math

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
# relative per-bin cost used to order waves (longest first)
ALGO_COST = {"SS": 1.0, "WIENER": 1.1, "MMSE": 2.0, "OMLSA": 3.0}


def canonical_algo(name):
    name = ALIASES.get(name, name)
    if name not in ALGOS:
        raise ValueError(f"unknown algorithm {name!r}")
    return name


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def n_frames(length, hop):
    return 1 + int(length) // int(hop)


def noise_key(alg, params, T):
    """Which noise PSD array a cell reads, mirroring each algorithm's pipeline.

    Returns (method, pct, eps, expand, mu):
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
        (mmse.py:48-54, advanced_mmse.py:60-66); mu=None means no smoothing.
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
    return (method, pct, eps, expand, mu)


def key_is_static(key):
    method, _, _, expand, mu = key
    return method in ("percentile", "simple") and not expand and mu is None


class Engine:
    """Runs batches of grid cells over batches of equal-length signals."""

    def __init__(self, device="cuda"):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.CseError("no GPU visible: the HIP engine has no CPU fallback")
        self.device = torch.device(device)

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

    def noise_estimate(self, method, P, percentile=20.0, eps=1e-10, out=None):
        S, T, B = P.shape
        code = {"percentile": 0, "min_tracking": 1, "true_noise": 2, "simple": 0}[method]
        static = method == "percentile" or (T < 5 and method != "true_noise")
        shape = (S, B) if (static and method != "min_tracking") else (S, T, B)
        if out is None:
            out = torch.empty(shape, dtype=torch.float32, device=P.device)
        ws = torch.empty(int(self.lib.cse_noise_workspace_bytes(S, T, B)), dtype=torch.uint8,
                         device=P.device)
        _lib.check(self.lib.cse_noise_estimate(code, _ptr(P), S, T, B, float(percentile),
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
    def run(self, noisy, specs, clean=None, want_waveforms=False, want_gains=False):
        """Enhance every cell spec; returns a dict of per-spec results.

        noisy/clean: [S, L] float64 cuda tensors (clean may be None if no spec
        uses true_noise and no SNR is wanted).  specs: list of
        (signal_index, algorithm_name, params).  Results (numpy, spec order):
          sse [n] f64, finite [n] bool, and optionally 'y' [n, L] f32 (cuda)
          and 'G' list of [T, B] f32 (cuda).
        """
        S, L = noisy.shape
        n = len(specs)
        sse = np.full(n, np.nan)
        finite = np.zeros(n, dtype=bool)
        y_all = (torch.zeros((n, L), dtype=torch.float32, device=noisy.device)
                 if want_waveforms else None)
        gains = [None] * n if want_gains else None
        by_fft = {}
        for idx, (sig, alg, params) in enumerate(specs):
            alg = canonical_algo(alg)
            p = dict(DEFAULTS.get(alg, {}))
            p.update(params)
            if p["hop_length"] not in (128, 256) or p["n_fft"] not in (512, 1024):
                raise ValueError("engine supports n_fft in {512,1024}, hop in {128,256}")
            if p["noise_method"] == "true_noise" and clean is None and n_frames(L, p["hop_length"]) >= 5:
                raise ValueError("TrueNoiseEstimator requires clean_audio and noisy_audio")
            by_fft.setdefault(int(p["n_fft"]), []).append((idx, int(sig), alg, p))
        for n_fft, items in by_fft.items():
            res = self._run_fft(n_fft, noisy, clean, items, want_waveforms, want_gains, y_all)
            for (idx, *_), s, f, g in zip(items, res["sse"], res["finite"], res["G"]):
                sse[idx], finite[idx] = s, f
                if want_gains:
                    gains[idx] = g
        out = {"sse": sse, "finite": finite}
        if want_waveforms:
            out["y"] = y_all
        if want_gains:
            out["G"] = gains
        return out

    def _run_fft(self, n_fft, noisy, clean, items, want_y, want_g, y_all):
        S, L = noisy.shape
        B = n_fft // 2 + 1
        hops = sorted({p["hop_length"] for (_, _, _, p) in items})
        # ---- spectra of every signal at every hop, one buffer (y_offset per cell)
        y_base, y_parts, P64 = {}, [], {}
        off = 0
        for hop in hops:
            T = n_frames(L, hop)
            Y, P = self.stft(noisy, n_fft, hop)
            y_parts.append(Y.reshape(-1))
            y_base[hop] = off
            off += S * T * B
            P64[hop] = P
        Ybuf = torch.cat(y_parts) if len(y_parts) > 1 else y_parts[0]
        # ---- noise pool: every distinct PSD the cells read
        keys = {}
        for (_, _, alg, p) in items:
            T = n_frames(L, p["hop_length"])
            keys.setdefault((p["hop_length"], noise_key(alg, p, T)), None)
        pool_parts, pool_off, noff = [], {}, 0
        true_P = {}
        for (hop, key) in keys:
            method, pct, eps, expand, mu = key
            T = n_frames(L, hop)
            P = P64[hop]
            if method == "true_noise":
                if hop not in true_P:
                    if clean is None:
                        raise ValueError("TrueNoiseEstimator requires clean_audio and noisy_audio")
                    true_P[hop] = self.stft(noisy, n_fft, hop, x_sub=clean, want_y=False)[1]
                N = self.noise_estimate("true_noise", true_P[hop], eps=eps)
            elif method == "simple":
                N = self.noise_estimate("percentile", P, 25.0, eps)
            else:
                N = self.noise_estimate(method, P, pct if pct is not None else 20.0, eps)
            if expand or mu is not None:
                N = self.noise_smooth(N, T, mu or 0.0)
            stride = 0 if N.dim() == 2 else B
            pool_parts.append(N.reshape(-1))
            pool_off[(hop, key)] = (noff, stride, N.shape[-1] if stride == 0 else T * B)
            noff += N.numel()
        pool = torch.cat(pool_parts) if len(pool_parts) > 1 else pool_parts[0]
        inv = {h: self.istft_norm(n_fft, h, L) for h in hops}
        # ---- cells
        G_bufs = [None] * len(items)
        cells = np.zeros(len(items), dtype=_lib.CELL_DTYPE)
        g_total = 0
        for c, (idx, sig, alg, p) in enumerate(items):
            code, _, names = ALGOS[alg]
            hop = p["hop_length"]
            T = n_frames(L, hop)
            o, stride, per_sig = pool_off[(hop, noise_key(alg, p, T))]
            cells["algo"][c] = _lib.ALGO[code]
            cells["hop"][c] = hop
            cells["y_offset"][c] = y_base[hop] + sig * T * B
            cells["noise_offset"][c] = o + sig * per_sig
            cells["noise_stride"][c] = stride
            cells["clean_offset"][c] = sig * L if clean is not None else -1
            cells["out_offset"][c] = idx * L if want_y else -1
            if want_g:
                cells["gain_offset"][c] = g_total
                g_total += T * B
            else:
                cells["gain_offset"][c] = -1
            prm = [float(p[k]) for k in names]
            cells["param"][c, :len(prm)] = prm
        packed, order = pack_waves(cells, n_fft)
        dev = noisy.device
        cells_d = torch.from_numpy(packed.view(np.uint8)).to(dev)
        g_out = torch.zeros(g_total, dtype=torch.float32, device=dev) if want_g else None
        sse_d = torch.zeros(len(packed), dtype=torch.float64, device=dev)
        fin_d = torch.zeros(len(packed), dtype=torch.uint8, device=dev)
        clean32 = clean.to(torch.float32).contiguous() if clean is not None else None
        _lib.check(self.lib.cse_enhance_cells(
            n_fft, L, _ptr(cells_d), len(packed), _ptr(Ybuf), _ptr(pool), _ptr(clean32),
            _ptr(inv.get(128)), _ptr(inv.get(256)), _ptr(y_all), _ptr(g_out), _ptr(sse_d),
            _ptr(fin_d), _stream()), "cse_enhance_cells")
        sse_p = sse_d.cpu().numpy()
        fin_p = fin_d.cpu().numpy().astype(bool)
        sse = np.empty(len(items))
        fin = np.empty(len(items), dtype=bool)
        sse[order[order >= 0]] = sse_p[order >= 0]
        fin[order[order >= 0]] = fin_p[order >= 0]
        if want_g:
            for c, (idx, sig, alg, p) in enumerate(items):
                T = n_frames(L, p["hop_length"])
                g0 = int(cells["gain_offset"][c])
                G_bufs[c] = g_out[g0:g0 + T * B].view(T, B)
        return {"sse": sse, "finite": fin, "G": G_bufs}


def pack_waves(cells, n_fft):
    """Group cells that share (hop, algo, spectrum, noise) into wave slots.

    Returns (packed cells incl. CSE_ALGO_NONE padding, order) where
    order[i] = index into ``cells`` of packed slot i, or -1 for padding.
    Waves are ordered longest-first (frames x algorithm cost) so the tail of the
    launch is short waves; groups stay contiguous so the kernel's XCD remap
    keeps a group's Y/N rows in one XCD's L2.
    """
    cpw = _lib.cells_per_wave(n_fft)
    code_name = {v: k for k, v in _lib.ALGO.items()}
    groups = {}
    for i, c in enumerate(cells):
        key = (int(c["hop"]), int(c["algo"]), int(c["y_offset"]), int(c["noise_offset"]))
        groups.setdefault(key, []).append(i)
    waves = []
    for key, idxs in groups.items():
        hop, algo = key[0], key[1]
        cost = (1 + 16000 // hop) * ALGO_COST[code_name[algo]]
        for s in range(0, len(idxs), cpw):
            chunk = idxs[s:s + cpw]
            waves.append((-cost, key, chunk + [-1] * (cpw - len(chunk))))
    waves.sort(key=lambda w: (w[0], w[1]))
    order = np.array([i for w in waves for i in w[2]], dtype=np.int64)
    packed = np.zeros(len(order), dtype=_lib.CELL_DTYPE)
    real = order >= 0
    packed[real] = cells[order[real]]
    # padding slots: same hop/algo as their wave (kernel skips them)
    for w, (_, key, chunk) in enumerate(waves):
        for s, i in enumerate(chunk):
            if i < 0:
                slot = w * cpw + s
                packed[slot] = cells[chunk[0]]
                packed[slot]["algo"] = -1
                packed[slot]["out_offset"] = -1
                packed[slot]["gain_offset"] = -1
    # a padded slot's algo = -1 would become the wave algo only if it were slot 0
    assert all(packed[w * cpw]["algo"] >= 0 for w in range(len(waves)))
    return packed, order


def snr_db(sse, clean_power):
    """calculate_snr (evaluation_metrics.py:39-58) from the kernel's error energy."""
    sse = np.asarray(sse, dtype=np.float64)
    with np.errstate(divide="ignore"):
        out = 10.0 * np.log10(clean_power / (sse + 1e-10))
    return np.where(sse == 0, math.inf, out)
