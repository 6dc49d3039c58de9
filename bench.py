#!/usr/bin/env python
"""bench.py — STFT frame-gain evaluations/s on MI355X (BASELINE.json metric).

Workload (one "step"): the n_fft=512 half of the reference's full HEAD grid
(parameter_ranges.py: SS 360 + MMSE 960 + Wiener 96 + OMLSA 3456 = 4872 cells
per pair, hops 128 and 256, all 4 algorithms) over synthetic 10-s 16-kHz pairs:
  STFT + noise PSDs (percentile 10/20, min-tracking, smoothing)   [per pair]
  fused gain recursion + ISTFT + clipped-SNR sums, every cell     [THE HOT PATH]
  per-cell records (sse, finite) gathered to every rank           [results table]
Unit = one frame-gain evaluation = one cell x one STFT frame, all 257 bins
(SURVEY §8(d)): 4,572,372 per pair.  Every cell is counted, including the
quarter that are exact duplicates (min_tracking ignores noise_percentile).

Scaling modes (one process per GPU under torchrun, RCCL = backend "nccl"):
  default  --pairs-total 100: BASELINE config 4's fixed job of 100 pairs,
           cells sharded over the ranks by search.assign_shards (contiguous
           runs of cell ids of equal modelled cost: whole pairs per rank);
           "scaling": "strong", value = 100 pairs' units / max-rank time.
  --pairs P: P pairs per GPU ("scaling": "weak").
Every step ends with one all_gather_into_tensor of the per-cell records.

The line also carries two labelled blocks beside the headline:
  full_grid     the same step over the whole HEAD grid, both n_fft halves
                (9,744 cells per pair), with each half's kernel time;
  sweep         the reference's whole job through search.run_grid: alignment,
                SNR and STOI of every cell, the gather and both sequential
                selections, wall seconds and cells/s;
and "roofline", the enhance kernel against VALU lane-op throughput (the
resource it spends: each instruction priced at the SIMD cycles it takes), with
the measured HBM GB/s and SURVEY §8(d)'s algorithmic byte figure beside it.

At N = 1 the line also carries
  parity        the timed step's per-cell SNR table of pair 0 against the
                oracle on every cell the CPU baseline computed, and the
                waveforms of 64 cells stratified over algorithm x hop x noise
                method against the oracle (north-star: rel-L2 and rel-max
                <= 1e-5); the run fails above tolerance;
  cpu_baseline  the oracle on this host's cores (see cpu_baseline()).

    python bench.py [--gpus N --steps K --warmup W --pairs-total 100 | --pairs P]
                    [--full-grid-steps F] [--no-sweep]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = ("STFT frame-gain evals/sec/node, 16kHz 512-pt FFT full grid; 1/2/4/8-GPU scaling")
HBM_PEAK = 8.0e12              # MI355X_MICROARCH.md: 8.0 TB/s spec
SIMDS = 1024                   # 256 CUs x 4 SIMD-32
FP32_PEAK = 157.3e12           # MI355X_MICROARCH.md: FP32 vector, spec (64 FLOP/clk/SIMD)
# SIMD cycles per wave64 VALU instruction, measured chip-wide at 8 waves/SIMD
# (tools/micro/valu_cal.hip, tools/micro/valu_mix.hip, HIP-event timed;
# profiles/r06_micro_valu_cal.json, r06_micro_valu_mix.txt): a packed v_pk_*_f32
# 4.0-4.2 and never overlapped by another VALU instruction (v_pk_fma_f32 153 TF =
# the 157.3 TF FP32 peak); a transcendental 8.1, also exclusive (v_fma_f32 and
# v_exp_f32 interleaved cost 4 + 8); an fp64 FMA 4.1-4.5; scalar f32 instructions
# of the SIMD's two halves issue in parallel (v_add/v_mul/v_mov/v_add_u32 streams
# 2.3-2.5, v_fma_f32 interleaved with v_add/v_mul/v_max 2.3-2.5 per instruction,
# a pure v_fma_f32 or v_max_f32 stream 4).  Scalar f32 is priced at the parallel
# rate, 2 (the guide's SIMD-32 figure, a lower bound on what the kernel's scalar
# instructions take).  The guide's transcendental price (4) is reported beside it.
VALU_CYC, PK_CYC, TRANS_CYC, F64_CYC = 2, 4, 8, 4
GUIDE_TRANS_CYC = 4
CLOCK = 2.4e9                  # max shader clock
TOL = 1e-5                     # north-star relative waveform tolerance
SNR_TOL_DB = 2e-4              # per-cell SNR tolerance of the parity tests

from classical_speech_enhancement_amd.parameter_ranges import grid_specs  # noqa: E402


# ---------------------------------------------------------------------------
# CPU side: the oracle (test infrastructure) as the reference's CPU path
# ---------------------------------------------------------------------------
def _cpu_cell(args):
    """One reference cell on the CPU: (cell index, frames, lag-0 SNR of the
    clipped output, waveform as f64 or None)."""
    idx, pair, alg, params, seconds, want_y = args
    import oracle
    from classical_speech_enhancement_amd.synth import make_pair
    if getattr(_cpu_cell, "key", None) != (pair, seconds):
        _cpu_cell.pair = make_pair(pair, seconds)
        _cpu_cell.key = (pair, seconds)
    clean, noisy = _cpu_cell.pair
    kw = dict(params)
    if kw["noise_method"] == "true_noise":
        kw["clean_audio"] = clean
    y = oracle.ALGORITHMS[alg](noisy, 16000, **kw)
    snr = oracle.calculate_snr(clean, np.clip(y, -1, 1))
    return idx, 1 + int(len(noisy)) // int(params["hop_length"]), snr, (y if want_y else None)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cpu_share():
    """(processes to use, affinity count, os.cpu_count()).  The pool uses every
    core this process may run on, capped by the per-GPU CPU share the GPU box
    allots (it exports OMP_NUM_THREADS = its share, 16 per GPU, and asks for
    worker pools of that size)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = os.environ.get("CSE_CPU_BASELINE_PROCS") or os.environ.get("OMP_NUM_THREADS")
    n = aff if not share else min(aff, max(1, int(share)))
    return n, aff, os.cpu_count()


def parity_cells(seconds, n_fft, per_stratum=4, seed=7):
    """Indices into grid_specs(1, n_fft): per_stratum cells drawn from every
    (algorithm, hop, noise method) stratum (4 x 2 x 2 x 4 = 64 cells)."""
    specs = grid_specs(1, n_fft)
    strata = {}
    for i, (_, alg, p) in enumerate(specs):
        strata.setdefault((alg, p["hop_length"], p["noise_method"]), []).append(i)
    rng = np.random.default_rng(seed)
    out = []
    for key in sorted(strata):
        ids = strata[key]
        out += sorted(rng.choice(ids, min(per_stratum, len(ids)), replace=False).tolist())
    return out


def cpu_run(budget_s, seconds, n_fft, y_cells, timed=True, pair=0):
    """Run the oracle on the host cores: first the y_cells (waveforms kept for
    the parity check), then (timed) cells drawn uniformly at random from the
    pair's grid until budget_s of wall time.  Returns (baseline dict or None,
    {cell: snr}, {cell: y}); cells are indices into grid_specs(1, n_fft)."""
    import multiprocessing as mp
    procs, aff, ncpu = _cpu_share()
    specs = grid_specs(1, n_fft)
    rng = np.random.default_rng(0)
    want = set(y_cells)
    order = [i for i in rng.permutation(len(specs)).tolist() if i not in want]
    work = [(i, pair, specs[i][1], specs[i][2], seconds, i in want)
            for i in list(y_cells) + order]
    env_keys = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")
    saved = {k: os.environ.get(k) for k in env_keys}
    for k in env_keys:
        os.environ[k] = "1"
    snr, ys = {}, {}
    units = cells = 0
    dt = 0.0
    try:
        with mp.get_context("spawn").Pool(procs) as pool:
            # warm the workers (imports + synth) outside the window
            list(pool.imap_unordered(_cpu_cell, [(0, pair, w[2], w[3], seconds, False)
                                                 for w in work[:procs]]))
            stream = work if timed else work[:len(y_cells)]
            t0 = time.perf_counter()
            for idx, u, s, y in pool.imap_unordered(_cpu_cell, stream, chunksize=1):
                snr[idx] = s
                if y is not None:
                    ys[idx] = y
                units += u
                cells += 1
                if timed and len(ys) == len(want) and time.perf_counter() - t0 > budget_s:
                    break
            dt = time.perf_counter() - t0
            pool.terminate()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    base = None
    if timed:
        base = {"value": units / dt, "unit": "frame-gain evals/s", "cores": procs, "kind": "port",
                "cpu_model": _cpu_model(), "affinity_cores": aff, "os_cpu_count": ncpu,
                "sample": (f"{cells} cells of the n_fft={n_fft} HEAD grid on pair 0 (10-s): "
                           f"{len(y_cells)} stratified parity cells, then cells drawn uniformly "
                           f"at random; oracle/ fp64 numpy (the reference's algorithm, per-cell "
                           f"STFT + noise estimate, per-frame loops), {procs} single-threaded "
                           f"processes (the GPU box's per-GPU CPU share; {aff} cores in this "
                           f"process's affinity), {dt:.1f} s wall")}
    return base, snr, ys


def load_pmc(units_per_launch, n_fft):
    """Counters of the enhance kernel for this exact launch size and n_fft,
    from the committed rocprofv3 PMC passes (profiles/pmc_*.json,
    tools/pmc_summary.py; the newest round wins; roofline_block uses them only
    while their kernel_src_sha matches this build's)."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if (d.get("units_per_launch") == units_per_launch and f"<{n_fft}" in d.get("kernel", "")
                and (best is None or str(d.get("round", "")) >= str(best.get("round", "")))):
            best = d
    return best


def code_text(src):
    """C/C++/HIP source with its comments removed and whitespace runs
    collapsed (string and character literals kept): what kernel_src_sha
    hashes, so documentation edits leave the digest alone."""
    import re
    tok = re.compile(r'//[^\n]*|/\*.*?\*/|"(?:\\.|[^"\\\n])*"|\'(?:\\.|[^\'\\\n])*\'', re.S)
    out = tok.sub(lambda m: " " if m.group(0)[0] == "/" else m.group(0), src)
    return re.sub(r"\s+", " ", out).strip()


def kernel_src_sha():
    """Digest of the enhance kernel's sources (code only: code_text) and build
    flags: a committed PMC profile counts the instructions of one binary, so
    bench.py uses its counters only while this digest matches the one the
    profile recorded."""
    import hashlib
    import __graft_entry__ as ge
    h = hashlib.sha256()
    paths = [os.path.join(ge.CSRC, f) for f in ("cse_enhance.hip", "cse_enhance_512.hip",
                                                 "cse_enhance_1024.hip", "cse_common.hpp",
                                                 "cse_special.hpp")]
    for path in paths + [os.path.join(REPO, "include", "cse.h")]:
        h.update(code_text(open(path, encoding="utf-8").read()).encode())
    h.update(repr(sorted(ge.OWN_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def rank_job(args, world, rank, n_fft):
    """(pair ids of this rank, its cell specs as (slot, algorithm, params),
    their global cell ids, units of the whole job per step, pairs in the whole
    job).  n_fft None: the full grid (both halves)."""
    from classical_speech_enhancement_amd import search
    from classical_speech_enhancement_amd.engine import n_frames
    L = int(round(args.seconds * 16000))
    if args.pairs is not None:   # weak: P pairs per rank
        total_pairs = args.pairs * world
        pair_ids = [rank * args.pairs + i for i in range(args.pairs)]
        local = [tuple(s) for s in search.job_specs(args.pairs, n_fft=n_fft)]
        gids = rank * len(local) + np.arange(len(local), dtype=np.int64)
    else:                        # strong: the fixed job, contiguous cost-balanced shards
        total_pairs = args.pairs_total
        specs = search.job_specs(total_pairs, n_fft=n_fft)
        rank_of, _ = search.assign_shards(specs, [L] * total_pairs, world)
        mine = np.flatnonzero(rank_of == rank)
        pair_ids = sorted(set(specs.pair[mine].tolist()))
        slot = {p: s for s, p in enumerate(pair_ids)}
        local = [(slot[int(specs.pair[c])],) + tuple(specs[int(c)])[1:] for c in mine]
        gids = mine.astype(np.int64)
    units = sum(n_frames(L, p["hop_length"]) for (_, _, p) in grid_specs(1, n_fft)) * total_pairs
    return pair_ids, local, gids, units, total_pairs


class ClockSampler:
    """The shader clock's DPM level while the timed steps run: sysfs
    pp_dpm_sclk (the level marked '*'), read every 50 ms on a thread, so a line
    from a box that held a lower clock says so (the level is what the power
    manager selected; a power-capped part may run below it).  Empty where sysfs
    is not readable."""

    def __init__(self, period=0.05):
        import threading
        self.files = self._card_files()
        self.period, self.samples = period, []
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True)

    @staticmethod
    def _card_files():
        """pp_dpm_sclk of the GPU this process uses (the host's sysfs lists
        every card): matched by PCI bus id, from torch's device properties or
        hipDeviceGetPCIBusId of the HIP runtime already loaded; [] if unknown."""
        import ctypes
        import glob
        try:
            import torch
            dev = torch.cuda.current_device()
            bus = None
            prop = torch.cuda.get_device_properties(dev)
            if getattr(prop, "pci_bus_id", None) is not None:
                bus = "%02x:%02x" % (prop.pci_bus_id, getattr(prop, "pci_device_id", 0))
            if bus is None:
                lib = next((line.split()[-1] for line in open("/proc/self/maps")
                            if "libamdhip64.so" in line), None)
                if lib:
                    buf = ctypes.create_string_buffer(64)
                    if ctypes.CDLL(lib).hipDeviceGetPCIBusId(buf, 64, dev) == 0:
                        bus = buf.value.decode().lower().split(":", 1)[-1].rsplit(".", 1)[0]
            if bus:
                import os as _os
                return [f + "/pp_dpm_sclk" for f in sorted(glob.glob("/sys/class/drm/card*/device"))
                        if _os.path.basename(_os.path.realpath(f)).lower().rsplit(".", 1)[0].endswith(bus)]
        except Exception:
            pass
        return []

    def _read(self):
        import re
        best = None
        for f in self.files:
            try:
                for line in open(f):
                    if "*" in line:
                        m = re.search(r"(\d+)\s*[Mm][Hh]z", line)
                        if m:
                            best = max(best or 0, int(m.group(1)))
            except OSError:
                pass
        return best

    def _run(self):
        while not self._stop.is_set():
            v = self._read()
            if v is not None:
                self.samples.append(v)
            self._stop.wait(self.period)

    def start(self):
        if self.files:
            self._thread.start()
        return self

    def stop(self):
        if self.files:
            self._stop.set()
            self._thread.join()
        x = self.samples
        return {"source": ("sysfs pp_dpm_sclk of this process's GPU (DPM level, every 50 ms during "
                           "the timed steps)"), "files": self.files,
                "n": len(x), "mean_mhz": (sum(x) / len(x)) if x else None,
                "min_mhz": min(x) if x else None, "max_mhz": max(x) if x else None}


class TimedJob:
    """A rank's share of one step's work — STFT + noise PSDs, the fused enhance
    of every cell (one launch per n_fft), one all_gather of the per-cell records
    and their copy to the host — over device-resident pairs.  n_buf plan sets
    rotate: the analysis of step k + n_buf - 1 is queued on a side stream right
    after step k's enhance (no data shared).  With device collectives (RCCL, or world 1) the
    records of step k reach pinned host memory on a copy stream while step k+1
    computes; the timed region's closing synchronize covers the last copy."""

    def __init__(self, eng, noisy, clean, specs, gids, n_buf, align, dist_ctx):
        import torch
        self.torch = torch
        S, L = noisy.shape
        self.noisy, self.clean, self.align = noisy, clean, align
        self.dist, self.coll_dev, self.world = dist_ctx
        self.n_buf = n_buf
        self.mps = [eng.plan(S, L, specs, with_clean=True, align=align) for _ in range(n_buf)]
        self.units = self.mps[0].units
        self.n_cells = len(specs)
        self.main_s = torch.cuda.current_stream()
        # the analysis side stream (priority: CSE_PREP_PRIORITY, default 0).  Its
        # first STFT (80 KB of LDS) cannot take the slot of one finished enhance
        # workgroup, so the chain starts in the launch's drain tail, where the
        # freed CUs are idle anyway; r05 measured the chain inside the launch
        # (STFT at 47 KB, priority -1): no faster at 512, 4 % slower at 1024
        # ("analysis overlap")
        prio = int(os.environ.get("CSE_PREP_PRIORITY", "0"))
        self.prep_s = torch.cuda.Stream(priority=prio) if n_buf > 1 else self.main_s
        self.ev_prep = [torch.cuda.Event() for _ in range(n_buf)]
        self.ev_done = [None] * n_buf
        self.k = 0
        n_rec = sum(p.n_packed for p in self.mps[0].plans)
        if self.dist is not None:
            t = torch.tensor([n_rec], dtype=torch.int64, device=self.coll_dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            n_rec = int(t.item())
        # records: sse, finite, global cell id (-1: padding slot) per packed slot,
        # one set per plan set (a step's records are still being copied while
        # the next step writes its own)
        ids = torch.full((n_rec,), -1.0, dtype=torch.float64)
        o = 0
        for p in self.mps[0].plans:  # every plan set packs alike
            real = p.order >= 0
            g = np.full(p.n_packed, -1, dtype=np.int64)
            g[real] = np.asarray(gids, dtype=np.int64)[p.idx[p.order[real]]]
            ids[o:o + p.n_packed] = torch.as_tensor(g.astype(np.float64))
            o += p.n_packed
        self.rec_pad = []
        for _ in range(n_buf):
            r = torch.zeros((3, n_rec), dtype=torch.float64, device="cuda")
            r[2] = ids.to("cuda")
            self.rec_pad.append(r)
        self.rec_all = [torch.empty((self.world * 3, n_rec), dtype=torch.float64,
                                    device=self.coll_dev) for _ in range(n_buf)]
        # device collectives: host copies ride a copy stream into pinned memory
        self.async_host = self.dist is None or str(self.coll_dev).startswith("cuda")
        if self.async_host:
            self.copy_s = torch.cuda.Stream()
            self.host_rec = [torch.empty((self.world * 3, n_rec), dtype=torch.float64,
                                         pin_memory=True) for _ in range(n_buf)]
            self.ev_copied = [None] * n_buf
        self.gathered = None
        self.gathered_buf = None
        self.prep_evs = None
        for k in range(n_buf - 1):  # the analyses of the first n_buf - 1 steps
            self.prep(k)

    def prep(self, k):
        b = k % self.n_buf
        torch = self.torch
        with torch.cuda.stream(self.prep_s):
            if self.ev_done[b] is not None:
                self.prep_s.wait_event(self.ev_done[b])  # the enhance that last read these buffers
            ev = None
            if self.prep_evs is not None:  # timed region: the analysis chain's span
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record(self.prep_s)
            # every plan's STFTs, then every plan's noise chains (GridPlan.prepare_stft)
            # (full grid, A/B on one box: 571.2 / 572.3 ms/step against 575.4 /
            # 572.8 with each plan's STFTs and chains in turn)
            for p in self.mps[b].plans:
                p.prepare_stft(self.noisy, self.clean)
            for p in self.mps[b].plans:
                p.prepare_noise(self.clean)
            if ev is not None:
                ev[1].record(self.prep_s)
                self.prep_evs.append(ev)
            self.ev_prep[b].record(self.prep_s)

    def step(self, evs=None):
        """evs: per plan (start, end) timing events around its enhance launch."""
        torch = self.torch
        b = self.k % self.n_buf
        self.k += 1
        mp = self.mps[b]
        if self.n_buf == 1:
            self.prep(self.k - 1)
        self.main_s.wait_event(self.ev_prep[b])
        for j, plan in enumerate(mp.plans):
            if evs is not None:
                evs[j][0].record()
            plan.enhance()
            if evs is not None:
                evs[j][1].record()
            if self.align:
                plan.finalize()
        self.ev_done[b] = torch.cuda.Event()
        self.ev_done[b].record(self.main_s)
        if self.n_buf > 1:
            # the analysis n_buf - 1 steps ahead, into the buffers step k - 1
            # read (it waits for that enhance); it overlaps this step's enhance
            # (the timed region holds K preps)
            self.prep(self.k + self.n_buf - 2)
        rec = self.rec_pad[b]
        if self.async_host and self.ev_copied[b] is not None:
            self.main_s.wait_event(self.ev_copied[b])  # the copy that last read rec[b]
        o = 0
        for plan in mp.plans:
            m = plan.n_packed
            rec[0, o:o + m] = plan.sse_d
            rec[1, o:o + m] = plan.fin_d
            o += m
        if self.dist is not None:
            self.dist.all_gather_into_tensor(self.rec_all[b], rec.to(self.coll_dev))
            src = self.rec_all[b]
        else:
            src = rec
        if self.async_host:
            ev = torch.cuda.Event()
            ev.record(self.main_s)
            self.copy_s.wait_event(ev)
            with torch.cuda.stream(self.copy_s):
                self.host_rec[b].copy_(src, non_blocking=True)
            self.ev_copied[b] = torch.cuda.Event()
            self.ev_copied[b].record(self.copy_s)
            self.gathered, self.gathered_buf = self.host_rec[b], b
        else:
            self.gathered = src.cpu()
        return self.gathered

    def table(self, n_cells):
        """The last step's gathered records as [n_cells, 2] (sse, finite) by
        global cell id; every cell exactly once."""
        if self.async_host:
            self.ev_copied[self.gathered_buf].synchronize()
        r = self.gathered.numpy().reshape(self.world, 3, -1).transpose(1, 0, 2).reshape(3, -1)
        ids = r[2].astype(np.int64)
        keep = ids >= 0
        ids = ids[keep]
        assert len(ids) == n_cells and len(np.unique(ids)) == n_cells, "gathered records"
        out = np.empty((n_cells, 2))
        out[ids, 0] = r[0][keep]
        out[ids, 1] = r[1][keep]
        return out

    def run(self, steps, warmup):
        """Warmup, then K timed steps bracketed by barrier + synchronize; returns
        (seconds, max over ranks; mean enhance-kernel ms per plan).  Also sets
        self.rank_stats: this rank's own figures (its wall seconds before the
        max, the summed enhance-kernel ms per step, the analysis chain's span
        per step on its side stream, units and pairs per step)."""
        torch = self.torch
        for _ in range(warmup):
            self.step()
        torch.cuda.synchronize()
        n_pl = len(self.mps[0].plans)
        evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(n_pl)] for _ in range(steps)]
        self.prep_evs = []
        if self.dist is not None:
            self.dist.barrier()
        torch.cuda.synchronize()
        clock = ClockSampler().start()
        t0 = time.perf_counter()
        for k in range(steps):
            self.step(evs[k])
        torch.cuda.synchronize()
        local = time.perf_counter() - t0
        self.clock = clock.stop()
        if self.dist is not None:
            self.dist.barrier()
        dt = time.perf_counter() - t0
        if self.dist is not None:
            t = torch.tensor([dt], dtype=torch.float64, device=self.coll_dev)
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            dt = float(t.item())
        kern = [float(np.mean([e[j][0].elapsed_time(e[j][1]) for e in evs])) for j in range(n_pl)]
        ana = [s.elapsed_time(e) for s, e in self.prep_evs]
        self.prep_evs = None
        self.rank_stats = {"wall_s": local, "kernel_ms": float(sum(kern)),
                           "analysis_ms": float(np.mean(ana)) if ana else 0.0,
                           "units": float(self.units), "cells": float(self.n_cells)}
        return dt, kern

    def last_plans(self):
        return self.mps[(self.k - 1) % self.n_buf].plans


RANK_FIELDS = ("wall_s", "kernel_ms", "analysis_ms", "units", "cells", "pairs")


def gather_rank_stats(stats, dist_ctx):
    """Every rank's own figures (TimedJob.rank_stats + its pair count) on every
    rank, with the spread of the work over the ranks: max / mean of the
    enhance-kernel time, of the rank's own wall time and of its units.  One
    all_gather_into_tensor (RCCL on device tensors for backend nccl)."""
    import torch
    dist, coll_dev, world = dist_ctx
    v = torch.tensor([float(stats[k]) for k in RANK_FIELDS], dtype=torch.float64)
    if dist is not None:
        out = torch.empty(world * len(RANK_FIELDS), dtype=torch.float64, device=coll_dev)
        dist.all_gather_into_tensor(out, v.to(coll_dev))
        v = out.cpu()
    rows = v.numpy().reshape(-1, len(RANK_FIELDS))
    ranks = [{k: (int(r[i]) if k in ("units", "cells", "pairs") else float(r[i]))
              for i, k in enumerate(RANK_FIELDS)} for r in rows]

    def spread(k):
        x = rows[:, RANK_FIELDS.index(k)]
        return float(x.max() / x.mean()) if x.mean() > 0 else None
    return {"per_rank": ranks,
            "imbalance_max_over_mean": {"kernel_ms": spread("kernel_ms"),
                                        "wall_s": spread("wall_s"), "units": spread("units")},
            "fields": ("wall_s: the rank's own timed seconds (before the max over ranks); "
                       "kernel_ms: its enhance launch(es) per step, HIP events on the launch "
                       "stream; analysis_ms: its STFT + noise-PSD chain per step, HIP events on "
                       "the side stream it overlaps the enhance from; units, cells, pairs: its "
                       "share of one step")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs-total", type=int, default=100,
                    help="strong scaling: this many 10-s pairs in all, sharded over the ranks "
                         "(BASELINE config 4: 100)")
    ap.add_argument("--pairs", type=int, default=None,
                    help="weak scaling: this many 10-s pairs per GPU instead")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--nfft", type=int, default=512, choices=(512, 1024),
                    help="which half of the HEAD grid (the metric is quoted at 512)")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="plan sets in flight: the analysis runs pipeline - 1 steps ahead of "
                         "the enhance it feeds (each step still does one analysis and one "
                         "enhance; 3 measured 173.2 vs 174.3 ms/step for 2, 4 no better)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run each step's prep and enhance back to back on one stream")
    ap.add_argument("--align", action="store_true",
                    help="also run finalize_enhanced's alignment (xcorr lag + lag-shifted rescoring)"
                         " inside the step (SURVEY §8(f) row 1; not part of the §8(d) timed region)")
    ap.add_argument("--full-grid-steps", type=int, default=None,
                    help="timed steps of the full_grid block (both n_fft halves; default "
                         "min(steps, 5)); 0 skips the block")
    ap.add_argument("--dump-table", default=None,
                    help="rank 0 saves the last timed step's gathered records [cells, 2] "
                         "(sse, finite) by global cell id to this .npy (multi-rank tests)")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the sweep block (search.run_grid with alignment and STOI)")
    args = ap.parse_args()
    if args.pipeline < 1:
        ap.error("--pipeline must be >= 1")

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = "WORLD_SIZE" in os.environ  # launched by torchrun (any world size)
    if use_dist:
        # "nccl" is RCCL on ROCm; CSE_DIST_BACKEND=gloo rehearses the
        # multi-rank path with several ranks sharing one GPU (1-GPU boxes)
        dist.init_process_group(os.environ.get("CSE_DIST_BACKEND", "nccl"))
    torch.cuda.set_device(local % torch.cuda.device_count())
    from classical_speech_enhancement_amd.engine import Engine, snr_db
    from classical_speech_enhancement_amd.synth import make_pair
    nccl = use_dist and dist.get_backend() == "nccl"
    coll_dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    dist_ctx = (dist if use_dist else None, coll_dev, world)
    weak = args.pairs is not None

    pair_ids, local_specs, gids, total_units, total_pairs = rank_job(args, world, rank, args.nfft)
    eng = Engine()
    pairs = [make_pair(i, args.seconds) for i in pair_ids]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    clean_pow = np.array([float(np.dot(c, c)) for c, _ in pairs])
    job = TimedJob(eng, noisy, clean, local_specs, gids, 1 if args.no_overlap else args.pipeline,
                   args.align, dist_ctx)
    units = job.units
    dt, kern = job.run(args.steps, args.warmup)
    kern_ms = kern[0]
    clock = job.clock
    ranks = gather_rank_stats(dict(job.rank_stats, pairs=len(pair_ids)), dist_ctx)
    n_cells_job = len(grid_specs(1, args.nfft)) * total_pairs
    table = job.table(n_cells_job)
    if args.dump_table and rank == 0:
        np.save(args.dump_table, table)

    # sanity of the step's output: every cell finite, SNRs finite
    sse, fin = job.last_plans()[0].results()[:2]
    assert fin.all(), "non-finite enhanced output"
    snr_local = snr_db(sse, clean_pow[[s for (s, _, _) in local_specs]])
    assert np.isfinite(snr_local).all()
    del job

    # ---- full_grid: both n_fft halves of the HEAD grid per step (9,744 cells per pair)
    full = None
    fsteps = min(args.steps, 5) if args.full_grid_steps is None else args.full_grid_steps
    if fsteps > 0:
        f_ids, f_specs, f_gids, f_units, _ = rank_job(args, world, rank, None)
        f_pairs = [make_pair(i, args.seconds) for i in f_ids]
        f_clean = torch.as_tensor(np.stack([c for c, _ in f_pairs])).cuda()
        f_noisy = torch.as_tensor(np.stack([n for _, n in f_pairs])).cuda()
        fjob = TimedJob(eng, f_noisy, f_clean, f_specs, f_gids, 1 if args.no_overlap else args.pipeline,
                        False, dist_ctx)
        fdt, fkern = fjob.run(fsteps, 1)
        full = {"what": ("the whole HEAD grid per step: both n_fft halves (9,744 cells per pair, "
                         "all 4 algorithms, hops 128+256), STFT + noise PSDs + fused "
                         "gain/ISTFT/SNR per cell, records all-gathered; same sharding and timing "
                         "rules as the headline"),
                "value": f_units * fsteps / fdt, "unit": "frame-gain evals/s",
                "units_per_step": f_units, "cells_per_step": 9744 * total_pairs,
                "steps": fsteps, "warmup": 1, "ms_per_step": fdt / fsteps * 1e3,
                "kernel_ms": {str(p.n_fft): k for p, k in zip(fjob.mps[0].plans, fkern)},
                "units_per_launch_rank0": {str(p.n_fft): p.units for p in fjob.mps[0].plans},
                "roofline": {str(p.n_fft): roofline_block(p.n_fft, p.units, k)
                             for p, k in zip(fjob.mps[0].plans, fkern)}}
        del fjob, f_clean, f_noisy

    # ---- sweep: the reference's whole job (speech_enhancement_comparison.py:441-455 ->
    # :156-226) through search.run_grid: every cell aligned, SNR and STOI scored,
    # records gathered, both sequential selections
    sweep = None
    if not args.no_sweep:
        torch.cuda.empty_cache()  # the timed jobs' plans are gone: their memory goes back
        sweep = sweep_block(args, world, total_pairs, weak)

    # ---- parity on every rank: the pair it holds most cells of, stratified
    # cells' waveforms and the timed step's SNRs against the oracle; at N = 1
    # the CPU baseline runs in the same pool (rank 0 only)
    base, par = None, None
    want_base = rank == 0 and world == 1 and not args.no_cpu_baseline
    if not args.no_parity or want_base:
        slot, held = rank_pair_cells(local_specs, args.nfft)
        y_cells = [] if args.no_parity else pick_parity_cells(args.seconds, args.nfft, held)
        base, cpu_snr, cpu_y = cpu_run(args.cpu_budget, args.seconds, args.nfft, y_cells,
                                       timed=want_base, pair=pair_ids[slot])
        if y_cells:
            dev_snr = {g: float(snr_local[j]) for g, j in held.items()}
            par = parity_block(eng, noisy[slot:slot + 1], clean[slot:slot + 1], clean_pow[slot],
                               args.nfft, dev_snr, cpu_snr, cpu_y)
            par["pair"] = int(pair_ids[slot])
    par_all = gather_parity(par, dist_ctx) if not args.no_parity else None

    if rank != 0:
        if use_dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    value = total_units * args.steps / dt
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "frame-gain evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if weak else "strong",
        "vs_baseline": None,
        "dtype": ("f32 gain recursion + ISTFT + per-frame error sums; f64 STFT, noise PSDs, "
                  "cross-frame SNR sums, alignment re-evaluation and STOI"),
        "data": "synthetic",
        "config": {
            "workload": (f"{total_pairs} x 10-s 16-kHz synthetic pairs "
                         f"({'per GPU' if weak else 'in all, cells sharded over the GPUs'})"
                         f", HEAD parameter_ranges.py grid at n_fft={args.nfft} (all 4 algorithms, "
                         f"4872 cells/pair, hops 128+256): STFT + noise PSDs + fused "
                         f"gain/ISTFT/SNR per cell, records all-gathered"),
            "pairs_total": total_pairs, "clip_s": args.seconds, "sr": 16000, "n_fft": args.nfft,
            "cells_total": n_cells_job,
            "gathered_cells_finite": int(table[:, 1].sum()),
            "units_per_step": total_units, "units_per_step_rank0": units,
            "pairs_rank0": len(pair_ids),
            "parallelism": (f"{'pairs' if weak else 'contiguous cost-balanced cell shards'} over "
                            f"{world} rank(s), one all_gather_into_tensor of per-cell records per "
                            f"step ({'RCCL' if nccl else ('gloo' if use_dist else 'single process')})"),
            "finalize_alignment": bool(args.align),
        },
        "roofline": roofline_block(args.nfft, units, kern_ms),
        "clock": clock,
        "ranks": ranks,
    }
    if full is not None:
        res["full_grid"] = full
    if sweep is not None:
        res["sweep"] = sweep
    if base:
        res["cpu_baseline"] = base
    if par_all is not None:
        res["parity"] = dict(par or {}, **par_all)
    print(json.dumps(res))
    sys.stdout.flush()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    if "parity" in res and not res["parity"]["pass"]:
        sys.exit("parity check failed: " + json.dumps(res["parity"]))


def valu_calibration():
    """The chip-wide VALU rates the pricing rests on (tools/micro/valu_cal.hip,
    HIP-event timed, profiles/r06_micro_valu_cal.json): TFLOP/s and SIMD cycles
    per wave-instruction of dense independent streams at 8 and 3 waves/SIMD."""
    path = os.path.join(REPO, "profiles", "r06_micro_valu_cal.json")
    if not os.path.exists(path):
        return None
    rows = json.load(open(path))["rows"]
    out = {"source": "profiles/r06_micro_valu_cal.json (tools/micro/valu_cal.hip)"}
    for r in rows:
        if r["waves_per_simd"] in (3, 8):
            out[f'{r["op"]}@{r["waves_per_simd"]}w'] = {"TFLOPs": round(r["tflops"], 2),
                                                          "cycles_per_wave_inst": round(r["cycles_per_wave_inst"], 3)}
    mix = json.load(open(path)).get("mix") or {}
    keep = ("v_fma_f32(vvv) + v_fma_f32(vvv)", "v_add_f32 + v_add_f32", "v_fma_f32(vvv) + v_add_f32",
            "v_fma_f32(vvv) + v_max_f32", "v_fma_f32(vvv) + v_pk_fma_f32", "v_fma_f32(vvv) + v_exp_f32",
            "v_pk_fma_f32 + v_exp_f32", "v_fma_f32(vvv) + v_fma_f64")
    out["mix_cycles_per_wave_inst_8w"] = {k: mix[k].get("8") for k in keep if k in mix}
    return out


def roofline_block(n_fft, units, kern_ms):
    """The enhance kernel against the resource it spends: VALU lane-op throughput.

    The product binary's own instruction counts (PMC of this launch size and
    n_fft, committed under profiles/ and matched to this build by a digest of
    the kernel sources and flags), each priced at the SIMD cycles the
    chip-wide micro-benchmarks measure for its kind (VALU_CYC, PK_CYC,
    TRANS_CYC, F64_CYC: f32 VALU 2, packed v_pk_*_f32 4, transcendental 8,
    fp64 4), over the live HIP-event kernel time:
    `achieved` = those SIMD cycles per second, `peak` = 1024 SIMDs x 2.4 GHz.
    The packed count is measured (tools/pmc_summary.py: the F32 class counters
    of the scalar build CSE_PK=0 minus the product's, checked by the FLOP
    counter).  Beside it:
      fp32_flops   SQ_INSTS_VALU_FLOPS_FP32 (per wave-instruction, weighted by
                   the FLOPs of each lane: x 64) against the 157.3 TF FP32 peak;
      calibration  the chip-wide micro-benchmark of the per-instruction prices;
      traffic      the measured HBM bytes (PMC) and SURVEY 8(d)'s nominal
                   12 B/bin (read P, read N, write G) as a byte count only: the
                   fused kernel never writes G and reads the shared rows once per
                   16-cell workgroup, so those bytes are not moved and are not
                   a bandwidth."""
    bytes_per_unit = 12 * (n_fft // 2 + 1)
    ks = kern_ms / 1e3
    nominal = units * bytes_per_unit
    roof = {"bound": "valu",
            "bound_note": ("VALU throughput: every VALU instruction of the launch priced at the SIMD "
                           "cycles a dense stream of its kind takes on this part (f32 2, packed f32 4, "
                           "transcendental 8, f64 4 per wave64 instruction; tools/micro/valu_cal.hip, "
                           "valu_mix.hip); HBM traffic is 2 % of peak"),
            "achieved": None,
            "peak": SIMDS * CLOCK / 1e9,
            "unit": "G SIMD VALU cycles/s (1024 SIMDs x 2.4 GHz)", "frac": None, "traffic": None,
            "kernel": f"cse::enhance_kernel<{n_fft}>", "kernel_ms": kern_ms,
            "units_per_launch": units,
            "nominal_unfused_bytes_per_unit": bytes_per_unit,
            "nominal_unfused_bytes_per_launch": nominal,
            "nominal_unfused_note": ("SURVEY 8(d)'s 12 B/bin (P, N read, G written, f32) for an "
                                     "unfused gain kernel; the fused kernel does not move these "
                                     "bytes, so no bandwidth is derived from them"),
            "pmc_traffic_over_nominal": None,
            "hbm_measured_GBps": None, "hbm_measured_frac": None,
            "kernel_src_sha": kernel_src_sha(),
            "calibration": valu_calibration()}
    pmc = load_pmc(units, n_fft)
    if not pmc:
        roof["note"] = "no committed PMC profile for this launch size: VALU figures absent"
        return roof
    roof["pmc_source"] = pmc.get("source")
    roof["pmc_matches_build"] = pmc.get("kernel_src_sha") == roof["kernel_src_sha"]
    if not roof["pmc_matches_build"]:
        roof["note"] = ("the committed PMC profile was taken on other kernel sources: "
                        "VALU and traffic figures omitted")
        return roof
    tb = pmc.get("hbm_bytes_per_launch")
    if tb:
        roof["traffic"] = tb
        roof["hbm_measured_GBps"] = tb / ks / 1e9
        roof["hbm_measured_frac"] = tb / ks / HBM_PEAK
        roof["pmc_traffic_over_nominal"] = tb / nominal
    vi, tr = pmc.get("sq_insts_valu"), pmc.get("sq_insts_valu_trans")
    pk, f64 = pmc.get("packed_insts"), pmc.get("sq_insts_valu_f64") or 0.0
    if vi and tr is not None and pk is not None:
        need = VALU_CYC * (vi - tr - pk - f64) + PK_CYC * pk + TRANS_CYC * tr + F64_CYC * f64
        roof["achieved"] = need / ks / 1e9
        roof["frac"] = need / ks / (SIMDS * CLOCK)
        roof["valu_cycles_per_launch"] = need
        roof["valu_insts"] = vi
        roof["packed_insts"] = pk
        roof["trans_insts"] = tr
        roof["f64_insts"] = f64
        roof["cycles_per"] = {"f32_valu": VALU_CYC, "packed_f32": PK_CYC, "transcendental": TRANS_CYC,
                              "f64": F64_CYC}
        guide = need - (TRANS_CYC - GUIDE_TRANS_CYC) * tr
        roof["frac_transcendental_at_4"] = guide / ks / (SIMDS * CLOCK)
        if pmc.get("packed"):
            roof["packed_source"] = {k: pmc["packed"].get(k) for k in ("add", "mul", "fma", "flop_check",
                                                                        "valu_difference")}
        clk = pmc.get("clock_ghz_profiled")
        if clk:
            roof["clock_ghz_profiled"] = clk
            roof["frac_at_held_clock"] = need / ks / (SIMDS * clk * 1e9)
        fl = pmc.get("sq_insts_valu_flops_fp32")
        if fl:
            roof["fp32_flops"] = {"achieved_TFLOPs": fl * 64 / ks / 1e12,
                                  "peak_TFLOPs": FP32_PEAK / 1e12,
                                  "frac": fl * 64 / ks / FP32_PEAK,
                                  "counter": ("SQ_INSTS_VALU_FLOPS_FP32 x 64: the counter counts per "
                                              "wave-instruction, weighted by FLOPs per lane")}
        for k in ("share_wait_inst_any", "share_wait_any", "share_wait_inst_lds",
                  "share_active_inst_valu", "share_active_inst_any",
                  "lds_array_busy", "lds_conflict_cycles_per_lds_inst", "vgprs", "waves_per_simd"):
            if pmc.get(k) is not None:
                roof[k] = pmc[k]
    elif vi:
        roof["note"] = "the committed PMC profile has no packed-instruction count: VALU figures omitted"
    return roof


def sweep_block(args, world, total_pairs, weak):
    """search.run_grid over the whole job: pairs x 9,744 cells, alignment + SNR
    + STOI, one all_gather, sequential selections.  One warm call (plans
    allocated), then one timed call bracketed by barrier + synchronize, max over
    ranks."""
    import torch
    import torch.distributed as dist
    from classical_speech_enhancement_amd import search
    from classical_speech_enhancement_amd.engine import Engine
    from classical_speech_enhancement_amd.synth import make_pair
    pairs = [make_pair(i, args.seconds) for i in range(total_pairs)]
    clean = [c for c, _ in pairs]
    noisy = [n for _, n in pairs]
    specs = search.job_specs(total_pairs)
    seng = Engine()
    # every batch structure of the job stays cached between calls: the STOI
    # path alternates two plans for the full batches, plus the last, shorter
    # batch (3 plans; 2 made the timed call rebuild plans, +0.48 s of 1.6 s)
    seng.plan_cache_size = 4

    def compute(c, n, s, ids):
        return search.engine_compute(c, n, s, ids, engine=seng)
    use_dist = dist.is_available() and dist.is_initialized()
    search.run_grid(clean, noisy, specs, compute=compute)  # warm: plans allocated
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    table, best = search.run_grid(clean, noisy, specs, compute=compute)
    best_stoi = search.select_best(specs, table, "stoi")
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([dt], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    L = int(round(args.seconds * 16000))
    units = sum(1 + L // int(p["hop_length"]) for (_, _, p) in specs[:specs.per_pair]) * total_pairs
    st = table[:, 5].astype(np.int64)
    out = {"what": ("search.run_grid over the whole job (speech_enhancement_comparison.py:"
                    "441-455 -> 156-226): STFT, noise PSDs, fused enhance of every cell, "
                    "finalize_enhanced alignment (xcorr lag, lag-shifted rescoring), SNR and "
                    "STOI of every cell, one all_gather of the records, the sequential SNR "
                    "and STOI selections; host-resident pairs in, winners out (second call: "
                    "device plans reused)"),
           "pairs": total_pairs, "cells": len(specs), "units": units, "wall_s": dt,
           "cells_per_s": len(specs) / dt, "units_per_s": units / dt,
           "cells_computed": "min_tracking cells that differ only in noise_percentile are "
                             "computed once and their rows copied (a quarter of the grid)",
           "finite_cells": int(table[:, 2].sum()),
           "xcorr_status": {"ok": int((st == 0).sum()), "flat": int((st == 1).sum()),
                            "nonfinite": int((st == 2).sum())},
           "nonzero_lags": int((table[:, 4] != 0).sum()),
           "stoi_batch_wave_bytes": search.stoi_wave_bytes(),
           "winners": {"snr": sum(1 for v in best.values() if v[0] >= 0),
                       "stoi": sum(1 for v in best_stoi.values() if v[0] >= 0),
                       "groups": len(best)}}
    del seng
    return out


def rank_pair_cells(local_specs, n_fft):
    """(slot, {grid index: local cell index}) for the pair this rank holds most
    cells of; grid indices into grid_specs(1, n_fft)."""
    index = {(alg, tuple(p.items())): g for g, (_, alg, p) in enumerate(grid_specs(1, n_fft))}
    by_slot = {}
    for j, (s, alg, p) in enumerate(local_specs):
        by_slot.setdefault(s, {})[index[(alg, tuple(p.items()))]] = j
    slot = max(sorted(by_slot), key=lambda s: len(by_slot[s]))
    return slot, by_slot[slot]


def pick_parity_cells(seconds, n_fft, held):
    """The stratified parity cells this rank holds; when it holds few of them
    (a partial pair at a shard end), 64 of its held cells at random instead."""
    cells = [g for g in parity_cells(seconds, n_fft) if g in held]
    if len(cells) < 16:
        rng = np.random.default_rng(7)
        hs = sorted(held)
        cells = sorted(rng.choice(hs, min(64, len(hs)), replace=False).tolist())
    return cells


def parity_block(eng, noisy1, clean1, clean_pow1, n_fft, dev_snr, cpu_snr, cpu_y):
    """Device vs oracle on one pair: the timed step's SNR of every cell the
    oracle computed (dev_snr: grid index -> device SNR), and the waveforms of
    the stratified cells (recomputed through the same kernel, one launch)."""
    from classical_speech_enhancement_amd.engine import snr_db
    specs0 = grid_specs(1, n_fft)
    ids = sorted(i for i in cpu_snr if i in dev_snr)
    snr_err = max(abs(dev_snr[i] - cpu_snr[i]) for i in ids) if ids else None
    y_ids = sorted(cpu_y)
    res = eng.run(noisy1, [(0, specs0[i][1], specs0[i][2]) for i in y_ids], clean=clean1,
                  want_waveforms=True)
    yd = res["y"].double().cpu().numpy()
    e2 = em = 0.0
    for j, i in enumerate(y_ids):
        ref = cpu_y[i]
        e2 = max(e2, float(np.linalg.norm(yd[j] - ref) / np.linalg.norm(ref)))
        em = max(em, float(np.max(np.abs(yd[j] - ref)) / np.max(np.abs(ref))))
    # the re-run cells give the timed step's SNR exactly (no cell depends on its batch)
    rerun_same = bool(np.array_equal(snr_db(res["sse"], clean_pow1),
                                      np.array([dev_snr[i] for i in y_ids]))) if y_ids else None
    ok = (e2 <= TOL and em <= TOL and (snr_err is None or snr_err <= SNR_TOL_DB)
          and rerun_same is not False)
    return {"cells_snr": len(ids), "max_snr_abs_db": snr_err, "snr_tol_db": SNR_TOL_DB,
            "cells_waveform": len(y_ids), "max_rel_l2": e2, "max_rel_max": em, "tol": TOL,
            "waveform_cells_from_timed_launch_snr_identical": rerun_same,
            "strata": ("4 cells per (algorithm, hop, noise method) of the n_fft grid of the pair "
                       "the rank holds most cells of"),
            "pass": bool(ok)}


PARITY_FIELDS = ("pass", "pair", "cells_snr", "cells_waveform", "max_rel_l2", "max_rel_max",
                 "max_snr_abs_db")


def gather_parity(par, dist_ctx):
    """Every rank's parity summary on every rank (one all_gather): the line is
    self-verifying at N > 1 too; "pass" holds only if every rank passed."""
    import torch
    dist, coll_dev, world = dist_ctx
    nan = float("nan")
    v = torch.tensor([nan if par is None or par.get(k) is None else float(par[k])
                      for k in PARITY_FIELDS], dtype=torch.float64)
    if dist is not None:
        out = torch.empty(world * len(PARITY_FIELDS), dtype=torch.float64, device=coll_dev)
        dist.all_gather_into_tensor(out, v.to(coll_dev))
        v = out.cpu()
    rows = v.numpy().reshape(-1, len(PARITY_FIELDS))
    per = []
    for r in rows:
        d = {k: (None if np.isnan(x) else x) for k, x in zip(PARITY_FIELDS, r.tolist())}
        d["pass"] = d["pass"] == 1.0
        for k in ("pair", "cells_snr", "cells_waveform"):
            d[k] = None if d[k] is None else int(d[k])
        per.append(d)
    return {"per_rank": per, "pass": all(d["pass"] for d in per),
            "ranks_checked": sum(1 for d in per if d["cells_waveform"])}


if __name__ == "__main__":
    main()
