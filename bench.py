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
           cells sharded over the ranks by search.assign_lpt (the sweep
           driver's greedy LPT over (pair, n_fft, hop, algorithm) items);
           "scaling": "strong", value = 100 pairs' units / max-rank time.
  --pairs P: P pairs per GPU ("scaling": "weak").
Every step ends with one all_gather_into_tensor of the per-cell records.

At N = 1 the line also carries
  parity        the timed step's per-cell SNR table of pair 0 against the
                oracle on every cell the CPU baseline computed, and the
                waveforms of 64 cells stratified over algorithm x hop x noise
                method against the oracle (north-star: rel-L2 and rel-max
                <= 1e-5); the run fails above tolerance;
  cpu_baseline  the oracle on this host's cores (see cpu_baseline()).

    python bench.py [--gpus N --steps K --warmup W --pairs-total 100 | --pairs P]
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
VALU_CYC, TRANS_CYC = 2, 4     # wave64 issue cycles: v_fma_f32 (SIMD-32), transcendental (2x: tools/micro/valu_rate.hip)
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
    idx, alg, params, seconds, want_y = args
    import oracle
    from classical_speech_enhancement_amd.synth import make_pair
    if getattr(_cpu_cell, "seconds", None) != seconds:
        _cpu_cell.pair = make_pair(0, seconds)
        _cpu_cell.seconds = seconds
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


def cpu_run(budget_s, seconds, n_fft, y_cells, timed=True):
    """Run the oracle on the host cores: first the y_cells (waveforms kept for
    the parity check), then (timed) cells drawn uniformly at random from the
    pair-0 grid until budget_s of wall time.  Returns (baseline dict or None,
    {cell: snr}, {cell: y})."""
    import multiprocessing as mp
    procs, aff, ncpu = _cpu_share()
    specs = grid_specs(1, n_fft)
    rng = np.random.default_rng(0)
    want = set(y_cells)
    order = [i for i in rng.permutation(len(specs)).tolist() if i not in want]
    work = [(i, specs[i][1], specs[i][2], seconds, i in want) for i in list(y_cells) + order]
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
            list(pool.imap_unordered(_cpu_cell, [(0, w[1], w[2], seconds, False)
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
    tools/pmc_summary.py; the newest round wins)."""
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
    ap.add_argument("--no-overlap", action="store_true",
                    help="run each step's prep and enhance back to back on one stream")
    ap.add_argument("--align", action="store_true",
                    help="also run finalize_enhanced's alignment (xcorr lag + lag-shifted rescoring)"
                         " inside the step (SURVEY §8(f) row 1; not part of the §8(d) timed region)")
    args = ap.parse_args()

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
    from classical_speech_enhancement_amd import search
    from classical_speech_enhancement_amd.engine import Engine, n_frames, snr_db
    from classical_speech_enhancement_amd.synth import make_pair
    nccl = use_dist and dist.get_backend() == "nccl"
    coll_dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")

    L = int(round(args.seconds * 16000))
    if args.pairs is not None:   # weak: P pairs per rank
        weak = True
        pair_ids = [rank * args.pairs + i for i in range(args.pairs)]
        local_specs = grid_specs(args.pairs, args.nfft)
        total_pairs = args.pairs * world
    else:                        # strong: the fixed job, cells sharded by LPT
        weak = False
        total_pairs = args.pairs_total
        all_specs = grid_specs(total_pairs, args.nfft)
        rank_of, _ = search.assign_lpt(all_specs, [L] * total_pairs, world)
        mine = np.nonzero(rank_of == rank)[0]
        pair_ids = sorted({all_specs[c][0] for c in mine})
        slot = {p: s for s, p in enumerate(pair_ids)}
        local_specs = [(slot[all_specs[c][0]], all_specs[c][1], all_specs[c][2]) for c in mine]
    total_units = sum(n_frames(L, p["hop_length"]) for p in
                      (s[2] for s in grid_specs(1, args.nfft))) * total_pairs

    eng = Engine()
    pairs = [make_pair(i, args.seconds) for i in pair_ids]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    clean_pow = np.array([float(np.dot(c, c)) for c, _ in pairs])
    # Two plans, double-buffered: the next step's STFT + noise PSDs run on a
    # side stream while this step's enhance kernel runs (no data is shared
    # between a step's prep and the previous step's enhance).
    n_buf = 1 if args.no_overlap else 2
    mps = [eng.plan(len(pairs), L, local_specs, with_clean=True, align=args.align)
           for _ in range(n_buf)]
    plans = [m.plans[0] for m in mps]
    units = mps[0].units
    main_s = torch.cuda.current_stream()
    prep_s = torch.cuda.Stream() if n_buf > 1 else main_s
    ev_prep = [torch.cuda.Event() for _ in range(n_buf)]
    ev_done = [None] * n_buf
    counter = [0]
    # records of every rank, padded to the largest shard: one all_gather per step
    n_rec = plans[0].n_packed
    if use_dist:
        t = torch.tensor([n_rec], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n_rec = int(t.item())
    rec_pad = torch.zeros((2, n_rec), dtype=torch.float64, device="cuda")
    rec_all = torch.empty((world * 2, n_rec), dtype=torch.float64, device=coll_dev)

    def prep(k):
        b = k % n_buf
        with torch.cuda.stream(prep_s):
            if ev_done[b] is not None:
                prep_s.wait_event(ev_done[b])  # the enhance that last read these buffers
            plans[b].prepare(noisy, clean)
            ev_prep[b].record(prep_s)

    def step(ev=None):
        k = counter[0]
        counter[0] += 1
        b = k % n_buf
        plan = plans[b]
        if n_buf == 1:
            prep(k)
        main_s.wait_event(ev_prep[b])
        if ev is not None:
            ev[0].record()
        plan.enhance()
        if ev is not None:
            ev[1].record()
        if args.align:
            plan.finalize()
        ev_done[b] = torch.cuda.Event()
        ev_done[b].record(main_s)
        if n_buf > 1:
            prep(k + 1)  # overlaps this step's enhance (the timed region holds K preps)
        m = plan.n_packed
        rec_pad[0, :m] = plan.sse_d
        rec_pad[1, :m] = plan.fin_d
        if use_dist:
            dist.all_gather_into_tensor(rec_all, rec_pad.to(coll_dev))
            return rec_all.cpu()
        return rec_pad.cpu()

    if n_buf > 1:
        prep(0)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))

    # sanity of the step's output: every cell finite, SNRs finite
    last = plans[(counter[0] - 1) % n_buf]
    sse, fin = last.results()[:2]
    assert fin.all(), "non-finite enhanced output"
    snr_local = snr_db(sse, clean_pow[[s for (s, _, _) in local_specs]])
    assert np.isfinite(snr_local).all()

    if rank != 0:
        if use_dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    value = total_units * args.steps / dt
    bytes_per_unit = 12 * (args.nfft // 2 + 1)
    achieved = units * bytes_per_unit / (kern_ms / 1e3)
    pmc = load_pmc(units, args.nfft)
    roof = {
        "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
        "frac": achieved / HBM_PEAK, "traffic": None,
        "kernel": f"cse::enhance_kernel<{args.nfft}>", "kernel_ms": kern_ms,
        "bytes_per_unit": bytes_per_unit, "units_per_launch": units,
        "note": ("frac is SURVEY §8(d)'s algorithmic-byte roofline (12 B per bin per unit). "
                 "The kernel is fused: its HBM traffic ('traffic', PMC) is a few % of those "
                 "bytes, and VALU issue ('valu') is the resource it actually spends"),
    }
    if pmc:
        roof["traffic"] = pmc.get("hbm_bytes_per_launch")
        vi, tr = pmc.get("sq_insts_valu"), pmc.get("sq_insts_valu_trans")
        if vi:
            need = VALU_CYC * (vi - (tr or 0)) + TRANS_CYC * (tr or 0)  # SIMD issue cycles
            v = {"insts_valu": vi, "insts_trans": tr, "issue_cycles": need,
                 "frac_at_2p4ghz": need / (SIMDS * CLOCK * kern_ms / 1e3),
                 "cycles_per": f"VALU {VALU_CYC}, transcendental {TRANS_CYC} per wave64 per SIMD",
                 "source": pmc.get("source")}
            busy = pmc.get("sq_busy_cycles")
            if busy:  # per-SE cycles with waves resident (summed over 32 SEs): the clock held
                cyc = busy / 32
                v["clock_ghz"] = cyc / (pmc["kernel_ms"] / 1e3) / 1e9
                v["frac"] = need / (SIMDS * cyc)
            roof["valu"] = v
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
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": (f"{total_pairs} x 10-s 16-kHz synthetic pairs "
                         f"({'per GPU' if weak else 'in all, cells sharded over the GPUs by LPT'})"
                         f", HEAD parameter_ranges.py grid at n_fft={args.nfft} (all 4 algorithms, "
                         f"4872 cells/pair, hops 128+256): STFT + noise PSDs + fused "
                         f"gain/ISTFT/SNR per cell, records all-gathered"),
            "pairs_total": total_pairs, "clip_s": args.seconds, "sr": 16000, "n_fft": args.nfft,
            "cells_total": len(grid_specs(1, args.nfft)) * total_pairs,
            "units_per_step": total_units, "units_per_step_rank0": units,
            "pairs_rank0": len(pair_ids),
            "parallelism": (f"{'pairs' if weak else 'LPT cell shards'} over {world} rank(s), "
                            f"one all_gather_into_tensor of per-cell records per step "
                            f"({'RCCL' if nccl else ('gloo' if use_dist else 'single process')})"),
            "finalize_alignment": bool(args.align),
        },
        "roofline": roof,
    }
    if world == 1:
        # pair 0 is the CPU's pair: its grid is this plan's first cells
        y_cells = [] if args.no_parity else parity_cells(args.seconds, args.nfft)
        base, cpu_snr, cpu_y = None, {}, {}
        if not args.no_cpu_baseline or y_cells:
            base, cpu_snr, cpu_y = cpu_run(args.cpu_budget, args.seconds, args.nfft, y_cells,
                                           timed=not args.no_cpu_baseline)
        if base:
            res["cpu_baseline"] = base
        if y_cells:
            res["parity"] = parity_block(eng, noisy, clean, clean_pow, args.nfft, snr_local,
                                         cpu_snr, cpu_y, weak)
    print(json.dumps(res))
    sys.stdout.flush()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    if "parity" in res and not res["parity"]["pass"]:
        sys.exit("parity check failed: " + json.dumps(res["parity"]))


def parity_block(eng, noisy, clean, clean_pow, n_fft, snr_local, cpu_snr, cpu_y, weak):
    """Device vs oracle on pair 0 (the CPU baseline's pair): the timed step's
    SNR of every cell the oracle computed, and the waveforms of the stratified
    cells (recomputed through the same kernel, one launch)."""
    from classical_speech_enhancement_amd.engine import snr_db
    specs0 = grid_specs(1, n_fft)
    # the plan's first len(specs0) cells are pair 0's grid in grid order (both modes at N=1)
    d_snr = snr_local[:len(specs0)]
    ids = sorted(cpu_snr)
    snr_err = max(abs(d_snr[i] - cpu_snr[i]) for i in ids) if ids else None
    y_ids = sorted(cpu_y)
    res = eng.run(noisy[:1], [(0, specs0[i][1], specs0[i][2]) for i in y_ids], clean=clean[:1],
                  want_waveforms=True)
    yd = res["y"].double().cpu().numpy()
    e2 = em = 0.0
    for j, i in enumerate(y_ids):
        ref = cpu_y[i]
        e2 = max(e2, float(np.linalg.norm(yd[j] - ref) / np.linalg.norm(ref)))
        em = max(em, float(np.max(np.abs(yd[j] - ref)) / np.max(np.abs(ref))))
    # the re-run cells give the timed step's SNR exactly (no cell depends on its batch)
    rerun_same = bool(np.array_equal(snr_db(res["sse"], clean_pow[0]),
                                      d_snr[y_ids])) if y_ids else None
    ok = (e2 <= TOL and em <= TOL and (snr_err is None or snr_err <= SNR_TOL_DB)
          and rerun_same is not False)
    return {"cells_snr": len(ids), "max_snr_abs_db": snr_err, "snr_tol_db": SNR_TOL_DB,
            "cells_waveform": len(y_ids), "max_rel_l2": e2, "max_rel_max": em, "tol": TOL,
            "waveform_cells_from_timed_launch_snr_identical": rerun_same,
            "strata": "4 cells per (algorithm, hop, noise method) of pair 0's n_fft grid",
            "pass": bool(ok)}


if __name__ == "__main__":
    main()
