#!/usr/bin/env python
"""bench.py — STFT frame-gain evaluations/s on MI355X (BASELINE.json metric).

Workload (one "step"): for P (default 13) synthetic 10-s 16-kHz pairs per GPU, the n_fft=512
half of the reference's full HEAD grid (parameter_ranges.py: SS 360 + MMSE 960
+ Wiener 96 + OMLSA 3456 = 4872 cells per pair, hops 128 and 256):
  STFT + noise PSDs (percentile 10/20, min-tracking, smoothing)   [per pair]
  fused gain recursion + ISTFT + clipped-SNR sums, every cell     [THE HOT PATH]
  per-cell records (sse, finite) -> host, all-gathered over ranks [results table]
Unit = one frame-gain evaluation = one cell x one STFT frame, all 257 bins
(SURVEY §8(d)): 4,572,372 per pair.  Every cell is counted, including the
quarter that are exact duplicates (min_tracking ignores noise_percentile).

Multi-GPU: one process per GPU (torchrun), pairs sharded across ranks (weak
scaling, no data-path collective); value = all ranks' units / max-rank time.

    python bench.py [--gpus N --steps K --warmup W --pairs P]
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
BYTES_PER_UNIT_512 = 12 * 257  # read P + read N + write G, fp32, per frame
HBM_PEAK = 8.0e12              # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK = 157.3e12


from classical_speech_enhancement_amd.parameter_ranges import grid_specs  # noqa: E402


def _cpu_cell(args):
    alg, params, seconds = args
    import oracle
    from classical_speech_enhancement_amd.synth import make_pair
    clean, noisy = _cpu_cell.pair if hasattr(_cpu_cell, "pair") else (None, None)
    if clean is None:
        clean, noisy = make_pair(0, seconds)
        _cpu_cell.pair = (clean, noisy)
    kw = dict(params)
    if kw["noise_method"] == "true_noise":
        kw["clean_audio"] = clean
    fn = oracle.ALGORITHMS[alg]
    y = fn(noisy, 16000, **kw)
    e = np.clip(y, -1, 1)
    oracle.calculate_snr(clean, e)
    return 1 + int(len(noisy)) // int(params["hop_length"])


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(budget_s=15.0, seconds=10.0, n_fft=512):
    """The oracle (the reference's algorithm restated, fp64, per-frame Python
    loops, one STFT+estimate per cell exactly like the reference) on the host
    cores, over cells drawn uniformly at random from the same grid, for a fixed
    wall-clock budget.  Returns frame-gain evals/s."""
    import multiprocessing as mp
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(16, cores))
    specs = grid_specs(1, n_fft)
    rng = np.random.default_rng(0)
    order = rng.permutation(len(specs))
    work = [(specs[i][1], specs[i][2], seconds) for i in order]
    env_keys = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")
    saved = {k: os.environ.get(k) for k in env_keys}
    for k in env_keys:
        os.environ[k] = "1"
    ctx = mp.get_context("spawn")
    units = cells = 0
    try:
        with ctx.Pool(cores) as pool:
            # warm the workers (imports + synth) outside the window
            list(pool.imap_unordered(_cpu_cell, work[:cores]))
            t0 = time.perf_counter()
            it = pool.imap_unordered(_cpu_cell, work[cores:] * 4, chunksize=1)
            for u in it:
                units += u
                cells += 1
                if time.perf_counter() - t0 > budget_s:
                    break
            dt = time.perf_counter() - t0
            pool.terminate()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {"value": units / dt, "unit": "frame-gain evals/s", "cores": cores, "kind": "port",
            "cpu_model": _cpu_model(),
            "sample": (f"{cells} cells drawn uniformly from the n_fft={n_fft} HEAD grid, "
                       f"one 10-s pair, oracle/ fp64 numpy (reference algorithm incl. per-cell "
                       f"STFT+noise estimate), {cores} single-threaded processes, "
                       f"{dt:.1f} s wall")}


def load_traffic(units_per_launch):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if d.get("units_per_launch") == units_per_launch:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=13,
                    help="10-s pairs per GPU (13 x 8 GPUs = 104 >= the 100 pairs of config 4)")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
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
    if world > 1:
        # "nccl" is RCCL on ROCm; CSE_DIST_BACKEND=gloo rehearses the
        # multi-rank path with several ranks sharing one GPU (1-GPU boxes)
        dist.init_process_group(os.environ.get("CSE_DIST_BACKEND", "nccl"))
    torch.cuda.set_device(local % torch.cuda.device_count())
    from classical_speech_enhancement_amd.engine import Engine, snr_db
    from classical_speech_enhancement_amd.synth import make_pair

    eng = Engine()
    P = args.pairs
    pairs = [make_pair(rank * P + i, args.seconds) for i in range(P)]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    clean_pow = np.array([float(np.dot(c, c)) for c, _ in pairs])
    L = noisy.shape[1]
    specs = grid_specs(P, args.nfft)
    # Two plans, double-buffered: the next step's STFT + noise PSDs run on a
    # side stream while this step's enhance kernel runs (no data is shared
    # between a step's prep and the previous step's enhance).
    n_buf = 1 if args.no_overlap else 2
    mps = [eng.plan(P, L, specs, with_clean=True, align=args.align) for _ in range(n_buf)]
    plans = [m.plans[0] for m in mps]
    units = mps[0].units
    main_s = torch.cuda.current_stream()
    prep_s = torch.cuda.Stream() if n_buf > 1 else main_s
    ev_prep = [torch.cuda.Event() for _ in range(n_buf)]
    ev_done = [None] * n_buf
    counter = [0]

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
        rec = torch.stack([plan.sse_d, plan.fin_d.double()])
        if world > 1:
            if dist.get_backend() == "gloo":
                rec = rec.cpu()
            out = torch.empty((world * rec.shape[0],) + rec.shape[1:], dtype=rec.dtype,
                              device=rec.device)
            dist.all_gather_into_tensor(out, rec.contiguous())
            rec = out.view((world,) + rec.shape)
        return rec.cpu()

    if n_buf > 1:
        prep(0)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        rec = step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64,
                         device="cpu" if dist.get_backend() == "gloo" else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))

    # sanity of the step's output: every cell finite, SNRs finite
    sse, fin = plans[(counter[0] - 1) % n_buf].results()[:2]
    if not os.environ.get("CSE_BENCH_NOCHECK"):  # set only for timing-only ablation builds
        assert fin.all(), "non-finite enhanced output"
        snr = snr_db(sse, clean_pow[[s for (s, _, _) in specs]])
        assert np.isfinite(snr).all()

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    total_units = units * world * args.steps
    value = total_units / dt
    bytes_per_unit = 12 * (args.nfft // 2 + 1)
    achieved = units * bytes_per_unit / (kern_ms / 1e3)
    traffic = load_traffic(units)
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "frame-gain evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": (f"{P} x 10-s 16-kHz synthetic pairs per GPU, HEAD parameter_ranges.py "
                         f"grid at n_fft={args.nfft} (all 4 algorithms, 4872 cells/pair, hops 128+256): "
                         f"STFT+noise PSDs+fused gain/ISTFT/SNR per cell"),
            "pairs_per_gpu": P, "clip_s": args.seconds, "sr": 16000, "n_fft": args.nfft,
            "cells_per_gpu": len(specs), "units_per_step_per_gpu": units,
            "parallelism": f"pairs sharded over {world} rank(s), all_gather of per-cell records",
            "finalize_alignment": bool(args.align),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic,
            "kernel": f"cse::enhance_kernel<{args.nfft}>", "kernel_ms": kern_ms,
            "bytes_per_unit": bytes_per_unit, "units_per_launch": units,
        },
    }
    if not args.no_cpu_baseline and world == 1:
        res["cpu_baseline"] = cpu_baseline(args.cpu_budget, args.seconds, args.nfft)
    print(json.dumps(res))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
