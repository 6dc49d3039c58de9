"""End-to-end sweep timing on one GPU (GPU box): the reference's main() loop
body for P synthetic 10-s pairs x the full HEAD grid (both n_fft halves, all
four algorithms, 9,744 cells per pair): STFT + noise PSDs + fused enhance,
finalize_enhanced alignment and rescoring, STOI and SNR per cell, and the
sequential selections — search.run_grid on one rank.

    python tools/bench_sweep.py [--pairs P --reps R]

Prints one JSON line: wall time per sweep with and without STOI, cells/s.
"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from classical_speech_enhancement_amd import search  # noqa: E402
from classical_speech_enhancement_amd.engine import Engine  # noqa: E402
from classical_speech_enhancement_amd.synth import make_pair  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--profile", action="store_true", help="cProfile the timed STOI sweeps (host side)")
    ap.add_argument("--wave-gb", type=float, default=None,
                    help="override search.STOI_WAVE_BYTES (GiB of cell waveforms per STOI batch)")
    a = ap.parse_args()
    if a.wave_gb is not None:
        search.STOI_WAVE_BYTES = int(a.wave_gb * (1 << 30))
    import torch
    pairs = [make_pair(200 + i, a.seconds) for i in range(a.pairs)]
    clean = [c for c, _ in pairs]
    noisy = [n for _, n in pairs]
    specs = search.job_specs(a.pairs)
    eng = Engine()
    eng.plan_cache_size = 4  # every batch structure stays cached between the timed calls
    out = {"pairs": a.pairs, "clip_s": a.seconds, "cells": len(specs)}
    for stoi in (False, True):
        if stoi:
            # a fresh engine, like bench.py's sweep block: with the SNR-only
            # plans still cached, the STOI batches shrank to the memory left
            # (19 instead of 10 batches) and the first two missed the plan
            # cache (1.57 s instead of 1.27 s per 100-pair sweep, r05)
            del eng
            torch.cuda.empty_cache()
            eng = Engine()
            eng.plan_cache_size = 4

        def compute(c, n, s, ids):
            return search.engine_compute(c, n, s, ids, engine=eng, stoi=stoi)
        search.run_grid(clean, noisy, specs, compute=compute)  # warm-up
        torch.cuda.synchronize()
        ts = []
        prof = None
        if a.profile and stoi:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        for _ in range(a.reps):
            t0 = time.perf_counter()
            table, best = search.run_grid(clean, noisy, specs, compute=compute)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        if prof is not None:
            import pstats
            prof.disable()
            pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(40)
            pstats.Stats(prof, stream=sys.stderr).sort_stats("tottime").print_stats(30)
        key = "with_stoi" if stoi else "snr_only"
        out[key] = {"s_per_sweep": float(np.median(ts)), "cells_per_s": len(specs) / float(np.median(ts))}
        if stoi:
            sb = search.select_best(specs, table, "stoi")
            out["stoi_winner_mean"] = float(np.mean([v[1] for v in sb.values()]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
