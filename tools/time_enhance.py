"""Kernel time of one enhance launch (bench workload, no output checks): for
timing-only variant builds whose outputs are wrong by construction.

    CSE_LIB=... python tools/time_enhance.py [--pairs 13 --nfft 512 --reps 5]
                                             [--hop-map 128:32,256:64]

--hop-map moves the grid's cells to other hops (here the short hops of
cse_enhance_cells_short_hop); the line then also gives frame-gain evals/s.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=13)
    ap.add_argument("--nfft", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--hop-map", default="")
    a = ap.parse_args()
    hop_map = dict(tuple(int(v) for v in kv.split(":")) for kv in a.hop_map.split(",") if kv)
    import torch
    from classical_speech_enhancement_amd.engine import Engine
    from classical_speech_enhancement_amd.parameter_ranges import grid_specs
    from classical_speech_enhancement_amd.synth import make_pair
    pairs = [make_pair(i, 10.0) for i in range(a.pairs)]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    specs = [(s, alg, dict(p, hop_length=hop_map.get(p["hop_length"], p["hop_length"])))
             for (s, alg, p) in grid_specs(a.pairs, a.nfft)]
    plan = Engine().plan(a.pairs, 160000, specs, with_clean=True).plans[0]
    plan.prepare(noisy, clean)
    plan.enhance()
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.enhance()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    med = float(np.median(ms))
    print(json.dumps({"lib": os.environ.get("CSE_LIB", "libcse.so"), "n_fft": a.nfft,
                      "hop_map": hop_map, "kernel_ms": med, "units": plan.units,
                      "evals_per_s": plan.units / (med * 1e-3)}))


if __name__ == "__main__":
    main()
