"""Does the STOI kernel overlap with the enhance kernel? (GPU box, analysis only)

Times one enhance launch (bench workload, --pairs pairs at n_fft 512) and one
STOI launch (--cells 10-s cells) alone, back to back on one stream, and
concurrently on two streams.

    python tools/overlap_probe.py [--pairs 4 --cells 8192 --reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--cells", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from classical_speech_enhancement_amd.engine import Engine
    from classical_speech_enhancement_amd.metrics import StoiPlan
    from classical_speech_enhancement_amd.parameter_ranges import grid_specs
    from classical_speech_enhancement_amd.synth import make_pair

    L = 160000
    pairs = [make_pair(i, 10.0) for i in range(a.pairs)]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    eng = Engine()
    mp = eng.plan(a.pairs, L, grid_specs(a.pairs, 512), with_clean=True)
    plan = mp.plans[0]
    plan.prepare(noisy, clean)

    rng = np.random.default_rng(0)
    sig = np.arange(a.cells) % a.pairs
    gains = torch.as_tensor(rng.uniform(0.3, 3.0, a.cells).astype(np.float32)).cuda()
    y = (noisy.float()[torch.as_tensor(sig).cuda()] * gains[:, None]).contiguous().view(-1)
    lag = rng.integers(-1600, 1601, a.cells)
    off = np.arange(a.cells, dtype=np.int64) * L
    sp = StoiPlan(clean)
    side = torch.cuda.Stream()

    def run(mode):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode in ("enhance", "serial", "concurrent"):
            plan.enhance()
        if mode in ("stoi", "serial"):
            sp.score_async(y, off, sig, lag=lag)
        if mode == "concurrent":
            with torch.cuda.stream(side):
                sp.score_async(y, off, sig, lag=lag)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for m in ("enhance", "stoi"):
        run(m)  # warm-up
    out = {}
    for m in ("enhance", "stoi", "serial", "concurrent"):
        out[m + "_ms"] = float(np.median([run(m) for _ in range(a.reps)]))
    out["cells_enhance"] = int(plan.n_packed)
    out["cells_stoi"] = a.cells
    print(json.dumps(out))


if __name__ == "__main__":
    main()
