"""Kernel times of one plan's analysis chain pieces on the bench workload
(100 x 10-s pairs, n_fft 512): the whole prepare() and each hop's batched
cse_noise_finish launch, HIP events, median of R runs.  For A/B of noise-kernel
variants (CSE_LIB=...).

    python tools/time_noise.py [--pairs 100 --reps 5]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from classical_speech_enhancement_amd import _lib
    from classical_speech_enhancement_amd.engine import Engine, _ptr, _stream
    from classical_speech_enhancement_amd.parameter_ranges import grid_specs
    from classical_speech_enhancement_amd.synth import make_pair
    pairs = [make_pair(i, 10.0) for i in range(a.pairs)]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    gp = Engine().plan(a.pairs, 160000, grid_specs(a.pairs, 512), with_clean=True).plans[0]
    gp.prepare(noisy, clean)
    torch.cuda.synchronize()

    def timed(fn):
        ms = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        return float(np.median(ms))

    out = {"prepare_ms": timed(lambda: gp.prepare(noisy, clean))}
    pool_ref = gp.pool.clone()
    for hop in gp.hops:
        j0, nj = gp.hop_jobs[hop]
        jobs = ctypes.c_void_p(gp.jobs_d.data_ptr() + j0 * _lib.NOISE_JOB_DTYPE.itemsize)

        def fin():
            _lib.check(gp.lib.cse_noise_finish(jobs, nj, gp.S, gp.B, _ptr(gp.raw), _ptr(gp.pool),
                                               _stream()), "finish")
        out[f"finish_hop{hop}_ms"] = timed(fin)
    torch.cuda.synchronize()
    out["pool_unchanged"] = bool(torch.equal(gp.pool, pool_ref))
    out["lib"] = os.environ.get("CSE_LIB", "libcse.so")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
