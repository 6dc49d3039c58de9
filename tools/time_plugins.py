"""Wall time of one plugin call (INTEGRATION level 1: the reference's loop
calling the device mirrors one cell at a time), 10-s input, after warm-up;
the oracle's CPU time for the same call beside it (analysis only).

    python tools/time_plugins.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import oracle
    from classical_speech_enhancement_amd import plugins
    from classical_speech_enhancement_amd.synth import make_pair
    clean, noisy = make_pair(0, seconds=10.0)
    cases = [
        ("wiener", plugins.wiener_filter, oracle.wiener_filter,
         dict(alpha=0.95, gain_floor=0.05, noise_percentile=10.0, noise_method="percentile")),
        ("omlsa", plugins.advanced_mmse, oracle.advanced_mmse,
         dict(alpha=0.9, ksi_min=0.005, q=0.4, noise_mu=0.95, gain_floor=0.1,
              noise_percentile=10.0, noise_method="min_tracking")),
    ]
    for name, dev, ref, kw in cases:
        for n_fft, hop in ((512, 128), (512, 160), (1024, 256)):
            p = dict(kw, n_fft=n_fft, hop_length=hop)
            dev(noisy, 16000, **p)  # warm-up (library load, first plan)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                y = dev(noisy, 16000, **p)
                ts.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            r = ref(noisy, 16000, **p)
            tc = time.perf_counter() - t0
            err = float(np.linalg.norm(y - r) / np.linalg.norm(r))
            print(json.dumps({"plugin": name, "n_fft": n_fft, "hop": hop,
                              "device_ms": 1e3 * float(np.median(ts)), "oracle_cpu_ms": 1e3 * tc,
                              "rel_l2": err}), flush=True)


if __name__ == "__main__":
    main()
