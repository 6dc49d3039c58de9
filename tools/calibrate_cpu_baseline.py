"""Calibrate bench.py's CPU baseline (the oracle port) against the reference.

Runs in the dev container only (it imports the reference modules from
/root/reference through tests/golden/make_golden.py's librosa shim, the same
way the golden fixtures are made).  Times the unmodified reference plugins and
the oracle on the same cells of one 10-s synthetic pair, single-threaded, and
prints the per-cell ratio.  The result is recorded in DESIGN.md §5; nothing
from here runs on the GPU box.

    python tools/calibrate_cpu_baseline.py [N_CELLS]
"""

import os
import sys
import time

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import oracle  # noqa: E402
from classical_speech_enhancement_amd.parameter_ranges import grid_specs  # noqa: E402
from classical_speech_enhancement_amd.synth import make_pair  # noqa: E402
from make_golden import ref_modules  # noqa: E402

NAME = {"spectralSubtractor": "ss", "wiener": "wiener", "mmse": "mmse", "omlsa": "omlsa"}


def main(n=24):
    R = ref_modules()
    clean, noisy = make_pair(0, 10.0)
    specs = grid_specs(1, 512)
    rng = np.random.default_rng(1)
    pick = rng.choice(len(specs), size=n, replace=False)
    t_ref = t_ora = 0.0
    frames = 0
    for i in pick:
        _, alg, p = specs[i]
        kw = dict(p)
        if kw["noise_method"] == "true_noise":
            kw["clean_audio"] = clean
        t0 = time.perf_counter()
        y_ref = R[NAME[alg]](noisy, 16000, **kw)
        t1 = time.perf_counter()
        y_ora = oracle.ALGORITHMS[alg](noisy, 16000, **kw)
        t2 = time.perf_counter()
        t_ref += t1 - t0
        t_ora += t2 - t1
        frames += 1 + len(noisy) // int(p["hop_length"])
        assert np.allclose(y_ref, y_ora, rtol=0, atol=1e-9 * max(1.0, np.abs(y_ref).max()))
    print(f"{n} cells (n_fft 512 HEAD grid, 10-s pair, one core): reference {t_ref / n * 1e3:.1f} ms/cell"
          f" = {frames / t_ref:.0f} evals/s; oracle {t_ora / n * 1e3:.1f} ms/cell = {frames / t_ora:.0f}"
          f" evals/s; oracle/reference speed {t_ref / t_ora:.2f}")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:2]))
