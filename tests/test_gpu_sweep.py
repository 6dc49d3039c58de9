"""The device batch driver end to end (search.run_sweep): selection, WAV and
summary files in the reference's layout, against the oracle (needs a GPU)."""

import os

import numpy as np
import pytest

import oracle
from classical_speech_enhancement_amd import results, search

from _grid_worker import SMALL_GRIDS, oracle_compute, pairs

pytestmark = pytest.mark.gpu


def test_run_sweep_files_and_selection(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    clean, noisy = pairs(2, 0.6)
    stems = ["p00", "p01"]
    grids = {k: SMALL_GRIDS[k] for k in ("spectralSubtractor", "mmse")}
    rows = search.run_sweep(clean, noisy, stems, str(tmp_path), grids=grids)
    assert len(rows) == 4
    specs = search.job_specs(2, list(grids), grids)
    ref = oracle_compute(clean, noisy, specs, np.arange(len(specs)))
    best = search.select_best(specs, ref)
    for r in rows:
        pair = stems.index(r["stem"])
        cid, score = best[(pair, r["alg"])]
        # the device pick scores within float noise of the oracle's pick
        assert abs(r["snr_balopt"] - score) < 1e-3, r
        path = os.path.join(tmp_path, f"results_{r['alg']}", f"{r['stem']}_{r['alg']}_optimized_snr.wav")
        y, sr = results.read_wav_pcm16(path)
        assert sr == 16000 and len(y) == len(clean[pair])
        p = r["best_params_snr"]
        e = oracle.finalize_enhanced(oracle.ALGORITHMS[r["alg"]](noisy[pair], 16000, **p),
                                     clean[pair], 16000)
        q = np.rint(e.astype(np.float32).astype(np.float64) * 32767)
        assert np.max(np.abs(np.rint(y * 32768) - q)) <= 1
    summ = os.path.join(tmp_path, "results_summary")
    for f in ("all_results.json", "summary_means.json", "all_results.csv"):
        assert os.path.exists(os.path.join(summ, f))
