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
    clean, noisy = pairs(2, 1.2)
    stems = ["p00", "p01"]
    grids = {k: SMALL_GRIDS[k] for k in ("spectralSubtractor", "mmse")}
    rows = search.run_sweep(clean, noisy, stems, str(tmp_path), grids=grids)
    assert len(rows) == 4
    specs = search.job_specs(2, list(grids), grids)
    ref = oracle_compute(clean, noisy, specs, np.arange(len(specs)))
    best = search.select_best(specs, ref)
    best_stoi = search.select_best(specs, ref, "stoi")
    from oracle import stoi_ref
    for r in rows:
        pair = stems.index(r["stem"])
        cid, score = best[(pair, r["alg"])]
        # the device pick scores within float noise of the oracle's pick
        assert abs(r["snr_snropt"] - score) < 1e-3, r
        assert r["snr_balopt"] is None and r["best_params_balanced"] == {}
        sid, sscore = best_stoi[(pair, r["alg"])]
        assert abs(r["stoi_stoiopt"] - sscore) < 4e-6, r
        assert abs(r["stoi_noisy"] - stoi_ref.stoi(clean[pair], noisy[pair].astype(np.float32)
                                                   .astype(np.float64), 16000)) < 1e-8
        assert os.path.exists(os.path.join(tmp_path, f"results_{r['alg']}",
                                           f"{r['stem']}_{r['alg']}_optimized_stoi.wav"))
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


def test_prepare_pair_matches_oracle():
    """prepare_pair (speech_enhancement_comparison.py:71-90): mono, 48 k -> 16 k,
    trim, device alignment of a delayed noisy copy == the oracle's
    align_to_reference on the same resampled arrays."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from scipy.signal import resample_poly
    from classical_speech_enhancement_amd import prepare
    from classical_speech_enhancement_amd.synth import make_pair
    c16, n16 = make_pair(21, 3.0)
    c48 = resample_poly(c16, 3, 1)
    for delay in (0, 37, -123):
        n48 = resample_poly(np.roll(n16, delay), 3, 1)
        stereo = np.stack([n48, 0.5 * n48], axis=1)  # (samples, 2): averaged like to_mono
        cl, nz, sr = prepare.prepare_pair(c48, 48000, stereo, 48000)
        rc = resample_poly(c48, 1, 3)
        rn = resample_poly(oracle.to_mono(stereo), 1, 3)
        L = min(len(rc), len(rn))
        rc, rn = rc[:L], rn[:L]
        ref = oracle.match_length(oracle.align_to_reference(rc, rn, 16000), L)
        assert sr == 16000
        np.testing.assert_array_equal(cl, rc)
        np.testing.assert_array_equal(nz, ref)
        lag = oracle.align_lag(rc, rn, 16000)
        assert lag == prepare.alignment_lag(rc, rn, 16000)


def test_sweep_records_do_not_depend_on_batching():
    """Per-cell records are the same whether pairs are batched one per plan
    (the STOI waveform budget forces it) or all together, and on a repeat:
    no cell's result depends on which other cells share its launch."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from classical_speech_enhancement_amd.engine import Engine
    clean, noisy = pairs(3, 1.5)
    specs = search.job_specs(3, grids=SMALL_GRIDS)
    ids = np.arange(len(specs))
    eng = Engine()
    keep = search.STOI_WAVE_BYTES
    try:
        search.STOI_WAVE_BYTES = 1
        a = search.engine_compute(clean, noisy, specs, ids, engine=eng)
        b = search.engine_compute(clean, noisy, specs, ids, engine=eng)
        search.STOI_WAVE_BYTES = 1 << 40
        c = search.engine_compute(clean, noisy, specs, ids, engine=eng)
    finally:
        search.STOI_WAVE_BYTES = keep
    assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(a, c, equal_nan=True)
