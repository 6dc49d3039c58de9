"""BASELINE configs 4 and 5 at their stated size on one MI355X (needs a GPU).

Config 4: 100 synthetic 10-s 16-kHz pairs (seeds 1000+i) x all
4 algorithms x the full 9,744-cell HEAD grid; config 5: the same sweep with the
recursive estimators (min_tracking, percentile) on the device.  Both run here
through the job-level driver search.run_grid (the rewrite of the reference's
loop speech_enhancement_comparison.py:441-455 -> :149-226): STFT, noise PSDs,
fused enhance, finalize_enhanced alignment, SNR and STOI of all 974,400 cells,
once in this process (world 1) and once sharded over two gloo ranks sharing the
card (the 8-GPU node runs the same code over RCCL).

Checked: every cell finite; min_tracking cells that differ only in
noise_percentile (which that estimator ignores) bit-identical (copied in the
deduplicated sweep, computed separately in a plain-list job); the alignment
status of every cell counted (no non-finite head; lags of the flat-correlation
cells, if any, against the oracle); the table
identical across shardings; 64 cells stratified over algorithm x n_fft x hop x
noise method against the oracle: waveform rel-L2 and rel-max <= 1e-5 (the
north-star tolerance), the alignment lag equal, the aligned SNR within
2e-4 dB and STOI within 2e-6 of the oracle's scores.
"""

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_PAIRS = 100
SECONDS = 10.0
TOL = 1e-5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _job():
    from classical_speech_enhancement_amd import search
    from classical_speech_enhancement_amd.synth import make_pair
    pairs = [make_pair(i, SECONDS) for i in range(N_PAIRS)]
    clean = [c for c, _ in pairs]
    noisy = [x for _, x in pairs]
    return clean, noisy, search.job_specs(N_PAIRS)


def _rank(rank, world, port, outdir):
    import sys
    import torch
    import torch.distributed as dist
    repo = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path.insert(0, repo)
    from classical_speech_enhancement_amd import search
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        clean, noisy, specs = _job()
        table, _ = search.run_grid(clean, noisy, specs)
        np.save(os.path.join(outdir, f"full{rank}.npy"), table)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def tables(tmp_path_factory):
    import torch
    if torch.cuda.device_count() == 0:
        pytest.skip("no GPU")
    import torch.multiprocessing as tmp
    out = tmp_path_factory.mktemp("full")
    # the sharded run first: its ranks start before this process holds GPU state
    tmp.spawn(_rank, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    sharded = [np.load(out / f"full{r}.npy") for r in range(2)]
    from classical_speech_enhancement_amd import search
    clean, noisy, specs = _job()
    table, best = search.run_grid(clean, noisy, specs)
    return dict(table=table, best=best, sharded=sharded, clean=clean, noisy=noisy, specs=specs)


def test_full_sweep_shape_finite_and_sharding(tables):
    t, specs = tables["table"], tables["specs"]
    assert len(specs) == N_PAIRS * 9744 and t.shape == (len(specs), 6)
    assert t[:, 2].all(), "non-finite cells"
    assert np.isfinite(t[:, 1]).all()
    assert np.isfinite(t[:, 3]).all()  # 10-s clips: every cell has >= 30 STOI frames
    for s in tables["sharded"]:
        assert np.array_equal(s, t, equal_nan=True)
    # every (pair, algorithm) has a winner under both device objectives
    from classical_speech_enhancement_amd import search
    assert all(c >= 0 for c, _ in tables["best"].values())
    assert all(c >= 0 for c, _ in search.select_best(specs, t, "stoi").values())


def test_min_tracking_duplicate_rows_copied(tables):
    """The sweep computes each min_tracking duplicate (cells that differ only in
    noise_percentile, which that estimator ignores) once and copies its row:
    this checks the copy.  The engine-level identity is checked below."""
    t, specs = tables["table"], tables["specs"]
    first, n = {}, 0
    for cid, (pair, alg, p) in enumerate(specs):
        if p["noise_method"] != "min_tracking":
            continue
        k = (pair, alg) + tuple((a, b) for a, b in p.items() if a != "noise_percentile")
        if k in first:
            assert np.array_equal(t[cid], t[first[k]]), (pair, alg, p)
            n += 1
        else:
            first[k] = cid
    assert n == N_PAIRS * 9744 // 4


def test_min_tracking_duplicates_computed_separately_bit_identical(tables):
    """A plain-list job (not JobSpecs, so no deduplication): every min_tracking
    cell of 2 pairs x the full grid goes through the engine on its own, aligned
    and STOI-scored, and each duplicate's row equals its twin's bit for bit."""
    from classical_speech_enhancement_amd import search
    specs = [s for s in tables["specs"][:2 * 9744] if s[2]["noise_method"] == "min_tracking"]
    vals = search.engine_compute(tables["clean"], tables["noisy"], specs, np.arange(len(specs)))
    first, n = {}, 0
    for cid, (pair, alg, p) in enumerate(specs):
        k = (pair, alg) + tuple((a, b) for a, b in p.items() if a != "noise_percentile")
        if k in first:
            assert np.array_equal(vals[cid], vals[first[k]], equal_nan=True), (pair, alg, p)
            n += 1
        else:
            first[k] = cid
    assert n == len(specs) // 2 == 2 * 9744 // 4


def test_alignment_status_counted_flat_cells_exact(tables):
    """cse_xcorr_lag's status over all 974,400 cells (search table column
    'xstatus'): no non-finite head; FLAT cells (more than 64 near-maximal lags,
    every one re-evaluated in fp64) are counted, and up to 32 of them are
    checked against the oracle's lag."""
    import multiprocessing as mp
    from _grid_worker import oracle_cell_full
    t, specs = tables["table"], tables["specs"]
    st = t[:, 5].astype(np.int64)
    lag = t[:, 4]
    print(f"xcorr status: ok {(st == 0).sum()}, flat {(st == 1).sum()}, nonfinite "
          f"{(st == 2).sum()}; non-zero lags {(lag != 0).sum()} of {len(t)}")
    assert (st == 2).sum() == 0
    flat = np.flatnonzero(st == 1)
    if len(flat) == 0:
        return
    pick = flat[np.linspace(0, len(flat) - 1, min(32, len(flat))).astype(np.int64)]
    procs = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("spawn").Pool(procs) as pool:
        ref = pool.map(oracle_cell_full, [specs[int(c)] + (SECONDS,) for c in pick], chunksize=1)
    for c, (_, lag_ref, _, _) in zip(pick, ref):
        assert int(lag[c]) == lag_ref, (int(c), lag[c], lag_ref)


def test_nonzero_lag_cells_match_oracle(tables):
    """The cells whose alignment lag is not 0 (config 4 has ~1,500 of them).

    They are the only ones that exercise the 7-block FFT correlation's argmax
    away from lag 0, the lag-shifted rescoring (enhance_kernel with cell.lag)
    and the lag-shifted STOI input (speech_enhancement_comparison.py:38-69,60,
    92-106, 180).  Up to 128 of them, drawn round-robin over the strata
    algorithm x n_fft x hop x sign(lag) so that every populated stratum
    (both lag signs included) contributes, against the oracle: lag equal,
    aligned SNR within 2e-4 dB, STOI within 2e-6, waveform rel-L2 and rel-max
    within 1e-5."""
    import multiprocessing as mp
    import torch
    from classical_speech_enhancement_amd.engine import Engine
    from _grid_worker import oracle_cell_full
    t, specs = tables["table"], tables["specs"]
    lag = t[:, 4].astype(np.int64)
    nz = np.flatnonzero(lag != 0)
    assert len(nz) >= 64, f"only {len(nz)} non-zero-lag cells"
    strata = {}
    for cid in nz.tolist():
        _, alg, p = specs[cid]
        strata.setdefault((alg, p["n_fft"], p["hop_length"], int(np.sign(lag[cid]))), []).append(cid)
    rng = np.random.default_rng(4242)
    pools = {k: list(rng.permutation(v)) for k, v in sorted(strata.items())}
    pick = []
    while len(pick) < 128 and any(pools.values()):
        for k in sorted(pools):
            if pools[k] and len(pick) < 128:
                pick.append(int(pools[k].pop()))
    signs = {int(np.sign(lag[c])) for c in pick}
    print(f"non-zero lags: {len(nz)} cells in {len(strata)} strata "
          f"({sorted((k, len(v)) for k, v in strata.items())}); checking {len(pick)}")
    assert len(pick) >= 64
    procs = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("spawn").Pool(procs) as pool:
        ref = pool.map(oracle_cell_full, [specs[c] + (SECONDS,) for c in pick], chunksize=1)
    eng = Engine()
    # device waveforms and lags, one launch per pair (the cells of a pair share Y/N)
    by_pair = {}
    for j, cid in enumerate(pick):
        by_pair.setdefault(specs[cid][0], []).append(j)
    y_dev, lag_dev = [None] * len(pick), [None] * len(pick)
    for pair, js in by_pair.items():
        x = torch.as_tensor(tables["noisy"][pair]).cuda().view(1, -1)
        c = torch.as_tensor(tables["clean"][pair]).cuda().view(1, -1)
        res = eng.run(x, [(0, specs[pick[j]][1], specs[pick[j]][2]) for j in js], clean=c,
                      want_waveforms=True, align=True)
        for r, j in enumerate(js):
            y_dev[j] = res["y"][r].double().cpu().numpy()
            lag_dev[j] = int(res["lag"][r])
    worst = dict(l2=0.0, mx=0.0, snr=0.0, stoi=0.0)
    for j, (cid, (y_ref, lag_ref, snr_ref, stoi_ref)) in enumerate(zip(pick, ref)):
        assert lag_ref != 0 and int(lag[cid]) == lag_ref, (cid, lag[cid], lag_ref)
        assert lag_dev[j] == lag_ref, (cid, lag_dev[j], lag_ref)
        y = y_dev[j]
        l2 = np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref)
        mx = np.max(np.abs(y - y_ref)) / np.max(np.abs(y_ref))
        assert l2 <= TOL and mx <= TOL, (cid, specs[cid], l2, mx)
        assert abs(t[cid, 1] - snr_ref) <= 2e-4, (cid, t[cid, 1], snr_ref)
        assert abs(t[cid, 3] - stoi_ref) <= 2e-6, (cid, t[cid, 3], stoi_ref)
        worst = dict(l2=max(worst["l2"], l2), mx=max(worst["mx"], mx),
                     snr=max(worst["snr"], abs(t[cid, 1] - snr_ref)),
                     stoi=max(worst["stoi"], abs(t[cid, 3] - stoi_ref)))
    lags = [int(lag[c]) for c in pick]
    print(f"{len(pick)} non-zero-lag cells (lags {min(lags)}..{max(lags)}, signs {sorted(signs)}) "
          f"match the oracle; worst: {worst}")


def test_stratified_cells_match_oracle(tables):
    import multiprocessing as mp
    import torch
    from classical_speech_enhancement_amd.engine import Engine
    from _grid_worker import oracle_cell_full
    t, specs = tables["table"], tables["specs"]
    strata = {}
    for cid, (pair, alg, p) in enumerate(specs):
        strata.setdefault((alg, p["n_fft"], p["hop_length"], p["noise_method"]), []).append(cid)
    assert len(strata) == 32
    rng = np.random.default_rng(2024)
    pick = [int(c) for k in sorted(strata) for c in rng.choice(strata[k], 2, replace=False)]
    procs = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context("spawn").Pool(procs) as pool:
        ref = pool.map(oracle_cell_full, [specs[c] + (SECONDS,) for c in pick], chunksize=1)
    eng = Engine()
    worst = dict(l2=0.0, mx=0.0, snr=0.0, stoi=0.0)
    for cid, (y_ref, lag_ref, snr_ref, stoi_ref) in zip(pick, ref):
        pair, alg, p = specs[cid]
        x = torch.as_tensor(tables["noisy"][pair]).cuda().view(1, -1)
        c = torch.as_tensor(tables["clean"][pair]).cuda().view(1, -1)
        res = eng.run(x, [(0, alg, p)], clean=c, want_waveforms=True, align=True)
        y = res["y"][0].double().cpu().numpy()
        l2 = np.linalg.norm(y - y_ref) / np.linalg.norm(y_ref)
        mx = np.max(np.abs(y - y_ref)) / np.max(np.abs(y_ref))
        assert l2 <= TOL and mx <= TOL, (cid, alg, p, l2, mx)
        assert int(res["lag"][0]) == lag_ref, (cid, res["lag"][0], lag_ref)
        assert abs(t[cid, 1] - snr_ref) <= 2e-4, (cid, t[cid, 1], snr_ref)
        assert abs(t[cid, 3] - stoi_ref) <= 2e-6, (cid, t[cid, 3], stoi_ref)
        worst = dict(l2=max(worst["l2"], l2), mx=max(worst["mx"], mx),
                     snr=max(worst["snr"], abs(t[cid, 1] - snr_ref)),
                     stoi=max(worst["stoi"], abs(t[cid, 3] - stoi_ref)))
    print("worst over 64 stratified cells:", worst)
