"""Helpers for the multi-process grid tests (CPU, gloo): an oracle-backed
compute function standing in for the device engine, and the rank entry point.
Test infrastructure only."""

import os

import numpy as np

SMALL_GRIDS = {
    "spectralSubtractor": {"alpha": [1.0, 2.0], "beta": [0.01, 0.1], "n_fft": [512],
                           "hop_length": [128, 256], "noise_percentile": [10.0],
                           "noise_method": ["percentile", "min_tracking"]},
    "mmse": {"alpha": [0.95], "ksi_min": [0.01, 0.1], "gain_min": [0.05], "gain_max": [1.0],
             "n_fft": [512], "hop_length": [128], "noise_percentile": [10.0, 20.0],
             "noise_method": ["percentile", "min_tracking"]},
    "wiener": {"alpha": [0.9, 0.98], "gain_floor": [0.05], "n_fft": [512, 1024],
               "hop_length": [256], "noise_percentile": [20.0], "noise_method": ["percentile"]},
    "omlsa": {"alpha": [0.9], "ksi_min": [0.01], "gain_floor": [0.1], "noise_mu": [0.95],
              "q": [0.3, 0.5], "n_fft": [512], "hop_length": [128],
              "noise_percentile": [10.0], "noise_method": ["percentile", "min_tracking"]},
}


def pairs(n=3, seconds=0.3):
    from classical_speech_enhancement_amd.synth import make_pair
    out = [make_pair(i, seconds) for i in range(n)]
    return [c for c, _ in out], [x for _, x in out]


def oracle_compute(clean, noisy, specs, ids, align=True, stoi=True):
    """Per-cell (sse, snr, finite, stoi, lag, xstatus = 0) from the CPU oracle
    (search.RECORD_FIELDS without cell_id): finalize_enhanced
    (alignment, length match, finiteness, clip) then calculate_snr and
    calculate_stoi, like the reference's grid loop
    (speech_enhancement_comparison.py:165-180); align=False scores the clipped
    output at lag 0; stoi=False leaves the STOI column NaN.  STOI sees the
    output rounded to f32, the type the device writes."""
    import oracle
    from oracle import stoi_ref
    out = np.zeros((len(ids), 6))
    for j, cid in enumerate(ids):
        pair, alg, p = specs[cid]
        kw = dict(p)
        if kw["noise_method"] == "true_noise":
            kw["clean_audio"] = clean[pair]
        y = oracle.ALGORITHMS[alg](noisy[pair], 16000, **kw)
        c = np.asarray(clean[pair], np.float64)
        e = oracle.finalize_enhanced(y, c, 16000, do_align=align)
        lag = (oracle.align_lag(c, y, 16000) or 0) if align else 0
        if e is None:
            out[j] = (np.nan, np.nan, 0, np.nan, 0, 0)
            continue
        st = None
        if stoi:
            e32 = oracle.finalize_enhanced(np.asarray(y, np.float32).astype(np.float64), c, 16000,
                                           do_align=align)
            st = stoi_ref.calculate_stoi(c, e32, 16000)
        out[j] = (np.sum((c - e) ** 2), oracle.calculate_snr(c, e), 1,
                  np.nan if st is None else st, lag, 0)
    return out


def rank_main(rank, world, port, outdir):
    import torch.distributed as dist
    from classical_speech_enhancement_amd import search
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        clean, noisy = pairs()
        specs = search.job_specs(len(noisy), grids=SMALL_GRIDS)
        calls = []

        def compute(c, n, s, ids):
            calls.append(list(map(int, ids)))
            return oracle_compute(c, n, s, ids)
        table, best = search.run_grid(clean, noisy, specs, compute=compute)
        win = np.array([[k[0], list(SMALL_GRIDS).index(k[1]), v[0]] for k, v in best.items()])
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), table=table, win=win,
                 ids=np.array([i for c in calls for i in c], dtype=np.int64))
    finally:
        dist.destroy_process_group()


def oracle_cell_full(args):
    """One 10-s cell through the oracle for the full-size sweep test: the
    enhanced waveform, finalize_enhanced's lag, the aligned SNR and STOI (of the
    output rounded to f32, the type the device writes).  Pool worker."""
    import oracle
    from oracle import stoi_ref
    from classical_speech_enhancement_amd.synth import make_pair
    pair, alg, p, seconds = args
    clean, noisy = make_pair(pair, seconds)
    y = oracle.ALGORITHMS[alg](noisy, 16000, **p)
    lag = oracle.align_lag(clean, y, 16000) or 0
    e = oracle.finalize_enhanced(y, clean, 16000)
    snr = oracle.calculate_snr(clean, e)
    e32 = oracle.finalize_enhanced(np.asarray(y, np.float32).astype(np.float64), clean, 16000)
    st = stoi_ref.calculate_stoi(clean, e32, 16000)
    return y, int(lag), snr, np.nan if st is None else st


_PAIR_CACHE = {}


def oracle_cell_scores(args):
    """(cell id, sse, snr, finite, stoi, lag) of one cell through the oracle,
    scored like the reference's grid loop (speech_enhancement_comparison.py:
    165-180: finalize_enhanced, calculate_snr, calculate_stoi of the output
    rounded to f32, the type the device writes).  The pair is synthesised in
    the worker (make_pair(pair, seconds)).  Pool worker."""
    import oracle
    from oracle import stoi_ref
    from classical_speech_enhancement_amd.synth import make_pair
    cid, pair, alg, p, seconds = args
    key = (pair, seconds)
    if key not in _PAIR_CACHE:
        _PAIR_CACHE.clear()
        _PAIR_CACHE[key] = make_pair(pair, seconds)
    clean, noisy = _PAIR_CACHE[key]
    kw = dict(p)
    if kw["noise_method"] == "true_noise":
        kw["clean_audio"] = clean
    y = oracle.ALGORITHMS[alg](noisy, 16000, **kw)
    e = oracle.finalize_enhanced(y, clean, 16000)
    if e is None:
        return cid, np.nan, np.nan, 0.0, np.nan, 0
    lag = oracle.align_lag(clean, y, 16000) or 0
    e32 = oracle.finalize_enhanced(np.asarray(y, np.float32).astype(np.float64), clean, 16000)
    st = stoi_ref.calculate_stoi(clean, e32, 16000)
    return (cid, float(np.sum((clean - e) ** 2)), oracle.calculate_snr(clean, e), 1.0,
            np.nan if st is None else st, int(lag))
