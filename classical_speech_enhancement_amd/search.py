"""Grid-search driver: the data-parallel rewrite of the reference's sweep.

The reference walks pairs -> algorithms -> parameter combinations one cell at
a time (speech_enhancement_comparison.py:149-226 inside optimize_parameters,
called per algorithm from run_algorithm_on_pair :278-294 and main :440-455).
Here the whole (pair x algorithm x grid cell) set is one job:

  job_specs      the reference's enumeration order; a cell's index in this
                 list is its cell_id (grid order inside each (pair, algorithm))
  work_items     cells grouped by what they share on the device:
                 (pair, n_fft, hop, algorithm) -> one STFT, one set of noise
                 rows; cost = cells x frames x bins x algorithm weight
  assign_shards  contiguous runs of cell ids of equal modelled cost per rank
                 (SURVEY §8(e)'s cost model): whole pairs per rank, so each
                 pair's STFT and noise PSDs run on one rank (two at a cut)
  run_grid       each rank computes its cells (Engine on its GPU), then ONE
                 all_gather of fixed-size 56-B records (RECORD_FIELDS: cell_id,
                 sse, snr, finite, stoi, lag, xstatus; a 6-column table)
                 (RCCL over xGMI for backend "nccl", gloo in CPU tests)
  select_best    rank 0's sequential best-so-far scan in grid order
                 (speech_enhancement_comparison.py:183-216) — NOT an argmax:
                 a later cell replaces the incumbent only if it beats it by
                 more than tol, so ties within tol keep the earlier cell

Scores: the reference scores cells by STOI, PESQ and their balance
(evaluation_metrics.py:30-36, 104-115).  The device path computes STOI
(cse_stoi_cells, pystoi 0.4.1 restated) and the SNR of the clipped output
(evaluation_metrics.py:39-58).  PESQ's C extension is not in this image, so
the PESQ and balance objectives are not scored; STOI and SNR each get the
reference's sequential selection (the reference itself skips a cell whose
PESQ is None, speech_enhancement_comparison.py:180-181 — that rule is dropped, or nothing would be selected).
Each cell is scored like finalize_enhanced (:92-106): its output is aligned
to the clean reference by the cross-correlation lag (on the device,
cse_xcorr_lag), length-matched, checked for finiteness and clipped, then
calculate_snr and calculate_stoi.
"""

import math
import os
from collections import OrderedDict

import numpy as np

from .parameter_ranges import ALGORITHM_GRIDS, grid_cells

# per-bin cost weights (measured kernel time per frame, OMLSA ~ 3x SS)
ALGO_WEIGHT = {"spectralSubtractor": 1.0, "wiener": 1.1, "mmse": 2.0, "omlsa": 3.0}
# tolerance of the best-so-far update per objective (speech_enhancement_comparison.py:183,194,205)
TOLERANCE = {"stoi": 1e-6, "pesq": 1e-3, "balance": 1e-5, "snr": 1e-5}

# one float64 row per cell.  lag: finalize_enhanced's alignment lag (0 when
# not aligned); xstatus: cse_xcorr_lag's status (engine: XCORR_OK, XCORR_FLAT =
# the exact many-candidate path ran, XCORR_NONFINITE; 0 when not aligned)
RECORD_FIELDS = ("cell_id", "sse", "snr", "finite", "stoi", "lag", "xstatus")
TABLE_COLUMN = {"sse": 0, "snr": 1, "finite": 2, "stoi": 3, "lag": 4,
                "xstatus": 5}  # table = records without cell_id
NCOL = len(RECORD_FIELDS) - 1
# bound on the cell waveforms held at once for STOI scoring (f32 bytes): 48 GiB
# of the 288 GB HBM, i.e. 10 full 10-s pairs (7,308 computed cells x 640 KB each)
# per batch, two batches in flight.  100-pair sweep (late r04, call_r04s.sh in profiles/r04_commands.md):
# 16 GiB 1.48-1.49 s, 32 GiB 1.31-1.32 s, 48 GiB 1.256-1.258 s, 64 GiB
# 1.253-1.295 s; 96 GiB ran out of memory
STOI_WAVE_BYTES = 48 << 30
# share of the device memory free when a sweep starts that the two STOI
# batches in flight may take together (a smaller GPU, or plans cached by the
# caller, shrink the batches below STOI_WAVE_BYTES instead of running out)
STOI_FREE_SHARE = 0.6


def stoi_wave_bytes():
    """Bytes of cell waveforms per STOI batch: STOI_WAVE_BYTES, capped at half
    of STOI_FREE_SHARE of the device memory free now (two batches in flight)."""
    import torch
    free, _ = torch.cuda.mem_get_info()
    # blocks torch's caching allocator holds but no tensor uses are free to this
    # process too (mem_get_info counts them as taken)
    free += torch.cuda.memory_reserved() - torch.cuda.memory_allocated()
    return int(min(STOI_WAVE_BYTES, STOI_FREE_SHARE * free / 2))


class JobSpecs(list):
    """job_specs' result: the list of (pair, algorithm, params) tuples, plus
    numpy columns so the sweep's per-cell bookkeeping (grouping, duplicate
    cells, plan keys, selection) runs without per-cell Python loops:
      pair [n], alg [n] (index into .algorithms), cell [n] (index into
      .cells[alg], the algorithm's grid in reference order).
    Every pair shares the same params dict per grid cell (read-only)."""

    def __init__(self, n_pairs, algorithms, cells):
        algorithms = list(algorithms)
        super().__init__((pair, alg, p) for pair in range(n_pairs) for alg in algorithms
                         for p in cells[alg])
        self.algorithms = algorithms
        self.cells = cells
        per = [len(cells[a]) for a in algorithms]
        self.per_pair = int(sum(per))
        a_col = np.concatenate([np.full(n, k, dtype=np.int64) for k, n in enumerate(per)] or
                               [np.zeros(0, np.int64)])
        c_col = np.concatenate([np.arange(n, dtype=np.int64) for n in per] or [np.zeros(0, np.int64)])
        self.pair = np.repeat(np.arange(n_pairs, dtype=np.int64), self.per_pair)
        self.alg = np.tile(a_col, n_pairs)
        self.cell = np.tile(c_col, n_pairs)
        self._rep = {}

    def grid_rep(self, alg_index, length):
        """For each cell of one algorithm's grid, the first grid cell the engine
        computes identically for signals of this length: same n_fft, hop and
        algorithm parameters and the same noise PSD (engine.noise_key — e.g.
        min_tracking and true_noise ignore noise_percentile)."""
        key = (alg_index, int(length))
        if key not in self._rep:
            from .engine import ALGOS, DEFAULTS, n_frames, noise_key
            alg = self.algorithms[alg_index]
            names = ALGOS[alg][2]
            dflt = DEFAULTS.get(alg, {})
            first, rep = {}, []
            for c, p in enumerate(self.cells[alg]):
                hop = int(p["hop_length"])
                k = (int(p["n_fft"]), hop, tuple(float(p[n] if n in p else dflt[n]) for n in names),
                     noise_key(alg, p, n_frames(length, hop)))
                rep.append(first.setdefault(k, c))
            self._rep[key] = np.asarray(rep, dtype=np.int64)
        return self._rep[key]

    def nfft(self, ids):
        """n_fft of each of ``ids``."""
        if not hasattr(self, "_nfft"):
            self._nfft = [np.array([int(p["n_fft"]) for p in self.cells[a]], dtype=np.int64)
                          for a in self.algorithms]
        ids = np.asarray(ids, dtype=np.int64)
        out = np.empty(len(ids), dtype=np.int64)
        for a, col in enumerate(self._nfft):
            sel = self.alg[ids] == a
            out[sel] = col[self.cell[ids[sel]]]
        return out

    def representative(self, ids, lengths):
        """Global index of the cell computed in place of each of ``ids`` (the
        first identical cell of the same pair and algorithm)."""
        ids = np.asarray(ids, dtype=np.int64)
        lens = np.asarray(lengths, dtype=np.int64)
        present = np.zeros(len(lens), dtype=bool)
        present[self.pair[ids]] = True
        uL = np.unique(lens[present])
        if len(uL) <= 1:  # one clip length (the sweep's case): one table lookup per cell
            if len(uL) == 0:
                return ids.copy()
            L = int(uL[0])
            delta = np.concatenate([self.grid_rep(a, L) - np.arange(len(self.cells[alg]))
                                    for a, alg in enumerate(self.algorithms)])
            off = np.concatenate([[0], np.cumsum([len(self.cells[a]) for a in self.algorithms])[:-1]])
            return ids + delta[off[self.alg[ids]] + self.cell[ids]]
        out = ids.copy()
        for a in range(len(self.algorithms)):
            for L in {int(lengths[q]) for q in np.unique(self.pair[ids[self.alg[ids] == a]])}:
                sel = (self.alg[ids] == a) & (np.asarray(lengths)[self.pair[ids]] == L)
                c = self.cell[ids[sel]]
                out[sel] = ids[sel] - c + self.grid_rep(a, L)[c]
        return out


def job_specs(n_pairs, algorithms=None, grids=None, n_fft=None):
    """(pair, algorithm, params) for every pair x algorithm x grid cell, in the
    reference's order (pairs outermost, registry order of algorithms, grid
    order with the last key fastest), as a JobSpecs list.  One params dict per
    grid cell is shared by every pair (read-only): the engine recognises equal
    batch structures by params identity."""
    grids = grids or ALGORITHM_GRIDS
    algorithms = list(algorithms or grids)
    cells = {alg: [p for p in grid_cells(grids[alg]) if n_fft is None or p["n_fft"] == n_fft]
             for alg in algorithms}
    return JobSpecs(n_pairs, algorithms, cells)


def frames(length, hop):
    return 1 + int(length) // int(hop)


def work_items(specs, lengths):
    """Group cell ids by (pair, n_fft, hop, algorithm).  Returns a list of
    (cost, [cell ids]) (ids ascending within an item)."""
    if isinstance(specs, JobSpecs):
        # per grid cell: n_fft, hop; the group key is a mixed-radix integer
        nf = np.concatenate([[int(p["n_fft"]) for p in specs.cells[a]] for a in specs.algorithms])
        hp = np.concatenate([[int(p["hop_length"]) for p in specs.cells[a]] for a in specs.algorithms])
        off = np.concatenate([[0], np.cumsum([len(specs.cells[a]) for a in specs.algorithms])[:-1]])
        g = off[specs.alg] + specs.cell
        key = ((specs.pair * 4096 + nf[g]) * 4096 + hp[g]) * 64 + specs.alg
        uk, inv = np.unique(key, return_inverse=True)
        order = np.argsort(inv, kind="stable")
        bounds = np.searchsorted(inv[order], np.arange(len(uk) + 1))
        lengths = np.asarray(lengths)
        items = []
        for u in range(len(uk)):
            ids = order[bounds[u]:bounds[u + 1]]
            c0 = int(ids[0])
            alg = specs.algorithms[int(specs.alg[c0])]
            per_cell = (frames(lengths[specs.pair[c0]], hp[g[c0]]) * (int(nf[g[c0]]) // 2 + 1)
                        * ALGO_WEIGHT.get(alg, 1.0))
            items.append((per_cell * len(ids), ids.tolist()))
        return items
    groups = OrderedDict()
    for cid, (pair, alg, p) in enumerate(specs):
        key = (pair, int(p["n_fft"]), int(p["hop_length"]), alg)
        groups.setdefault(key, []).append(cid)
    items = []
    for (pair, n_fft, hop, alg), ids in groups.items():
        per_cell = frames(lengths[pair], hop) * (n_fft // 2 + 1) * ALGO_WEIGHT.get(alg, 1.0)
        items.append((per_cell * len(ids), ids))
    return items


def cell_costs(specs, lengths):
    """Modelled cost of every cell: frames x bins x algorithm weight."""
    lengths = np.asarray(lengths, dtype=np.int64)
    if isinstance(specs, JobSpecs):
        nf = np.concatenate([[int(p["n_fft"]) for p in specs.cells[a]] for a in specs.algorithms])
        hp = np.concatenate([[int(p["hop_length"]) for p in specs.cells[a]] for a in specs.algorithms])
        wt = np.concatenate([[ALGO_WEIGHT.get(a, 1.0)] * len(specs.cells[a])
                             for a in specs.algorithms])
        n_pairs = len(specs) // max(specs.per_pair, 1)
        if n_pairs and len(lengths) >= n_pairs and (lengths[:n_pairs] == lengths[0]).all():
            # one clip length: every pair's block of cells costs the same
            return np.tile((1 + int(lengths[0]) // hp) * (nf // 2 + 1) * wt, n_pairs)
        off = np.concatenate([[0], np.cumsum([len(specs.cells[a]) for a in specs.algorithms])[:-1]])
        g = off[specs.alg] + specs.cell
        return (1 + lengths[specs.pair] // hp[g]) * (nf[g] // 2 + 1) * wt[g]
    return np.array([frames(lengths[pair], p["hop_length"]) * (int(p["n_fft"]) // 2 + 1)
                     * ALGO_WEIGHT.get(alg, 1.0) for (pair, alg, p) in specs], dtype=np.float64)


def assign_shards(specs, lengths, world):
    """Rank of every cell and each rank's modelled load: the job cut into
    ``world`` contiguous runs of cell ids of equal modelled cost (a cell goes to
    the run its cost midpoint falls in).

    Cell ids run pairs -> algorithms -> grid (job_specs), so a rank holds whole
    pairs plus at most a part of one pair at each end of its run: the per-pair
    analysis (STFT and noise PSDs of each (n_fft, hop)) runs on at most
    ceil(pairs / world) + 1 pairs per rank, and every rank gets the same mix of
    algorithms and hops, so an error in the cost model (ALGO_WEIGHT) shifts
    every rank alike.  (A greedy LPT over (pair, n_fft, hop, algorithm) items,
    r01-r02, spread each pair's items over many ranks: at world 8 on the
    100-pair job every rank ran the analysis of 25 pairs instead of 13.)"""
    cost = cell_costs(specs, lengths).astype(np.float64)
    n = len(cost)
    rank_of = np.zeros(n, dtype=np.int64)
    if world > 1 and n:
        total = float(cost.sum())
        mid = np.cumsum(cost) - 0.5 * cost
        rank_of = np.minimum((mid * world / total).astype(np.int64), world - 1)
    load = np.bincount(rank_of, weights=cost, minlength=world).tolist() if n else [0.0] * world
    return rank_of, load


def _unique_inverse(x):
    """np.unique(x, return_inverse=True) for non-negative integer ids, in O(n)
    with a mark array instead of a sort (the sweep's 974,400 representatives)."""
    x = np.asarray(x, dtype=np.int64)
    if len(x) == 0:
        return x.copy(), np.zeros(0, dtype=np.int64)
    mark = np.zeros(int(x.max()) + 1, dtype=bool)
    mark[x] = True
    rank = np.cumsum(mark) - 1
    return np.flatnonzero(mark), rank[x]


def engine_compute(clean, noisy, specs, ids, engine=None, align=True, stoi=True):
    """Device compute of the cells ``ids``: per-cell (sse, snr, finite, stoi,
    lag, xstatus), scored after finalize_enhanced's alignment (align=False: at
    lag 0, lag and xstatus 0).  stoi=False leaves the STOI column NaN (no
    waveforms are kept).

    clean/noisy: lists of 1-D float arrays (host) indexed by pair.  Pairs are
    batched by length (the engine's signal batches are rectangular), and, when
    STOI is scored, in groups whose cell waveforms fit stoi_wave_bytes().  With
    job_specs' JobSpecs, cells the engine computes identically (a quarter of
    the HEAD grid: min_tracking ignores noise_percentile) are computed once
    and their rows copied, and batches of the same structure reuse one device
    plan (Engine.run(reuse=...)).

    Device memory: an engine made here is dropped with its cached plans on
    return.  A caller's engine keeps its plan_cache_size; the STOI path holds
    two plans while it runs (double-buffered waveforms: 2 x stoi_wave_bytes(),
    96 GiB peak on an idle 288-GB device, plus each plan's analysis buffers)
    and trims the cache back to
    the caller's size on return."""
    from .engine import Engine
    own = engine is None
    eng = engine or Engine()
    size0 = eng.plan_cache_size
    try:
        return _engine_compute(eng, clean, noisy, specs, ids, align, stoi)
    finally:
        if own:
            eng._plan_cache.clear()
        else:
            eng.plan_cache_size = size0
            while len(eng._plan_cache) > max(size0, 1):
                eng._plan_cache.popitem(last=False)


def _engine_compute(eng, clean, noisy, specs, ids, align, stoi):
    import torch
    from .engine import snr_db, spec_fingerprint, structure_digest
    from .metrics import StoiPlan
    ids = np.asarray(ids, dtype=np.int64)
    lengths = [len(x) for x in noisy]
    js_specs = isinstance(specs, JobSpecs)
    if js_specs:
        comp, back = _unique_inverse(specs.representative(ids, lengths))
        pair_of = specs.pair[comp]
    else:
        comp, back = ids, np.arange(len(ids))
        pair_of = np.fromiter((specs[c][0] for c in comp), dtype=np.int64, count=len(comp))
    vals = np.full((len(comp), NCOL), np.nan)
    by_len = OrderedDict()
    upairs, first = np.unique(pair_of, return_index=True)
    for pair in upairs[np.argsort(first, kind="stable")].tolist():  # first-appearance order
        by_len.setdefault(lengths[pair], []).append(pair)
    # STOI runs on the engine's side stream: the STOI of one n_fft's cells
    # overlaps the next n_fft's enhance and alignment on the main stream
    # (tools/overlap_probe.py: 20.4 -> 17.6 ms for one launch of each).
    # ready[key]: event after the last STOI that read the waveforms of the
    # plan with that reuse key (a reusing run overwrites them in place).
    main = torch.cuda.current_stream() if stoi else None
    side = eng.side_stream() if stoi else None
    inflight, ready = [], {}
    if stoi:  # consecutive batches alternate between two plans (waveform buffers)
        eng.plan_cache_size = max(eng.plan_cache_size, 2)
    nbatch = 0

    def collect(item):
        rows_, fin_, out_, ev_, _refs = item
        ev_.synchronize()
        vals[rows_, 3] = np.where(fin_, out_.cpu().numpy(), np.nan)

    sorted_pairs = len(pair_of) < 2 or bool((pair_of[1:] >= pair_of[:-1]).all())
    for L, pairs_l in by_len.items():
        if sorted_pairs:  # JobSpecs ids: each pair's cells are one run of comp
            pa = np.asarray(pairs_l, dtype=np.int64)
            lo, hi = np.searchsorted(pair_of, pa, "left"), np.searchsorted(pair_of, pa, "right")
            rows = {p: np.arange(a, b) for p, a, b in zip(pairs_l, lo.tolist(), hi.tolist())}
        else:
            rows = {p: np.flatnonzero(pair_of == p) for p in pairs_l}
        batches, cur, n_cur = [], [], 0
        cap = stoi_wave_bytes() if stoi else 0
        for pair in pairs_l:
            n = len(rows[pair])
            if stoi and cur and (n_cur + n) * L * 4 > cap:
                batches.append(cur)
                cur, n_cur = [], 0
            cur.append(pair)
            n_cur += n
        batches.append(cur)
        for pairs in batches:
            js = np.concatenate([rows[p] for p in pairs])
            slot_of = np.full(int(max(pairs)) + 1, -1, dtype=np.int64)
            slot_of[pairs] = np.arange(len(pairs))
            sig = slot_of[pair_of[js]]  # the batch slot of each cell's pair
            nz = torch.as_tensor(np.stack([np.asarray(noisy[p], np.float64) for p in pairs])).cuda()
            cl = torch.as_tensor(np.stack([np.asarray(clean[p], np.float64) for p in pairs])).cuda()
            cpow = np.array([float(np.dot(np.asarray(clean[p], np.float64),
                                          np.asarray(clean[p], np.float64))) for p in pairs])
            splan = StoiPlan(cl) if stoi else None
            state = {}

            def on_plan(p, sse, fin, lag, js=js, sig=sig, L=L, splan=splan, state=state):
                """one n_fft's cells are final: queue their STOI on the side stream"""
                idx = np.asarray(p.idx, dtype=np.int64)
                lg = lag if lag is not None else np.zeros(len(idx), dtype=np.int64)
                # uploads on the main stream (a pageable copy would wait for the
                # side stream's queue), then the side stream takes over
                off_d = torch.as_tensor(idx * L).cuda()
                sig_d = torch.as_tensor(sig[idx].astype(np.int32)).cuda()
                lag_d = torch.as_tensor(np.asarray(lg, dtype=np.int32)).cuda()
                y = p.y_all.view(-1)  # the run's waveform buffer (every n_fft's rows)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    out = splan.score_async(y, off_d, sig_d, lag=lag_d, clip=True)
                    ev = torch.cuda.Event()
                    ev.record(side)
                state["ev"] = ev
                inflight.append((js[idx], fin, out, ev, (y, off_d, sig_d, lag_d, splan)))
                while len(inflight) > 2:  # bound the STOI scratch held in flight
                    collect(inflight.pop(0))

            def sub(js=js, sig=sig):
                return [(int(sg), specs[int(c)][1], specs[int(c)][2]) for sg, c in zip(sig, comp[js])]
            if js_specs:
                # batches of the same structure reuse one device plan: the key
                # is the cells' (slot, algorithm, grid cell) and this JobSpecs
                h = structure_digest()
                for arr in (sig, specs.alg[comp[js]], specs.cell[comp[js]]):
                    h.update(np.ascontiguousarray(arr, dtype=np.int64))
                key = ("jobspecs", id(specs), h.hexdigest())
                run_specs, run_kw = sub, dict(reuse=key, keep=specs)
            else:
                run_specs = sub()
                key = spec_fingerprint(run_specs)
                run_kw = dict(reuse=key)
            if stoi:  # the next batch's run overlaps this batch's STOI
                key = (key, nbatch % 2)
                run_kw["reuse"] = key
            nbatch += 1
            rkey = (L, len(pairs), key)
            if stoi:
                if rkey in ready:  # the plan's waveforms are still read by that STOI
                    main.wait_event(ready[rkey])
                run_kw["on_plan"] = on_plan
            res = eng.run(nz, run_specs, clean=cl, align=align, want_waveforms=stoi, **run_kw)
            if stoi:
                ready[rkey] = state["ev"]
            vals[js, 0] = res["sse"]
            vals[js, 1] = snr_db(res["sse"], cpow[sig])
            vals[js, 2] = res["finite"]
            if "lag" in res:
                vals[js, 4] = res["lag"]
                vals[js, 5] = res["xcorr_status"]
            else:
                vals[js, 4:6] = 0
            del res
    for item in inflight:
        collect(item)
    return vals[back]


def gather_records(local, n_total, group=None, device=None):
    """All-gather per-cell records [n_local, 1 + NCOL] (RECORD_FIELDS) from
    every rank into one [n_total, NCOL] table indexed by cell_id.  Fixed-size
    rows padded to the largest shard so one all_gather_into_tensor moves them."""
    import torch
    import torch.distributed as dist
    dist_on = group is not None or (dist.is_available() and dist.is_initialized())
    world = dist.get_world_size(group) if dist_on else 1
    if dist_on:
        if device is None and dist.get_backend(group) == "nccl":
            # RCCL moves device tensors only: gather on this rank's GPU
            device = torch.device("cuda", torch.cuda.current_device())
    width = 1 + NCOL
    rec = torch.as_tensor(np.asarray(local, dtype=np.float64).reshape(-1, width))
    if dist_on:  # the collective runs at any world size, 1 included
        n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=device)
        counts = torch.zeros(world, dtype=torch.int64, device=device)
        dist.all_gather_into_tensor(counts, n, group=group)
        m = int(counts.max())
        pad = torch.full((m, width), -1.0, dtype=torch.float64)
        pad[:rec.shape[0]] = rec
        pad = pad.to(device) if device is not None else pad
        allrec = torch.empty((world * m, width), dtype=torch.float64, device=pad.device)
        dist.all_gather_into_tensor(allrec, pad, group=group)
        rec = allrec.cpu()
    rec = rec.numpy()
    if len(rec) and rec[:, 0].min() < 0:  # padding rows of the shorter shards
        rec = rec[rec[:, 0] >= 0]
    ids = rec[:, 0].astype(np.int64)
    # every cell exactly once (a count per id: O(n), no sort)
    inrange = len(ids) == 0 or (ids.min() >= 0 and ids.max() < n_total)
    seen = np.bincount(ids, minlength=n_total) if inrange and len(ids) else np.zeros(n_total, np.int64)
    if not inrange or len(ids) != n_total or (len(ids) and seen.max() != 1):
        raise RuntimeError(f"gather: {len(ids)} records for {n_total} cells "
                           f"({len(ids) - int(np.count_nonzero(seen))} duplicates or out of range)")
    if np.array_equal(ids, np.arange(n_total)):
        return rec[:, 1:]  # already in cell order (a view: no copy of the table)
    table = np.full((n_total, NCOL), np.nan)
    table[ids] = rec[:, 1:]
    return table


def _scan_records(sc, rec, ids, tol):
    """The sequential scan over the strict running maxima of one group (see
    select_best): returns (winner id or -1, score or None)."""
    incumbent, win = -1.0, -1
    for k in rec.tolist():
        if sc[k] > incumbent + tol:
            incumbent, win = float(sc[k]), int(ids[k])
    return win, (incumbent if win >= 0 else None)


def _select_best_blocks(specs, table, col, tol):
    """select_best over a JobSpecs table: each algorithm's cells of all pairs
    as one [pairs, grid] block (the columns of a (pair, algorithm) run are
    contiguous), running maxima along the grid axis in one call."""
    n_pairs = len(specs) // max(specs.per_pair, 1)
    # the score column with skipped cells at -inf (a finite cell whose score
    # is not NaN), as [pairs, cells of one pair]
    sc_all = np.asarray(table[:n_pairs * specs.per_pair, col], dtype=np.float64)
    ok = (table[:n_pairs * specs.per_pair, 2] != 0) & (sc_all == sc_all)
    sc_all = np.where(ok, sc_all, -np.inf).reshape(n_pairs, specs.per_pair)
    found = {}
    off = 0
    for a in specs.algorithms:
        n = len(specs.cells[a])
        if n:
            sc = sc_all[:, off:off + n]
            prev = np.empty_like(sc)
            prev[:, 0] = -np.inf
            np.maximum.accumulate(sc[:, :-1], axis=1, out=prev[:, 1:])
            recs = sc > prev
            for pair in range(n_pairs):
                ids = pair * specs.per_pair + off + np.arange(n)
                found[(pair, a)] = _scan_records(sc[pair], np.flatnonzero(recs[pair]), ids, tol)
        else:
            for pair in range(n_pairs):
                found[(pair, a)] = (-1, None)
        off += n
    return OrderedDict(((pair, a), found[(pair, a)]) for pair in range(n_pairs)
                       for a in specs.algorithms)


def select_best(specs, table, objective="snr", tol=None):
    """Per (pair, algorithm): the winner of the reference's sequential scan.

    Non-finite cells are skipped like finalize_enhanced returning None
    (speech_enhancement_comparison.py:102-103,173-175); the incumbent starts
    at -1 (:126-141); a NaN score (pystoi failure -> None) is skipped like
    :182-183.  Returns {(pair, alg): (cell_id or -1, score)}."""
    tol = TOLERANCE[objective] if tol is None else tol
    if objective not in ("snr", "stoi"):
        raise ValueError(f"objective {objective!r} is not scored on the device (pesq is absent)")
    col = TABLE_COLUMN[objective]
    if isinstance(specs, JobSpecs) and tol >= 0.0:
        return _select_best_blocks(specs, table, col, tol)
    groups = OrderedDict()
    if isinstance(specs, JobSpecs):  # (pair, algorithm) runs are contiguous
        per = [len(specs.cells[a]) for a in specs.algorithms]
        start = 0
        for pair in range(len(specs) // max(specs.per_pair, 1)):
            for a, n in zip(specs.algorithms, per):
                groups[(pair, a)] = np.arange(start, start + n)
                start += n
    else:
        for cid, (pair, alg, _) in enumerate(specs):
            groups.setdefault((pair, alg), []).append(cid)
    best = OrderedDict()
    for key, ids in groups.items():
        ids = np.asarray(ids, dtype=np.int64)
        sc = table[ids, col]
        ok = (table[ids, 2] != 0) & (sc == sc)  # finite cell, score not NaN
        sc = np.where(ok, sc, -np.inf)
        incumbent, win = -1.0, -1
        if tol >= 0.0 and len(sc):
            # Only a strict running maximum can replace the incumbent: after
            # any cell j the incumbent is >= sc[j] - tol (it took sc[j], or
            # sc[j] <= incumbent + tol), so a cell at or below an earlier score
            # never clears incumbent + tol and leaves the state alone.  The
            # scan runs over those records only (a few per group).
            prev = np.maximum.accumulate(np.concatenate(([-np.inf], sc[:-1])))
            best[key] = _scan_records(sc, np.flatnonzero(sc > prev), ids, tol)
            continue
        else:
            start = 0  # negative tolerance: the plain jump scan
            while start < len(ids):
                hit = np.flatnonzero(sc[start:] > incumbent + tol)
                if len(hit) == 0:
                    break
                k = start + int(hit[0])
                incumbent, win, start = float(sc[k]), int(ids[k]), k + 1
        best[key] = (win, incumbent if win >= 0 else None)
    return best


def run_grid(clean, noisy, specs, compute=None, group=None, device=None, objective="snr"):
    """Run every cell of ``specs`` across the ranks of ``group`` (or locally)
    and return (table [n_cells, NCOL] = sse, snr, finite, stoi, lag, xstatus;
    winners).  Every rank
    gets the full table (all_gather); the selection is the deterministic
    sequential scan, identical on every rank."""
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    lengths = [len(x) for x in noisy]
    rank_of, _ = assign_shards(specs, lengths, world)
    ids = np.nonzero(rank_of == rank)[0]
    compute = compute or engine_compute
    vals = compute(clean, noisy, specs, ids) if len(ids) else np.zeros((0, NCOL))
    if not dist_on and len(ids) == len(specs):  # one process, every cell in order: no gather
        table = np.asarray(vals, dtype=np.float64)
    else:
        local = np.concatenate([ids[:, None].astype(np.float64), vals], axis=1)
        table = gather_records(local, len(specs), group=group, device=device)
    return table, select_best(specs, table, objective)


def _snr_baseline(c, n):
    m = min(len(c), len(n))
    err = np.sum((c[:m] - n[:m]) ** 2)
    return math.inf if err == 0 else float(10 * np.log10(np.sum(c[:m] ** 2) / (err + 1e-10)))


def _device_stoi(clean, test, sr):
    from .metrics import calculate_stoi
    return calculate_stoi(clean, test, sr)


def _opt(v):
    return None if v != v else float(v)


def optimize_parameters(clean_reference, noisy_audio, sr, algorithm, param_ranges=None,
                        compute=None, stoi_fn=None):
    """Single-pair, single-algorithm mirror of the reference's
    optimize_parameters (speech_enhancement_comparison.py:109-252), scored by
    STOI and SNR: returns {'stoi': {'score', 'params', 'cell', 'snr'},
    'snr': {'score', 'params', 'cell', 'stoi'}, 'baseline': {'stoi', 'snr'},
    'improvements': {'stoi', 'snr'}, 'table'}; raises ValueError like :233-235
    when no cell produced a finite output.  The 'stoi' entry is None when no
    cell has a STOI value (a compute function that does not score STOI)."""
    from .engine import canonical_algo
    if sr != 16000:
        raise ValueError("the device path runs at 16 kHz (prepare_pair resamples to 16 kHz)")
    alg = canonical_algo(algorithm)
    grids = {alg: param_ranges or ALGORITHM_GRIDS[alg]}
    specs = job_specs(1, [alg], grids)
    clean = [np.asarray(clean_reference, np.float64)]
    noisy = [np.asarray(noisy_audio, np.float64)]
    table, best = run_grid(clean, noisy, specs, compute=compute)
    cid, score = best[(0, alg)]
    if cid < 0:
        raise ValueError("Optimization failed for snr - no valid parameters found!")
    base = _snr_baseline(clean[0], noisy[0])
    out = {"snr": {"score": score, "params": dict(specs[cid][2]), "cell": int(cid),
                   "stoi": _opt(table[cid, 3])},
           "baseline": {"snr": base}, "improvements": {"snr": score - base}, "table": table,
           "stoi": None}
    sid, sscore = select_best(specs, table, "stoi")[(0, alg)]
    if sid >= 0:
        bstoi = (stoi_fn or _device_stoi)(clean[0], noisy[0], sr) or 0  # :115 "or 0"
        out["stoi"] = {"score": sscore, "params": dict(specs[sid][2]), "cell": int(sid),
                       "snr": float(table[sid, 1])}
        out["baseline"]["stoi"] = bstoi
        out["improvements"]["stoi"] = sscore - bstoi
    return out


def run_sweep(clean, noisy, stems, out_root, sr=16000, algorithms=None, grids=None,
              group=None, device=None):
    """The reference's batch driver (main, speech_enhancement_comparison.py:375-473)
    on the device: every pair x algorithm x grid cell scored after
    finalize_enhanced (STOI and SNR), the STOI-best and SNR-best cells per
    (pair, algorithm) selected by the sequential tolerance scan, their
    waveforms written as results_{alg}/{stem}_{alg}_optimized_stoi.wav (the
    reference's name, :303) and ..._optimized_snr.wav, and the summary files
    (results.write_summary) under results_summary/.  Rank 0 writes."""
    import torch
    import torch.distributed as dist
    from . import results
    from .engine import Engine
    from .metrics import StoiPlan
    grids = grids or ALGORITHM_GRIDS
    algorithms = list(algorithms or grids)
    specs = job_specs(len(noisy), algorithms, grids)
    table, best = run_grid(clean, noisy, specs, group=group, device=device)
    rank = dist.get_rank(group) if (dist.is_available() and dist.is_initialized()) else 0
    if rank != 0:
        return None
    best_stoi = select_best(specs, table, "stoi")
    eng = Engine()
    rows = []
    for pair, stem in enumerate(stems):
        c = np.asarray(clean[pair], np.float64)
        n = np.asarray(noisy[pair], np.float64)
        snr_noisy = _snr_baseline(c, n)
        m = min(len(c), len(n))
        plan = StoiPlan(torch.as_tensor(c[:m]).cuda().view(1, -1))
        nf = torch.as_tensor(n[:m].astype(np.float32)).cuda()
        stoi_noisy = _opt(plan.score(nf, [0], [0], clip=False)[0])
        x = torch.as_tensor(n).cuda().view(1, -1)
        cl = torch.as_tensor(c).cuda().view(1, -1)
        for alg in algorithms:
            cid, score = best[(pair, alg)]
            if cid < 0:
                raise ValueError(f"Optimization failed for snr - no valid parameters found! ({stem}, {alg})")
            sid, sscore = best_stoi[(pair, alg)]
            out_dir = os.path.join(out_root, f"results_{alg}")
            os.makedirs(out_dir, exist_ok=True)
            for tag, k in (("snr", cid), ("stoi", sid)):
                if k < 0:
                    continue
                res = eng.run(x, [(0, alg, specs[k][2])], clean=cl, want_waveforms=True, align=True)
                y = res["y"][0].cpu().numpy().astype(np.float64)
                e = results.shift_and_fit(y, int(res["lag"][0]), len(c))
                results.write_wav_pcm16(os.path.join(out_dir, f"{stem}_{alg}_optimized_{tag}.wav"),
                                        e, sr)
            rows.append(results.result_row(
                stem, alg, sr, snr_noisy, float(score), specs[cid][2], stoi_noisy=stoi_noisy,
                stoi_best=None if sid < 0 else float(sscore),
                stoi_params=None if sid < 0 else specs[sid][2],
                snr_stoiopt=None if sid < 0 else float(table[sid, 1])))
    results.write_summary(rows, algorithms, os.path.join(out_root, "results_summary"))
    return rows
