"""bench.py's host-side multi-rank instrumentation on CPU: which pair a rank
checks and which of its cells, and the per-rank stats / parity gathers over
world_size 2 (gloo), the way the 8-GPU node runs them over RCCL."""

import os
import socket

import numpy as np
import pytest

import bench
from classical_speech_enhancement_amd import search
from classical_speech_enhancement_amd.parameter_ranges import grid_specs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Args:
    seconds = 10.0
    pairs = None
    pairs_total = 100


@pytest.mark.parametrize("world", [1, 8])
def test_rank_pair_cells_cover_the_rank_s_most_held_pair(world):
    """rank_job's local specs -> the pair slot a rank checks and the grid index
    of each held cell (grid_specs(1, 512) order, the oracle's cell order)."""
    g512 = grid_specs(1, 512)
    for rank in range(world):
        pair_ids, local, gids, _, _ = bench.rank_job(_Args, world, rank, 512)
        slot, held = bench.rank_pair_cells(local, 512)
        counts = {}
        for s, _, _ in local:
            counts[s] = counts.get(s, 0) + 1
        assert len(held) == max(counts.values())
        for g, j in held.items():
            s, alg, p = local[j]
            assert s == slot and (alg, p) == (g512[g][1], g512[g][2])
            # the global cell id is pair-major grid order
            assert gids[j] == pair_ids[slot] * len(g512) + g
        cells = bench.pick_parity_cells(10.0, 512, held)
        assert 16 <= len(cells) <= 64 and all(c in held for c in cells)
        if world == 1:
            assert slot == 0 and pair_ids[slot] == 0 and len(cells) == 64


def _rank(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        ctx = (dist, torch.device("cpu"), world)
        st = {"wall_s": 1.0 + rank, "kernel_ms": 10.0 * (rank + 1), "analysis_ms": 2.0,
              "units": 100 + rank, "cells": 7, "pairs": 3}
        r = bench.gather_rank_stats(st, ctx)
        par = {"pass": rank == 0, "pair": 5 + rank, "cells_snr": 64, "cells_waveform": 64,
               "max_rel_l2": 1e-7 * (rank + 1), "max_rel_max": 2e-7, "max_snr_abs_db": None}
        p = bench.gather_parity(par, ctx)
        np.save(os.path.join(out, f"r{rank}.npy"),
                np.array([r["imbalance_max_over_mean"]["kernel_ms"],
                          r["imbalance_max_over_mean"]["wall_s"],
                          sum(x["units"] for x in r["per_rank"]),
                          float(p["pass"]), p["per_rank"][1]["pair"],
                          p["per_rank"][1]["max_rel_l2"], p["ranks_checked"],
                          float(p["per_rank"][0]["max_snr_abs_db"] is None)]))
    finally:
        dist.destroy_process_group()


def test_rank_stats_and_parity_gather_world2(tmp_path):
    import torch.multiprocessing as tmp
    tmp.spawn(_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    a, b = np.load(tmp_path / "r0.npy"), np.load(tmp_path / "r1.npy")
    assert np.array_equal(a, b)  # every rank sees the same gathered figures
    assert a[0] == pytest.approx(20.0 / 15.0) and a[1] == pytest.approx(2.0 / 1.5)
    assert a[2] == 201
    assert a[3] == 0.0  # rank 1 failed: the line fails
    assert a[4] == 6 and a[5] == pytest.approx(2e-7) and a[6] == 2 and a[7] == 1.0


def test_single_process_gathers_need_no_process_group():
    import torch
    ctx = (None, torch.device("cpu"), 1)
    r = bench.gather_rank_stats({"wall_s": 1.0, "kernel_ms": 3.0, "analysis_ms": 1.0,
                                 "units": 10, "cells": 2, "pairs": 1}, ctx)
    assert r["imbalance_max_over_mean"]["kernel_ms"] == 1.0 and r["per_rank"][0]["units"] == 10
    p = bench.gather_parity(None, ctx)
    assert not p["pass"] and p["ranks_checked"] == 0


def test_roofline_block_prints_no_bandwidth_from_nominal_bytes():
    roof = bench.roofline_block(512, 457237200, 170.0)
    assert roof["nominal_unfused_bytes_per_launch"] == 457237200 * 3084
    assert not any("algorithmic_GBps" in k or "algorithmic_frac" in k for k in roof)
    for k, v in roof.items():
        if k.endswith("GBps") and v is not None:
            assert v < 8000.0, (k, v)
    if roof.get("traffic"):
        assert 0 < roof["pmc_traffic_over_nominal"] < 1


def test_job_units_match_shards():
    specs = search.job_specs(100, n_fft=512)
    total = 0
    for rank in range(8):
        _, local, _, units, _ = bench.rank_job(_Args, 8, rank, 512)
        total += len(local)
    assert total == len(specs) and units == 100 * 4572372


@pytest.mark.parametrize("n_fft", [512, 1024])
def test_roofline_block_prices_the_committed_pmc(n_fft):
    """The line's VALU roofline from the committed PMC of this build
    (profiles/pmc_enhance{n_fft}_<round>.json, digest-matched), every
    instruction kind priced at the SIMD cycles the chip-wide micro-benchmarks
    measure (tools/micro/valu_cal.hip, valu_mix.hip): f32 VALU 2, packed
    v_pk_*_f32 4, transcendental 8, fp64 4 (r06; r05 priced a packed
    instruction at 2 and a transcendental at 4).  frac = cycles / (1024 SIMDs x 2.4 GHz x kernel time);
    the packed count is the measured one (scalar-build class counts minus the
    product's), and it must agree with the FP32 FLOP counter; no
    dense_at_occupancy block and no bandwidth derived from SURVEY 8(d)'s
    nominal bytes."""
    import json
    units = 457237200
    pmc = bench.load_pmc(units, n_fft)
    if not pmc or pmc.get("kernel_src_sha") != bench.kernel_src_sha():
        pytest.skip("no committed PMC profile of these kernel sources")
    ks_ms = pmc["kernel_ms"]
    r = bench.roofline_block(n_fft, units, ks_ms)
    assert r["bound"] == "valu" and r["pmc_matches_build"]
    assert "frac_vs_dense_stream" not in r and "dense_at_occupancy" not in r
    ks = ks_ms / 1e3
    v, t = pmc["sq_insts_valu"], pmc["sq_insts_valu_trans"]
    pk, f64 = pmc["packed_insts"], pmc.get("sq_insts_valu_f64") or 0.0
    need = 2 * (v - t - pk - f64) + 4 * (pk + f64) + 8 * t
    assert abs(r["frac"] - need / (bench.SIMDS * bench.CLOCK * ks)) < 1e-12
    assert r["packed_insts"] == pk
    if n_fft == 1024:
        assert pk == 0  # the 1024 kernel is scalar f32
    else:
        assert pk > 0.5 * (v - t - f64)  # most of the 512 kernel's f32 work is packed
        chk = pmc["packed"]["flop_check"]["ratio"]
        assert abs(chk - 1) < 0.02, chk
    if pmc.get("sq_insts_valu_flops_fp32"):
        f = r["fp32_flops"]
        assert abs(f["frac"] - pmc["sq_insts_valu_flops_fp32"] * 64 / ks / 157.3e12) < 1e-12
        assert 0 < f["frac"] < 1
    assert 0.3 < r["frac"] < 1.0
    assert all("GBps" not in k or (r[k] or 0) < 8000 for k in r)
    json.dumps(r)  # the line must serialise


def test_valu_prices_match_the_committed_calibration():
    """bench.py's per-kind VALU prices are the chip-wide micro-benchmark's
    (profiles/r06_micro_valu_cal.json, tools/micro/valu_cal.hip and
    valu_mix.hip, 8 waves/SIMD): packed f32 and fp64 at 4, a transcendental at
    8 (within 10 %), and the scalar f32 price 2 no higher than what the
    dual-issuing mixes reach (2.3-2.5) — a lower bound on scalar cost."""
    import json
    path = os.path.join(bench.REPO, "profiles", "r06_micro_valu_cal.json")
    cal = json.load(open(path))
    s = cal["summary_8_waves"]
    assert abs(s["v_pk_fma_f32"]["cycles_per_wave_inst_8w"] / bench.PK_CYC - 1) < 0.1
    assert abs(s["v_exp_f32"]["cycles_per_wave_inst_8w"] / bench.TRANS_CYC - 1) < 0.1
    assert abs(s["v_fma_f64"]["cycles_per_wave_inst_8w"] / bench.F64_CYC - 1) < 0.15
    mix = cal["mix"]
    assert bench.VALU_CYC <= min(mix["v_add_f32 + v_add_f32"]["8"], mix["v_fma_f32(vvv) + v_add_f32"]["8"])
    # the FP32 peak needs packed math: a scalar FMA stream reaches about half
    assert s["v_pk_fma_f32"]["tflops_8w"] > 1.8 * s["v_fma_f32"]["tflops_8w"]


def test_kernel_digest_ignores_comments_only():
    """kernel_src_sha hashes the code of the enhance sources (code_text):
    comments and whitespace do not move it, code and string literals do."""
    import bench
    src = open(os.path.join(bench.REPO, "include", "cse.h")).read()
    assert bench.code_text(src) == bench.code_text(src.replace("/*", "/* edited:", 1))
    assert bench.code_text(src) == bench.code_text("// a new comment line\n" + src + "\n\n")
    t = 'int a = 1; // c\nconst char* s = "// kept /* kept */"; /* x */ char q = \'/\';'
    assert bench.code_text(t) == 'int a = 1; const char* s = "// kept /* kept */"; char q = \'/\';'
    assert bench.code_text("int a = 1;") != bench.code_text("int a = 2;")
    assert len(bench.kernel_src_sha()) == 16
