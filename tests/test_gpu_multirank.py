"""The multi-rank paths on one GPU (needs a GPU): two ranks share the card and
talk over gloo, the way the 8-GPU node runs them over RCCL (one process per
GPU).  Checks that bench.py's weak-scaling line counts both ranks' work and
that the sharded device sweep (search.run_grid) gives every rank the same
table as one process computing every cell."""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture(scope="module")
def gpu():
    # device_count() does not initialise the GPU in this process (is_available()
    # would): the ranks below are started as child processes, which must not
    # be forked from a process that holds GPU state
    import torch
    if torch.cuda.device_count() == 0:
        pytest.skip("no GPU")


def test_bench_two_ranks_weak_scaling(gpu):
    env = dict(os.environ, CSE_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--pairs", "1", "--seconds", "2", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    units = d["config"]["units_per_step"]  # both ranks' pairs
    assert units == 2 * d["config"]["units_per_step_rank0"]
    assert d["value"] == pytest.approx(units / (d["ms_per_step"] / 1e3), rel=1e-6)
    rk = d["ranks"]["per_rank"]
    assert [r["units"] for r in rk] == [units // 2] * 2 and [r["pairs"] for r in rk] == [1, 1]
    assert d["parity"]["pass"] and [p["pair"] for p in d["parity"]["per_rank"]] == [0, 1]


def _rank(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from classical_speech_enhancement_amd import search
    from _grid_worker import SMALL_GRIDS, pairs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        clean, noisy = pairs(3, 1.2)
        specs = search.job_specs(len(noisy), grids=SMALL_GRIDS)
        table, best = search.run_grid(clean, noisy, specs)
        np.save(os.path.join(outdir, f"rank{rank}.npy"), table)
    finally:
        dist.destroy_process_group()


def test_run_grid_two_ranks_equals_one_process(gpu, tmp_path):
    import torch.multiprocessing as tmp
    from classical_speech_enhancement_amd import search
    from _grid_worker import SMALL_GRIDS, pairs
    tmp.spawn(_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    # the reference table: this process touches the GPU only after the ranks exited
    t0 = np.load(tmp_path / "rank0.npy")
    t1 = np.load(tmp_path / "rank1.npy")
    clean, noisy = pairs(3, 1.2)
    specs = search.job_specs(len(noisy), grids=SMALL_GRIDS)
    ref, _ = search.run_grid(clean, noisy, specs)
    assert np.array_equal(t0, t1, equal_nan=True)
    assert np.array_equal(t0, ref, equal_nan=True)


def test_bench_two_ranks_strong_scaling(gpu):
    """--pairs-total: the fixed job's cells split by search.assign_shards; value
    counts the whole job once."""
    env = dict(os.environ, CSE_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--pairs-total", "3", "--seconds", "2", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    units = d["config"]["units_per_step"]
    assert d["value"] == pytest.approx(units / (d["ms_per_step"] / 1e3), rel=1e-6)
    assert 0 < d["config"]["units_per_step_rank0"] < units


def test_bench_rccl_world1(gpu):
    """bench.py under torchrun with the default backend "nccl" (RCCL) at world
    size 1: the per-step all_gather_into_tensor of device records, the
    all_reduce of the step time and the barriers run through RCCL."""
    env = {k: v for k, v in os.environ.items() if k != "CSE_DIST_BACKEND"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
           "--pairs-total", "2", "--seconds", "2", "--no-cpu-baseline", "--no-parity"]
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and "RCCL" in d["config"]["parallelism"]


def _rccl_rank(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from classical_speech_enhancement_amd import search
    from _grid_worker import SMALL_GRIDS, pairs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        assert dist.get_backend() == "nccl"
        clean, noisy = pairs(3, 1.2)
        specs = search.job_specs(len(noisy), grids=SMALL_GRIDS)
        table, _ = search.run_grid(clean, noisy, specs)  # device=None -> this rank's GPU
        np.save(os.path.join(outdir, f"rccl{rank}.npy"), table)
    finally:
        dist.destroy_process_group()


def test_run_grid_rccl_world1_equals_local(gpu, tmp_path):
    """search.run_grid / gather_records under init_process_group("nccl"): the
    count and record all_gather_into_tensor calls move device tensors through
    RCCL; the table equals the one computed without torch.distributed."""
    import torch.multiprocessing as tmp
    from classical_speech_enhancement_amd import search
    from _grid_worker import SMALL_GRIDS, pairs
    tmp.spawn(_rccl_rank, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    t0 = np.load(tmp_path / "rccl0.npy")
    clean, noisy = pairs(3, 1.2)
    specs = search.job_specs(len(noisy), grids=SMALL_GRIDS)
    ref, _ = search.run_grid(clean, noisy, specs)
    assert np.array_equal(t0, ref, equal_nan=True)


def test_bench_eight_ranks_strong_scaling_rehearsal(gpu, tmp_path):
    """The 8-GPU node's strong-scaling run, rehearsed with 8 gloo ranks sharing
    the card: BASELINE config 4's 100-pair job sharded by search.assign_shards.
    The line counts the whole job once, each rank holds at most 14 pairs (whole
    pairs plus a part at each end of its run), and the gathered per-cell
    records equal a world-1 run's bit for bit.  The line is instrumented for the
    first hardware run: per-rank kernel / analysis / wall time, units, cells
    and pairs with their max / mean spread, and a parity check on every rank
    (its most-held pair's stratified cells against the oracle)."""
    common = ["--steps", "1", "--warmup", "1", "--pairs-total", "100", "--full-grid-steps", "0",
              "--no-sweep", "--no-cpu-baseline"]
    # 8 ranks share this box's CPU share: 2 oracle processes each
    env = dict(os.environ, CSE_DIST_BACKEND="gloo", CSE_CPU_BASELINE_PROCS="2")
    t8, t1 = tmp_path / "t8.npy", tmp_path / "t1.npy"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "8", "--dump-table", str(t8)] + common
    out = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 8 and d["scaling"] == "strong"
    assert d["config"]["units_per_step"] == 100 * 4572372
    assert d["config"]["cells_total"] == d["config"]["gathered_cells_finite"] == 487200
    assert d["config"]["pairs_rank0"] <= 14
    assert abs(d["config"]["units_per_step_rank0"] - 100 * 4572372 / 8) < 0.02 * 100 * 4572372 / 8
    assert d["value"] == pytest.approx(d["config"]["units_per_step"] / (d["ms_per_step"] / 1e3),
                                       rel=1e-6)
    rk = d["ranks"]["per_rank"]
    assert len(rk) == 8
    assert sum(r["units"] for r in rk) == d["config"]["units_per_step"]
    assert sum(r["cells"] for r in rk) == 487200
    assert all(r["kernel_ms"] > 0 and r["analysis_ms"] > 0 and r["wall_s"] > 0 and
               1 <= r["pairs"] <= 14 for r in rk)
    imb = d["ranks"]["imbalance_max_over_mean"]
    assert 1.0 <= imb["units"] < 1.02 and imb["kernel_ms"] >= 1.0 and imb["wall_s"] >= 1.0
    par = d["parity"]
    assert par["pass"] and par["ranks_checked"] == 8 and len(par["per_rank"]) == 8
    assert len({p["pair"] for p in par["per_rank"]}) == 8  # each rank checks a pair of its own
    assert all(p["cells_waveform"] >= 16 and p["max_rel_l2"] <= 1e-5 for p in par["per_rank"])
    one = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dump-table", str(t1),
                          "--no-parity"] + common, cwd=REPO, capture_output=True, text=True,
                         timeout=420)
    assert one.returncode == 0, one.stderr[-3000:]
    a, b = np.load(t8), np.load(t1)
    assert a.shape == b.shape == (487200, 2)
    assert np.array_equal(a, b)
    print("8-rank rehearsal:", d["config"]["parallelism"], "pairs on rank 0:",
          d["config"]["pairs_rank0"], "ms/step", d["ms_per_step"], "spread", imb,
          "parity", [(p["pair"], p["max_rel_l2"]) for p in par["per_rank"]])
