"""The CPU baseline's scaling with process count on the GPU box (host only).

bench.py's cpu_baseline leg runs the oracle (test infrastructure: the
reference's algorithm restated in fp64 numpy) on the box's per-GPU CPU share,
16 single-threaded processes.  This times the same leg at 1, 4 and 16
processes so a node-level figure can be stated as a measured-slope
extrapolation instead of a guess.

    python tools/cpu_scaling.py [--budget S]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=10.0)
    a = ap.parse_args()
    import bench
    out = {"cpu_model": bench._cpu_model(), "os_cpu_count": os.cpu_count(), "points": []}
    for procs in (1, 4, 16):
        os.environ["CSE_CPU_BASELINE_PROCS"] = str(procs)
        base, _, _ = bench.cpu_run(a.budget, 10.0, 512, [], timed=True)
        out["points"].append({"procs": procs, "evals_per_s": base["value"],
                              "per_proc": base["value"] / procs})
        print(json.dumps(out["points"][-1]), flush=True)
    p1 = out["points"][0]["per_proc"]
    for pt in out["points"]:
        pt["efficiency_vs_1"] = pt["per_proc"] / p1
    print(json.dumps(out))


if __name__ == "__main__":
    main()
