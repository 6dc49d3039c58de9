"""Per-stage time of enhance_kernel inside the real kernel: a build with
-DCSE_ENH_STAMPS records, per workgroup (its wave 0), the shader cycles
(s_memtime) between the frame loop's stage markers; this runs one launch of
the bench workload (PAIRS pairs, one n_fft half of the HEAD grid) on such a
build and prints, per (hop, algorithm) specialisation, the mean cycles per
workgroup and the share of each stage.  Cycles are wall cycles of one wave:
they include the issue slots the SIMD's other waves take.

    python tools/build_stamps.py            (CPU: builds libcse_stamps.so)
    CSE_LIB=classical_speech_enhancement_amd/libcse_stamps.so python tools/enhance_stages.py [--pairs 13 --nfft 512]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STAGES = ["barrier + loop top", "gain", "mirror exchange", "row staging", "pass-1 DFT",
          "transpose + pass-2 DFT", "window", "retire"]
ALGO = {0: "ss", 1: "wiener", 2: "mmse", 3: "omlsa"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=13)
    ap.add_argument("--nfft", type=int, default=512)
    a = ap.parse_args()
    import torch
    from classical_speech_enhancement_amd.engine import Engine
    from classical_speech_enhancement_amd.parameter_ranges import grid_specs
    from classical_speech_enhancement_amd.synth import make_pair
    pairs = [make_pair(i, 10.0) for i in range(a.pairs)]
    clean = torch.as_tensor(np.stack([c for c, _ in pairs])).cuda()
    noisy = torch.as_tensor(np.stack([n for _, n in pairs])).cuda()
    plan = Engine().plan(a.pairs, 160000, grid_specs(a.pairs, a.nfft), with_clean=True).plans[0]
    plan.prepare(noisy, clean)
    plan.enhance()
    torch.cuda.synchronize()
    n_groups = plan.n_packed // plan.lib.cse_cells_per_group(a.nfft)
    buf = torch.zeros(n_groups * 10, dtype=torch.int64, device="cuda")
    fn = getattr(plan.lib, f"cse_enhance_stamp_buffer_{a.nfft}")
    fn.argtypes = [ctypes.c_void_p]
    assert fn(ctypes.c_void_p(buf.data_ptr())) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.enhance()
    e1.record()
    torch.cuda.synchronize()
    fn(ctypes.c_void_p(0))
    st = buf.view(n_groups, 10).cpu().numpy()
    out = {"pairs": a.pairs, "n_fft": a.nfft, "groups": int(n_groups), "launch_ms": e0.elapsed_time(e1),
           "stage_names": STAGES, "by_specialisation": {}}
    tot_all = st[:, :8].astype(np.float64).sum()
    for (alg, hop) in sorted({(int(r[8]), int(r[9])) for r in st}):
        m = (st[:, 8] == alg) & (st[:, 9] == hop)
        acc = st[m, :8].astype(np.float64)
        mean = acc.mean(axis=0)
        out["by_specialisation"][f"{ALGO.get(alg, alg)}-{hop}"] = {
            "groups": int(m.sum()), "cycles_per_group": float(mean.sum()),
            "share_of_launch_cycles": float(acc.sum() / tot_all),
            "stage_share": {n: round(float(mean[k] / mean.sum()), 4) for k, n in enumerate(STAGES)}}
    allm = st[:, :8].astype(np.float64).sum(axis=0)
    out["all"] = {n: round(float(allm[k] / allm.sum()), 4) for k, n in enumerate(STAGES)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
