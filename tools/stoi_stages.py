"""Per-stage time of stoi_cells_kernel inside the real kernel (VERDICT r04
item 3): a build with -DCSE_STOI_STAMPS records, per cell, the workgroup's
shader cycles (s_memtime) between its barriers by stage; this runs the
tools/bench_stoi.py workload on such a build and prints the mean cycles per
cell and the share of each stage.

    python tools/build_stamps.py            (CPU: builds libcse_stamps.so)
    CSE_LIB=classical_speech_enhancement_amd/libcse_stamps.so python tools/stoi_stages.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from classical_speech_enhancement_amd.metrics import StoiPlan  # noqa: E402
from classical_speech_enhancement_amd.synth import make_pair  # noqa: E402

STAGES = ["tables+first table", "staging", "resampling", "rfft", "band sums", "phase B"]


def main(cells=4096, pairs=4):
    prs = [make_pair(100 + i, 10.0) for i in range(pairs)]
    clean = torch.as_tensor(np.stack([c for c, _ in prs])).cuda()
    L = clean.shape[1]
    rng = np.random.default_rng(0)
    noisy = torch.as_tensor(np.stack([n for _, n in prs]).astype(np.float32)).cuda()
    sig = np.arange(cells) % pairs
    gains = torch.as_tensor(rng.uniform(0.3, 3.0, cells).astype(np.float32)).cuda()
    y = (noisy[torch.as_tensor(sig).cuda()] * gains[:, None]).contiguous().view(-1)
    lag = rng.integers(-1600, 1601, cells)
    plan = StoiPlan(clean)
    off = np.arange(cells, dtype=np.int64) * L
    plan.score_async(y, off, sig, lag=lag)
    torch.cuda.synchronize()
    buf = torch.zeros(cells * 8, dtype=torch.int64, device="cuda")
    lib = plan.lib
    lib.cse_stoi_stamp_buffer.argtypes = [ctypes.c_void_p]
    assert lib.cse_stoi_stamp_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.score_async(y, off, sig, lag=lag)
    e1.record()
    torch.cuda.synchronize()
    lib.cse_stoi_stamp_buffer(ctypes.c_void_p(0))
    st = buf.view(cells, 8).cpu().numpy().astype(np.float64)
    mean = st.mean(axis=0)
    tot = mean[6]
    out = {"cells": cells, "launch_ms": e0.elapsed_time(e1), "cycles_per_cell_total": tot,
           "stages": {n: {"cycles": mean[k], "share": mean[k] / tot} for k, n in enumerate(STAGES)},
           "unaccounted_share": 1 - mean[:6].sum() / tot}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
