"""Per-call time of the alignment lag kernel on flat, periodic and shifted heads.

The parity test tests/test_gpu_parity.py::test_alignment_flat_and_periodic_heads
checks the lags of these heads against oracle.align_lag; this script times
them (r05 removed the flat-head cliff: 43.6 ms -> 0.3 ms per call).  One
cse_xcorr_lag launch per head, HIP events on the stream it is launched on
(torch's current stream), median of 20 after a warm call; the host-side
preparation (uploads, cse_xcorr_prepare) is outside the events.

    python tools/time_alignment.py [out.json]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, REPO)


def main(out=None):
    import torch
    from classical_speech_enhancement_amd import _lib
    from classical_speech_enhancement_amd.engine import Engine, _ptr, _stream
    from classical_speech_enhancement_amd.synth import make_pair
    eng = Engine()
    lib, dev = eng.lib, eng.device
    clean, _ = make_pair(3, 3.0)
    n = 32000
    max_lag = 1600
    rng = np.random.default_rng(5)
    heads = {
        "zero": np.zeros(len(clean)),
        "dc": np.full(len(clean), 0.25),
        "dc_noise": 0.5 + 1e-4 * rng.standard_normal(len(clean)),
        "tone": 0.3 * np.sin(2 * np.pi * np.arange(len(clean)) / 37.0),
        "shift40": np.roll(clean, 40),
    }
    c = torch.as_tensor(clean[:n]).to(dev).view(1, -1)
    ws = torch.empty(int(lib.cse_xcorr_workspace_bytes(1, n, n, max_lag)), dtype=torch.uint8, device=dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    sig_of = torch.zeros(1, dtype=torch.int32, device=dev)
    lag = torch.zeros(1, dtype=torch.int32, device=dev)
    zero = torch.zeros(1, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    st = _stream()
    _lib.check(lib.cse_xcorr_prepare(_ptr(c), 1, n, n, max_lag, _ptr(ws), st), "cse_xcorr_prepare")
    res = {"what": ("HIP-event time of one cse_xcorr_lag launch (one cell, 2-s head, lags within "
                    "0.1 s), median of 20 after a warm call"), "heads": {}}
    for name, h in heads.items():
        head = torch.as_tensor(h[:n].astype(np.float32)).to(dev)

        def launch():
            _lib.check(lib.cse_xcorr_lag(_ptr(head), _ptr(off), _ptr(sig_of), 1, 1, n, max_lag, _ptr(ws),
                                         _ptr(lag), _ptr(zero), _ptr(status), None, st), "cse_xcorr_lag")
        launch()
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        res["heads"][name] = {"ms_median": float(np.median(ts)), "ms_min": float(np.min(ts)),
                              "lag": int(lag.item()), "status": int(status.item())}
        print(f"{name:9s} {np.median(ts):.4f} ms  lag {int(lag.item())}  status {int(status.item())}")
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return res


if __name__ == "__main__":
    main(*sys.argv[1:2])
