"""Stage-by-stage comparison of the HIP path with the oracle (GPU box debug aid)."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import oracle  # noqa: E402
from oracle import gain_ref  # noqa: E402
from classical_speech_enhancement_amd.engine import Engine  # noqa: E402
from classical_speech_enhancement_amd.synth import make_pair  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    clean, noisy = make_pair(7, seconds=0.75)
    eng = Engine()
    x = torch.as_tensor(noisy).cuda().view(1, -1)
    for n_fft, hop in ((512, 128), (512, 256), (1024, 256)):
        Y, P = eng.stft(x, n_fft, hop)
        Yd = Y[0].double().cpu().numpy()
        Yd = (Yd[..., 0] + 1j * Yd[..., 1]).T
        Yr = oracle.stft(noisy, n_fft, hop)
        print(n_fft, hop, "Y rel", rel(Yd, Yr), "P rel", rel(P[0].cpu().numpy().T, np.abs(Yr) ** 2))
        Nd = eng.noise_estimate("percentile", P, 10.0, 1e-10)[0].cpu().numpy()
        Nr = oracle.percentile_noise(np.abs(Yr) ** 2, 1e-10, 10.0)[:, 0]
        print("   N pct rel", rel(Nd, Nr))
        p = dict(alpha=2.0, beta=0.005, n_fft=n_fft, hop_length=hop, noise_percentile=10.0,
                 noise_method="percentile")
        res = eng.run(x, [(0, "spectralSubtractor", p)], want_waveforms=True, want_gains=True)
        y = res["y"][0].double().cpu().numpy()
        yr = oracle.spectral_subtraction(noisy, 16000, **p)
        print("   SS y rel", rel(y, yr))
        # identity gain check via SS with alpha=0, beta=1 -> Ps = max(P, N) ... use wiener floor 1
        p2 = dict(alpha=0.9, gain_floor=1.0, n_fft=n_fft, hop_length=hop, noise_percentile=10.0,
                  noise_method="percentile")
        r2 = eng.run(x, [(0, "wiener", p2)], want_waveforms=True)
        y2 = r2["y"][0].double().cpu().numpy()
        print("   identity (G=1) roundtrip rel", rel(y2, noisy),
              "oracle istft(Y)", rel(oracle.istft(Yr, hop_length=hop, length=len(noisy)), noisy))
        k = np.argmax(np.abs(y2 - noisy))
        print("   worst sample", k, y2[k], noisy[k])
        d = np.abs(y2 - noisy)
        print("   err by position (first 40 / mid / last 40):",
              d[:40].max(), d[1000:2000].max(), d[-40:].max())
        print("   err pattern mod 32 (mid):", np.round(d[2048:2048 + 64] * 1e3, 3))


if __name__ == "__main__":
    main()
