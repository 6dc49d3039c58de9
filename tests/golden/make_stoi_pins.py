"""Make tests/golden/stoi_pins.npz — STOI values the reference computed itself.

Data only: the reference's committed enhanced WAVs (Document/Presentation,
16-kHz PCM16) and the STOI numbers it recorded for the same stems in
Code/results_summary/*/all_results.json (rows written by
speech_enhancement_comparison.py:327-345 from pystoi 0.4.1).  The clean/noisy
16-kHz signals come from presentation_wavs.npz (make_golden.py).

  stoi|<stem>|noisy            <- row["stoi_noisy"]
  stoi|<stem>|<var>            <- row["stoi_<var>opt"], var in stoi/pesq/bal
  enhanced|<stem>|<var>        <- <stem>_<alg>_optimized_<var>.wav (int16)

Which results folder a WAV belongs to is fixed by its parameters:
29_menschenWM_mitTrueNoise for p257_090 (true-noise best params) and
21_kombiWM_ohneTrueNoise for p257_135 (min-tracking/percentile best params).
Run in the dev container only: python tests/golden/make_stoi_pins.py
"""

import json
import os
import wave

import numpy as np

BASE = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
CASES = {
    # stem: (presentation folder, alg, results folder)
    "p257_090": ("lowSTOI_SpectralSubtraction_p257_090", "spectralSubtractor", "29_menschenWM_mitTrueNoise"),
    "p257_135": ("wiener_p257_135", "wiener", "21_kombiWM_ohneTrueNoise"),
}
VARS = {"stoi": "stoi_stoiopt", "pesq": "stoi_pesqopt", "balanced": "stoi_balopt"}


def _read_wav(path):
    with wave.open(path) as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1 and w.getframerate() == 16000
        return np.frombuffer(w.readframes(w.getnframes()), dtype="<i2").copy()


def main():
    out = {}
    for stem, (folder, alg, res) in CASES.items():
        rows = json.load(open(f"{BASE}/Code/results_summary/{res}/all_results.json"))
        row = next(r for r in rows if r["stem"] == stem and r["alg"] == alg)
        out[f"stoi|{stem}|noisy"] = np.float64(row["stoi_noisy"])
        for var, key in VARS.items():
            out[f"enhanced|{stem}|{var}"] = _read_wav(f"{BASE}/Document/Presentation/{folder}/{stem}_{alg}_optimized_{var}.wav")
            out[f"stoi|{stem}|{var}"] = np.float64(row[key])
    np.savez_compressed(os.path.join(OUT, "stoi_pins.npz"), **out)
    print({k: float(v) for k, v in out.items() if k.startswith("stoi|")})


if __name__ == "__main__":
    main()
