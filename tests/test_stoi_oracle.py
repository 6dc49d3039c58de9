"""Pin the STOI oracle (pystoi 0.4.1 restatement) against the reference's own
recorded STOI values (no GPU).

pystoi is absent from the image, so the pin is the reference's output:
all_results.json rows for the two stems whose WAVs are committed
(tests/golden/make_stoi_pins.py).  The 16-kHz clean/noisy inputs pass through
a resampler stand-in and the enhanced WAVs are PCM16, so the tolerance is
5e-5 absolute STOI (observed: ≤ 1.9e-5).
"""

import numpy as np
import pytest

from oracle import stoi_ref
from conftest import load_golden

STEMS = ("p257_090", "p257_135")
PIN_TOL = 5e-5


@pytest.fixture(scope="module")
def pins():
    return load_golden("stoi_pins.npz"), load_golden("presentation_wavs.npz")


@pytest.mark.parametrize("stem", STEMS)
@pytest.mark.parametrize("var", ["noisy", "stoi", "pesq", "balanced"])
def test_stoi_matches_reference_results(pins, stem, var):
    p, w = pins
    clean = w[f"clean|{stem}"].astype(np.float64)
    if var == "noisy":
        test = w[f"noisy|{stem}"].astype(np.float64)
    else:
        test = p[f"enhanced|{stem}|{var}"].astype(np.float64) / 32768.0
    got = stoi_ref.calculate_stoi(clean, test, 16000)
    want = float(p[f"stoi|{stem}|{var}"])
    assert abs(got - want) < PIN_TOL, (got, want)


def test_thirdoct_bands():
    """Band edges of the 15 one-third-octave bands at 10 kHz / 512 points."""
    edges = stoi_ref.band_edges()
    assert len(edges) == 15
    assert edges[0] == (7, 9) and edges[-1][1] == 219
    for (a, b), (c, d) in zip(edges, edges[1:]):
        assert b == c  # contiguous


def test_resample_oct_filter():
    h = stoi_ref.resample_window_oct(10000, 16000)
    assert h.size == 581 and abs(h.sum() / 5 - 1.0) < 0.05


def test_short_signal_returns_floor():
    rng = np.random.default_rng(0)
    x = rng.standard_normal(3000)
    assert stoi_ref.stoi(x, x, 16000) == 1e-5


def test_identity_is_one():
    from classical_speech_enhancement_amd.synth import make_pair
    clean, _ = make_pair(3, seconds=1.5)
    assert abs(stoi_ref.stoi(clean, clean, 16000) - 1.0) < 1e-12


def test_no_frame_is_failure():
    """Fewer than 256 samples at 10 kHz: pystoi raises, calculate_stoi -> None."""
    x = np.ones(300)
    with pytest.raises(ValueError):
        stoi_ref.stoi(x, x, 16000)
    assert stoi_ref.calculate_stoi(x, x, 16000) is None
