"""CPU oracle for the STFT frame-gain path — TEST INFRASTRUCTURE ONLY.

This package is a float64 numpy restatement of the reference's hot path
(Katja39/Classical_Speech_Enhancement, ``Code/*.py``) plus the librosa-0.11
STFT/ISTFT semantics it relies on.  It exists to CHECK the HIP engine in
``classical_speech_enhancement_amd`` and to time a CPU baseline; it is never
part of the product path.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.

Pinning status:
  * algorithm / estimator / grid code: pinned against golden vectors produced by
    importing the unmodified reference modules in the dev container
    (``tests/golden/make_golden.py``) — fp64, ≤1e-12.
  * librosa 0.11 ``stft``/``istft``/``fix_length``: the library is absent from
    the image, so these are restated from its published algorithm; they are
    pinned only loosely by the reference's committed Presentation WAVs
    (≈1e-2 rel-L2, limited by resampler substitution + PCM16).
"""

from .stft_ref import stft, istft, fix_length, hann_periodic, n_frames_for
from .noise_ref import (noise_estimation, percentile_noise, min_tracking_noise,
                        true_noise, simple_noise)
from .gain_ref import (spectral_subtraction, wiener_filter, mmse, advanced_mmse,
                       ALGORITHMS)
from .pipeline_ref import (GRIDS, grid_cells, finalize_enhanced, calculate_snr,
                           align_to_reference, align_lag, match_length, to_mono,
                           combined_score, tolerance_scan)

__all__ = [
    "stft", "istft", "fix_length", "hann_periodic", "n_frames_for", "align_lag",
    "noise_estimation", "percentile_noise", "min_tracking_noise", "true_noise",
    "simple_noise", "spectral_subtraction", "wiener_filter", "mmse",
    "advanced_mmse", "ALGORITHMS", "GRIDS", "grid_cells", "finalize_enhanced",
    "calculate_snr", "align_to_reference", "match_length", "to_mono",
    "combined_score", "tolerance_scan",
]
