"""The HEAD parameter grids (Code/parameter_ranges.py:2-40), restated as data.

Key order is the enumeration order of speech_enhancement_comparison.py:149-151
(itertools.product over the values, last key varying fastest).  The method
options hinted at parameter_ranges.py:1 are "true_noise", "percentile",
"min_tracking"; the HEAD grid sweeps the last two.
"""

import itertools

param_ranges_ss = {
    "alpha": [0.5, 0.8, 1.0, 1.5, 2.0, 2.5, 3.0, 4.0, 5.0],
    "beta": [0.001, 0.005, 0.05, 0.1, 0.15],
    "n_fft": [512, 1024],
    "hop_length": [128, 256],
    "noise_percentile": [10.0, 20.0],
    "noise_method": ["percentile", "min_tracking"],
}

param_ranges_mmse = {
    "alpha": [0.90, 0.95, 0.98, 0.99],
    "ksi_min": [0.0001, 0.001, 0.01, 0.05, 0.1, 0.15],
    "gain_min": [0.001, 0.01, 0.05, 0.1, 0.2],
    "gain_max": [1.0],
    "n_fft": [512, 1024],
    "hop_length": [128, 256],
    "noise_percentile": [10.0, 20.0],
    "noise_method": ["percentile", "min_tracking"],
}

param_ranges_wiener = {
    "alpha": [0.90, 0.95, 0.98],
    "gain_floor": [0.01, 0.02, 0.05, 0.1],
    "n_fft": [512, 1024],
    "hop_length": [128, 256],
    "noise_percentile": [10.0, 20.0],
    "noise_method": ["percentile", "min_tracking"],
}

param_ranges_omlsa = {
    "alpha": [0.7, 0.80, 0.9, 0.95],
    "ksi_min": [0.001, 0.005, 0.01, 0.05],
    "gain_floor": [0.05, 0.1, 0.2],
    "noise_mu": [0.92, 0.95, 0.98],
    "q": [0.3, 0.4, 0.5],
    "n_fft": [512, 1024],
    "hop_length": [128, 256],
    "noise_percentile": [10.0, 20.0],
    "noise_method": ["percentile", "min_tracking"],
}

# registry order of speech_enhancement_comparison.py:395-401
ALGORITHM_GRIDS = {
    "spectralSubtractor": param_ranges_ss,
    "mmse": param_ranges_mmse,
    "wiener": param_ranges_wiener,
    "omlsa": param_ranges_omlsa,
}


def grid_cells(ranges):
    """Param dicts in the reference's enumeration order."""
    names = list(ranges)
    return [dict(zip(names, combo)) for combo in itertools.product(*ranges.values())]


def grid_specs(n_signals, n_fft=None, algorithms=None, grids=None):
    """(signal, algorithm, params) for every signal x algorithm x grid cell
    (optionally only one n_fft), signals outermost like the reference's pair loop."""
    grids = grids or ALGORITHM_GRIDS
    algorithms = algorithms or list(grids)
    out = []
    for sig in range(n_signals):
        for alg in algorithms:
            for p in grid_cells(grids[alg]):
                if n_fft is None or p["n_fft"] == n_fft:
                    out.append((sig, alg, p))
    return out
