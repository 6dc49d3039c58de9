"""ctypes binding of libcse.so (the C ABI declared in include/cse.h).

The product path has no CPU fallback: if the shared library (built for gfx950
by ``__graft_entry__.build()``) is missing, every entry point raises.
"""

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CSE_LIB", os.path.join(HERE, "libcse.so"))

CSE_OK = 0
# ABI revision this package mirrors (cse_version(); CELL_DTYPE == cse_cell_t,
# NOISE_JOB_DTYPE == cse_noise_job_t, NoiseParams == cse_noise_params_t)
ABI_VERSION = 5
ALGO = {"NONE": -1, "SS": 0, "WIENER": 1, "MMSE": 2, "OMLSA": 3}
NOISE = {"percentile": 0, "min_tracking": 1, "true_noise": 2}

# numpy mirror of cse_cell_t (include/cse.h) — 96 bytes
CELL_DTYPE = np.dtype([
    ("algo", np.int32), ("hop", np.int32), ("y_offset", np.int64),
    ("noise_offset", np.int64), ("noise_stride", np.int64), ("clean_offset", np.int64),
    ("out_offset", np.int64), ("gain_offset", np.int64), ("lag", np.int32),
    ("reserved", np.int32), ("param", np.float32, (8,)),
], align=True)
assert CELL_DTYPE.itemsize == 96

# numpy mirror of cse_noise_job_t — 40 bytes
NOISE_JOB_DTYPE = np.dtype([
    ("src_offset", np.int64), ("dst_offset", np.int64), ("src_frames", np.int32),
    ("out_frames", np.int32), ("mu", np.float64), ("inv_eps", np.float64)], align=True)
assert NOISE_JOB_DTYPE.itemsize == 40


class NoiseParams(ctypes.Structure):
    """cse_noise_params_t: estimator constructor parameters
    (noise_estimation.py:12-13, :60) and the TrueNoise frame fit (:149-153)."""
    _fields_ = [("percentile", ctypes.c_double), ("max_fraction", ctypes.c_double),
                ("floor_rel", ctypes.c_double), ("smoothing_factor", ctypes.c_double),
                ("min_frames", ctypes.c_int32), ("adaptive_short", ctypes.c_int32),
                ("window_size", ctypes.c_int32), ("src_frames", ctypes.c_int32)]


assert ctypes.sizeof(NoiseParams) == 48

EXPORTS = ("cse_version", "cse_last_error", "cse_cells_per_group", "cse_stft",
           "cse_noise_workspace_bytes", "cse_noise_default_params", "cse_noise_estimate_ex",
           "cse_noise_estimate", "cse_noise_smooth", "cse_noise_median",
           "cse_noise_percentile_med", "cse_noise_percentile_med2", "cse_noise_percentile_quad", "cse_noise_min_tracking_med", "cse_noise_finish",
           "cse_noise_invert", "cse_istft_norm", "cse_enhance_cells", "cse_enhance_cells_short_hop",
           "cse_enhance_cells_generic",
           "cse_xcorr_workspace_bytes", "cse_xcorr_prepare", "cse_xcorr_lag",
           "cse_stoi_workspace_bytes", "cse_stoi_scratch_bytes", "cse_stoi_prepare",
           "cse_stoi_cells", "cse_stoi_workspace_bytes_sr", "cse_stoi_scratch_bytes_sr",
           "cse_stoi_cells_sr")
XCORR_OK, XCORR_FLAT, XCORR_NONFINITE = 0, 1, 2  # FLAT: slow exact path ran (lag exact)


def cells_per_group(n_fft):
    """Cells per workgroup slot group (CSE_CELLS_PER_GROUP of the loaded build)."""
    n = int(load().cse_cells_per_group(int(n_fft)))
    if n <= 0:
        raise CseError(f"n_fft={n_fft} not supported")
    return n


class CseError(RuntimeError):
    pass


_lib = None


def load(path=LIB_PATH):
    """Load libcse.so and declare prototypes (raises if it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise CseError(f"{path} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    i32, i64, f64 = ctypes.c_int, ctypes.c_int64, ctypes.c_double
    lib.cse_version.restype = i32
    lib.cse_version.argtypes = []
    lib.cse_last_error.restype = ctypes.c_char_p
    lib.cse_last_error.argtypes = []
    lib.cse_cells_per_group.restype = i32
    lib.cse_cells_per_group.argtypes = [i32]
    lib.cse_stft.restype = i32
    lib.cse_stft.argtypes = [P, P, i64, i64, i32, i32, P, P, P]
    lib.cse_noise_workspace_bytes.restype = i64
    lib.cse_noise_workspace_bytes.argtypes = [i64, i32, i32]
    lib.cse_noise_default_params.restype = None
    lib.cse_noise_default_params.argtypes = [P]
    lib.cse_noise_estimate_ex.restype = i32
    lib.cse_noise_estimate_ex.argtypes = [i32, P, i64, i32, i32, P, f64, P, P, P]
    lib.cse_noise_estimate.restype = i32
    lib.cse_noise_estimate.argtypes = [i32, P, i64, i32, i32, f64, f64, P, P, P]
    lib.cse_noise_smooth.restype = i32
    lib.cse_noise_smooth.argtypes = [P, i64, i32, i32, i32, f64, P, P]
    lib.cse_noise_median.restype = i32
    lib.cse_noise_median.argtypes = [P, i64, i32, i32, P, P]
    lib.cse_noise_percentile_med.restype = i32
    lib.cse_noise_percentile_med.argtypes = [P, P, i64, i32, i32, f64, f64, P, P, P]
    lib.cse_noise_percentile_med2.restype = i32
    lib.cse_noise_percentile_med2.argtypes = [P, P, i64, i32, i32, f64, f64, f64, P, P, P, P]
    lib.cse_noise_percentile_quad.restype = i32
    lib.cse_noise_percentile_quad.argtypes = [P, P, i64, i32, i32, f64, f64, f64, f64, P, P, P, P, P,
                                              P]
    lib.cse_noise_min_tracking_med.restype = i32
    lib.cse_noise_min_tracking_med.argtypes = [P, P, i64, i32, i32, f64, P, f64, P, P, P]
    lib.cse_noise_finish.restype = i32
    lib.cse_noise_finish.argtypes = [P, i32, i64, i32, P, P, P]
    lib.cse_noise_invert.restype = i32
    lib.cse_noise_invert.argtypes = [P, i64, f64, P, P]
    lib.cse_istft_norm.restype = i32
    lib.cse_istft_norm.argtypes = [i32, i32, i64, P, P]
    lib.cse_xcorr_workspace_bytes.restype = i64
    lib.cse_xcorr_workspace_bytes.argtypes = [i64, i64, i32, i32]
    lib.cse_xcorr_prepare.restype = i32
    lib.cse_xcorr_prepare.argtypes = [P, i64, i64, i32, i32, P, P]
    lib.cse_xcorr_lag.restype = i32
    lib.cse_xcorr_lag.argtypes = [P, P, P, i64, i64, i32, i32, P, P, P, P, P, P]
    lib.cse_stoi_workspace_bytes.restype = i64
    lib.cse_stoi_workspace_bytes.argtypes = [i64, i64]
    lib.cse_stoi_scratch_bytes.restype = i64
    lib.cse_stoi_scratch_bytes.argtypes = [i64, i64]
    lib.cse_stoi_prepare.restype = i32
    lib.cse_stoi_prepare.argtypes = [P, i64, i64, i32, P, P]
    lib.cse_stoi_cells.restype = i32
    lib.cse_stoi_cells.argtypes = [P, P, P, P, i64, i64, i64, i32, P, P, P, P]
    lib.cse_stoi_workspace_bytes_sr.restype = i64
    lib.cse_stoi_workspace_bytes_sr.argtypes = [i64, i64, i32]
    lib.cse_stoi_scratch_bytes_sr.restype = i64
    lib.cse_stoi_scratch_bytes_sr.argtypes = [i64, i64, i32]
    lib.cse_stoi_cells_sr.restype = i32
    lib.cse_stoi_cells_sr.argtypes = [P, P, P, P, i64, i64, i64, i32, i32, P, P, P, P]
    lib.cse_enhance_cells.restype = i32
    lib.cse_enhance_cells.argtypes = [i32, i64, P, i64, P, P, P, P, i64, P, P, P, P]
    lib.cse_enhance_cells_short_hop.restype = i32
    lib.cse_enhance_cells_short_hop.argtypes = [i32, i64, P, i64, P, P, P, P, i64, P, P, P]
    lib.cse_enhance_cells_generic.restype = i32
    lib.cse_enhance_cells_generic.argtypes = [i32, i64, P, i64, P, P, P, P, i64, P, P, P, P]
    # the kernels read the cell/job tables laid out as this package packs them:
    # refuse a library of another ABI revision.  The packer (engine.pack_waves)
    # takes the slot-group size from the library itself; it must be usable.
    ver = lib.cse_version()
    if ver != ABI_VERSION:
        raise CseError(f"{path}: ABI version {ver}, this package mirrors {ABI_VERSION} (rebuild)")
    for n_fft in (512, 1024):
        per = lib.cse_cells_per_group(n_fft)
        if per <= 0 or per % 2:
            raise CseError(f"{path}: {per} cells per slot group at n_fft={n_fft}")
    _lib = lib
    return lib


def check(rc, what):
    if rc != CSE_OK:
        msg = load().cse_last_error().decode(errors="replace")
        raise CseError(f"{what} failed ({rc}): {msg}")
