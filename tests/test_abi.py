"""C-ABI checks that need no GPU: the library loads, exports every symbol that
include/cse.h declares, and rejects bad arguments with status codes."""

import ctypes
import os
import re

import numpy as np
import pytest

from classical_speech_enhancement_amd import _lib

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "cse.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cse_[a-z0-9_]+)\s*\(", text)) - {"cse_cell"})


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = _declared()
    assert set(names) == set(_lib.EXPORTS)
    for n in names:
        assert hasattr(lib, n), n


def test_version_and_error_channel(lib):
    assert lib.cse_version() == _lib.ABI_VERSION
    rc = lib.cse_stft(None, None, 1, 100, 512, 128, None, None, None)
    assert rc == -1
    assert b"x is NULL" in lib.cse_last_error()
    rc = lib.cse_stft(ctypes.c_void_p(16), None, 1, 100, 501, 128, None, None, None)
    assert rc == -1 and b"n_fft" in lib.cse_last_error()
    rc = lib.cse_stft(ctypes.c_void_p(16), None, 1, 100, 8192, 128, None, None, None)
    assert rc == -1 and b"n_fft" in lib.cse_last_error()
    args = (100, ctypes.c_void_p(16), 1, ctypes.c_void_p(16), ctypes.c_void_p(16), None, None, 0,
            None, None, None, None)
    for bad in (32, 385, 8192):
        rc = lib.cse_enhance_cells_generic(bad, *args)
        assert rc == -1 and b"cse_enhance_cells_generic: n_fft" in lib.cse_last_error()
    rc = lib.cse_enhance_cells(256, 100, ctypes.c_void_p(16), 1, ctypes.c_void_p(16),
                               ctypes.c_void_p(16), None, None, 0, None, None, None, None)
    assert rc == -1 and b"n_fft" in lib.cse_last_error()
    rc = lib.cse_noise_estimate(7, ctypes.c_void_p(16), 1, 100, 257, 20.0, 1e-10,
                                ctypes.c_void_p(16), ctypes.c_void_p(16), None)
    assert rc == -1 and b"Unbekannte Methode" in lib.cse_last_error()
    # n_fft 512 rows are read with 32-bit byte offsets (cse.h): the longest
    # signal is (1 + len/128) * 257 * 8 < 2^31; n_fft 1024 takes up to 2^30
    ok512 = ((2**31 - 1) // (257 * 8) - 1) * 128 + 127
    rc = lib.cse_enhance_cells(512, ok512 + 1, ctypes.c_void_p(16), 0, ctypes.c_void_p(16),
                               ctypes.c_void_p(16), None, None, 0, None, None, None, None)
    assert rc == -1 and b"too long for n_fft=512" in lib.cse_last_error()
    for n_fft, n in ((512, ok512), (1024, ok512 + 1)):  # n_cells = 0: checked, nothing launched
        rc = lib.cse_enhance_cells(n_fft, n, ctypes.c_void_p(16), 0, ctypes.c_void_p(16),
                                   ctypes.c_void_p(16), None, None, 0, None, None, None, None)
        assert rc == 0, lib.cse_last_error()
    # the short hops: rows at hop 32, so (1 + len/32) * 257 * 8 < 2^31 at 512
    ok32 = ((2**31 - 1) // (257 * 8) - 1) * 32 + 31
    args = (ctypes.c_void_p(16), 0, ctypes.c_void_p(16), ctypes.c_void_p(16), None, None, 0,
            None, None, None)
    rc = lib.cse_enhance_cells_short_hop(256, 100, *args)
    assert rc == -1 and b"cse_enhance_cells_short_hop: n_fft" in lib.cse_last_error()
    rc = lib.cse_enhance_cells_short_hop(512, ok32 + 1, *args)
    assert rc == -1 and b"too long for n_fft=512" in lib.cse_last_error()
    for n_fft, n in ((512, ok32), (1024, ok32 + 1)):
        assert lib.cse_enhance_cells_short_hop(n_fft, n, *args) == 0, lib.cse_last_error()


def test_stoi_rates(lib):
    """STOI sizes per input rate: 16 kHz is the plain functions' case, other
    rates in [1 kHz, 768 kHz] add the generic filter (2L + 1 taps) and the
    cells' 10-kHz test signals; unsupported rates report -1 and are refused."""
    n = 48000
    assert lib.cse_stoi_workspace_bytes_sr(2, n, 16000) == lib.cse_stoi_workspace_bytes(2, n)
    assert lib.cse_stoi_scratch_bytes_sr(3, n, 16000) == lib.cse_stoi_scratch_bytes(3, n)
    for sr in (999, 768001, -16000):
        assert lib.cse_stoi_workspace_bytes_sr(1, n, sr) == -1
        assert lib.cse_stoi_scratch_bytes_sr(1, n, sr) == -1
    for sr in (8000, 10000, 22050, 44100, 48000):
        assert lib.cse_stoi_workspace_bytes_sr(1, n, sr) > 0
        # scratch: envelopes + the 10-kHz signal, ceil(n 10000 / sr) doubles per cell
        n10 = -(-n * 10000 // sr)
        assert lib.cse_stoi_scratch_bytes_sr(1, n, sr) >= 8 * n10
    rc = lib.cse_stoi_prepare(ctypes.c_void_p(16), 1, n, 500, ctypes.c_void_p(16), None)
    assert rc == -1 and b"sr=500" in lib.cse_last_error()
    rc = lib.cse_stoi_cells_sr(ctypes.c_void_p(16), ctypes.c_void_p(16), None, ctypes.c_void_p(16),
                               0, 1, n, 900000, 1, ctypes.c_void_p(16), None, ctypes.c_void_p(16),
                               None)
    assert rc == -1 and b"sr=900000" in lib.cse_last_error()


def test_route_classes_pack_in_order():
    """pack_waves puts the short-hop groups after the sweep-hop ones and the
    generic shapes last (each class its own launch: GridPlan.launch),
    whatever their cost; route_slots counts the three parts."""
    from classical_speech_enhancement_amd.engine import (GENERIC, MAIN, SHORT, pack_waves, route,
                                                         route_slots)
    cells = np.zeros(11, dtype=_lib.CELL_DTYPE)
    cells["algo"] = [0, 3, 3, 1, 0, 3, 2, 2, 3, 3, 1]
    cells["hop"] = [32, 256, 64, 128, 128, 32, 256, 64, 128, 160, 512]
    cells["y_offset"] = np.arange(11)
    packed, order = pack_waves(cells, 512)
    G = _lib.cells_per_group(512)
    k_main, k_short, k_gen = route_slots(packed, 512)
    assert k_main == 5 * G  # five sweep-hop cells, each its own group (distinct rows)
    assert (k_short, k_gen) == (4 * G, 2 * G)
    assert set(packed["hop"][:k_main].tolist()) == {128, 256}
    assert set(packed["hop"][k_main:k_main + k_short].tolist()) == {32, 64}
    assert set(packed["hop"][k_main + k_short:].tolist()) == {160, 512}
    assert sorted(order[order >= 0].tolist()) == list(range(11))
    # inside each part: longest first (hop 32 OMLSA leads the short part)
    assert packed[k_main]["hop"] == 32 and packed[k_main]["algo"] == 3
    # other n_fft: every cell generic, one slot each, in the given order
    p2, o2 = pack_waves(cells, 256)
    assert len(p2) == 11 and o2.tolist() == list(range(11))
    assert route_slots(p2, 256) == (0, 0, 11)
    assert route(512, 128) == MAIN and route(1024, 64) == SHORT and route(512, 160) == GENERIC
    assert route(2048, 512) == GENERIC and route(1024, 512) == GENERIC
    assert route(400, 160) == GENERIC and route(500, 100) == GENERIC
    assert route(4096, 1024) == GENERIC
    assert route(401, 100) is None and route(8192, 1024) is None and route(256, 300) is None


def test_cells_per_group_matches_header(lib):
    import re
    text = open(HEADER).read()
    waves = int(re.search(r"#define CSE_WG_WAVES (\d+)", text).group(1))
    assert lib.cse_cells_per_group(512) == _lib.cells_per_group(512) == 4 * waves
    assert lib.cse_cells_per_group(1024) == 2 * waves
    assert lib.cse_cells_per_group(256) == 0


def test_cell_struct_layout():
    assert _lib.CELL_DTYPE.itemsize == 96
    off = {n: _lib.CELL_DTYPE.fields[n][1] for n in _lib.CELL_DTYPE.names}
    assert off == {"algo": 0, "hop": 4, "y_offset": 8, "noise_offset": 16, "noise_stride": 24,
                   "clean_offset": 32, "out_offset": 40, "gain_offset": 48, "lag": 56,
                   "reserved": 60, "param": 64}


def test_workspace_size_is_positive(lib):
    assert lib.cse_noise_workspace_bytes(4, 1251, 257) >= 4 * 1251 * 257 * 8


def test_wave_packing_groups_and_pads():
    from classical_speech_enhancement_amd.engine import pack_waves
    cells = np.zeros(7, dtype=_lib.CELL_DTYPE)
    cells["algo"] = [3, 3, 3, 3, 3, 0, 0]
    cells["hop"] = [128, 128, 256, 128, 128, 128, 128]
    cells["y_offset"] = [0, 0, 5, 0, 0, 0, 0]
    packed, order = pack_waves(cells, 512)
    G = _lib.cells_per_group(512)
    assert len(packed) % G == 0
    assert sorted(order[order >= 0].tolist()) == list(range(7))
    for w in range(len(packed) // G):
        slots = packed[G * w:G * w + G]
        real = slots[slots["algo"] >= 0]
        for f in ("hop", "algo", "y_offset", "noise_offset", "noise_stride", "clean_offset", "lag"):
            assert len(set(slots[f].tolist() if f != "algo" else real[f].tolist())) == 1, f
        assert slots[0]["algo"] >= 0
    # longest first: hop 128 OMLSA before hop 128 SS and hop 256 OMLSA
    assert packed[0]["algo"] == 3 and packed[0]["hop"] == 128


def _pack_waves_loop(cells, n_fft):
    """Straight per-cell restatement of the slot-group packing (the form the
    vectorised engine.pack_waves replaced): groups in (-cost, key) order,
    chunks of CSE_CELLS_PER_GROUP in cell order, padding copies the group's
    first cell with no algorithm and no outputs."""
    from classical_speech_enhancement_amd.engine import ALGO_COST
    per = _lib.cells_per_group(n_fft)
    code_name = {v: k for k, v in _lib.ALGO.items()}
    groups = {}
    for i, c in enumerate(cells):
        key = tuple(int(c[f]) for f in ("hop", "algo", "y_offset", "noise_offset",
                                        "noise_stride", "clean_offset", "lag"))
        groups.setdefault(key, []).append(i)
    slots = []
    for key, idxs in groups.items():
        cost = (1 + 16000 // key[0]) * ALGO_COST[code_name[key[1]]]
        for s in range(0, len(idxs), per):
            chunk = idxs[s:s + per]
            slots.append((-cost, key, chunk + [-1] * (per - len(chunk))))
    slots.sort(key=lambda w: (w[0], w[1]))
    order = np.array([i for w in slots for i in w[2]], dtype=np.int64)
    packed = np.zeros(len(order), dtype=_lib.CELL_DTYPE)
    real = order >= 0
    packed[real] = cells[order[real]]
    for g, (_, key, chunk) in enumerate(slots):
        for s, i in enumerate(chunk):
            if i < 0:
                slot = g * per + s
                packed[slot] = cells[chunk[0]]
                packed[slot]["algo"] = -1
                packed[slot]["out_offset"] = -1
                packed[slot]["gain_offset"] = -1
    return packed, order


@pytest.mark.parametrize("n_fft", [512, 1024])
def test_wave_packing_matches_per_cell_form(n_fft):
    from classical_speech_enhancement_amd.engine import pack_waves
    rng = np.random.default_rng(n_fft)
    n = 3000
    cells = np.zeros(n, dtype=_lib.CELL_DTYPE)
    cells["algo"] = rng.integers(0, 4, n)
    cells["hop"] = rng.choice([128, 256], n)
    cells["y_offset"] = rng.integers(0, 5, n) * 1000
    cells["noise_offset"] = rng.integers(0, 7, n) * 100
    cells["noise_stride"] = rng.choice([0, 257], n)
    cells["clean_offset"] = rng.integers(0, 3, n) * 10
    cells["lag"] = rng.choice([0, 0, 0, 5, -7], n)
    cells["out_offset"] = np.arange(n) * 3
    cells["gain_offset"] = np.arange(n) * 11
    cells["param"] = rng.random((n, 8)).astype(np.float32)
    got, go = pack_waves(cells, n_fft)
    ref, ro = _pack_waves_loop(cells, n_fft)
    assert np.array_equal(go, ro)
    assert got.tobytes() == ref.tobytes()
