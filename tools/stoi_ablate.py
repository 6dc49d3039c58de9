"""Timing-only ablation builds of the STOI cell kernel (never product code).

Writes a patched copy of csrc/cse_stoi.hip to a temporary directory with one
stage of stoi_cells_kernel switched off, and builds a libcse variant from it
(the other sources unchanged), for A/B timing with tools/ab_stoi.sh:

    python tools/stoi_ablate.py MASK [out.so]      MASK: sum of the bits below
      1  resampling arithmetic          2  rfft of the frames
      4  band sums                      8  phase B (segment correlations)
      16 16-kHz input loads (zeros staged)
      64 occupancy probe: 2 instead of 3 workgroups per CU (extra unused LDS)

The outputs of such a build are wrong by construction (tools/ab_stoi.sh runs
tools/bench_stoi.py with CSE_BENCH_NOCHECK=1).  DESIGN.md §3.5 records the
measured breakdown.
"""
import os
import shutil
import sys
import tempfile

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, REPO)

# (bit, anchor in the product source, replacement)
PATCHES = [
    (1, "if (tid < ns * GRP) {", "if (false) {"),
    (2, "        // ---- 512-point rfft of frame fl, 16 lanes per frame",
        "        if (false)\n        // ---- 512-point rfft of frame fl, 16 lanes per frame"),
    (4, "if (n1 < NBAND && fl < nf) {", "if (false) {"),
    (8, "for (int j0 = 0; j0 < J; j0 += 64) {", "for (int j0 = 0; j0 < 0; j0 += 64) {"),
    (16, "float v = (unsigned)(fbase + FW * u) < (unsigned)cnt ? pre[u] : 0.0f;", "float v = 0.0f;"),
    # occupancy probe (not a stage): 14 KiB of unused dynamic LDS per workgroup,
    # 3 -> 2 workgroups per CU
    (64, "dim3((unsigned)n_cells), dim3(stoi::NT), 0,", "dim3((unsigned)n_cells), dim3(stoi::NT), 14336,"),
]


def main(mask, out=None):
    import __graft_entry__ as g
    mask = int(mask)
    out = out or os.path.join(g.PKG, f"libcse_ab{mask}.so")
    src = open(os.path.join(g.CSRC, "cse_stoi.hip")).read()
    for bit, old, new in PATCHES:
        if mask & bit:
            if src.count(old) != 1:
                raise SystemExit(f"anchor for bit {bit} not found exactly once: {old!r}")
            src = src.replace(old, new)
    # a sibling of csrc/, so the sources' relative include of ../../include resolves
    tmp = tempfile.mkdtemp(prefix="cse_ablate_", dir=g.PKG)
    try:
        for f in os.listdir(g.CSRC):
            shutil.copy(os.path.join(g.CSRC, f), tmp)
        open(os.path.join(tmp, "cse_stoi.hip"), "w").write(src)
        csrc = g.CSRC
        g.CSRC = tmp
        try:
            g.build(out=out)
        finally:
            g.CSRC = csrc
    finally:
        shutil.rmtree(tmp)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:3])
