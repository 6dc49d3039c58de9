"""Citation hygiene (CPU): every `<reference file>.py:N[-M]` the package, the
oracle, the header and the bench cite points inside that reference file.

The line counts are those of the reference's Code/ files (the last line
counted also where the file has no final newline) (Katja39/
Classical_Speech_Enhancement HEAD), recorded here so the test
needs no copy of the reference.
"""

import glob
import os
import re

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

REFERENCE_LINES = {
    "advanced_mmse.py": 136,
    "debug_noise_analysis.py": 159,
    "evaluation_metrics.py": 115,
    "load_files.py": 22,
    "mmse.py": 120,
    "noise_estimation.py": 232,
    "parameter_ranges.py": 41,
    "spectral_subtractor.py": 65,
    "speech_enhancement_comparison.py": 477,
    "wiener_filter.py": 95,
}

CITE = re.compile(r"\b([A-Za-z_]+\.py):(\d+)(?:-(\d+))?")


def _sources():
    pats = ["classical_speech_enhancement_amd/*.py", "classical_speech_enhancement_amd/csrc/*",
            "include/*.h", "oracle/*.py", "bench.py", "__graft_entry__.py"]
    for p in pats:
        yield from sorted(glob.glob(os.path.join(REPO, p)))


def test_reference_citations_point_inside_the_files():
    bad, seen = [], 0
    for path in _sources():
        text = open(path, encoding="utf-8").read()
        for m in CITE.finditer(text):
            name = m.group(1)
            if name not in REFERENCE_LINES:
                continue
            seen += 1
            lo = int(m.group(2))
            hi = int(m.group(3)) if m.group(3) else lo
            n = REFERENCE_LINES[name]
            if not (1 <= lo <= hi <= n):
                bad.append(f"{os.path.relpath(path, REPO)}: {m.group(0)} (file has {n} lines)")
    assert seen > 50
    assert not bad, "\n".join(bad)


def test_search_citations_fixed_in_r05():
    text = open(os.path.join(REPO, "classical_speech_enhancement_amd", "search.py")).read()
    assert "raises ValueError like :233-235" in text
    assert "speech_enhancement_comparison.py:375-473" in text
