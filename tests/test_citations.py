"""Citation hygiene (CPU): every `<reference file>.py:N[-M]` the package, the
oracle, the header, the bench, the tools, the tests and the documents
(README.md) cite points inside that reference file,
and so does every bare `:N[-M]` a document or comment attributes to the file
it last named in the same paragraph.  Where a citation sits next to the name
of a reference function and starts within a few lines of that function's
`def`, it must start exactly there (and end at the function's last line when
it ends near it): r05's `main` (`:378-474` for 375-473) and PESQ-skip
(`:182-183` for 180-181) drifts are of that kind.

The line counts and function spans are those of the reference's Code/ files
(the last line counted also where the file has no final newline)
(Katja39/Classical_Speech_Enhancement HEAD), recorded here so the
test needs no copy of the reference.  A bare citation in a list that names
another file in between is written with its file (`X.py:N`): the attribution
is by the last file named before it.
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

# (def line, last line) of the reference's functions and classes
REFERENCE_SPANS = {
    "advanced_mmse.py": {"advanced_mmse": (7, 136)},
    "evaluation_metrics.py": {"calculate_pesq": (9, 27), "calculate_stoi": (30, 36),
                              "calculate_snr": (39, 58), "evaluate_audio_quality": (61, 101),
                              "calculate_combined_speech_score": (104, 115)},
    "mmse.py": {"mmse": (6, 120)},
    "noise_estimation.py": {"NoiseEstimator": (6, 9), "PercentileNoiseEstimator": (11, 56),
                            "MinTrackingNoiseEstimator": (59, 107), "TrueNoiseEstimator": (109, 155),
                            "noise_estimation": (158, 212), "_create_estimator": (215, 223),
                            "_simple_noise_estimate": (226, 232), "_get_window_size": (97, 99),
                            "_sliding_minimum": (101, 107)},
    "spectral_subtractor.py": {"spectral_subtraction": (6, 65)},
    "speech_enhancement_comparison.py": {
        "to_mono": (14, 21), "resample_to": (23, 27), "match_length": (29, 36),
        "align_to_reference": (38, 69), "prepare_pair": (71, 90), "finalize_enhanced": (92, 106),
        "optimize_parameters": (109, 252), "_find_pairs": (254, 267), "_ensure_dir": (269, 271),
        "_fmt": (273, 276), "run_algorithm_on_pair": (278, 338),
        "_compute_and_save_summary": (341, 373), "main": (375, 473),
        "algorithm_wrapper": (282, 292), "get_processed_stems": (406, 414)},
    "wiener_filter.py": {"wiener_filter": (7, 95)},
}

CITE = re.compile(r"\b([A-Za-z_]+\.py):(\d+)(?:-(\d+))?")
# a bare `:N[-M]` (not part of file.py:N, a time, a ratio or a path)
BARE = re.compile(r"(?<![\w.:/])`?:(\d+)(?:-(\d+))?`?(?![\w:.]\d)")
NAMED = re.compile(r"\b([A-Za-z_]+\.py)\b")
NEAR = 3        # lines: a citation this close to a whole function must match its span
NAME_WINDOW = 60  # characters before a citation searched for a function name

DOCS = ["DESIGN.md", "INTEGRATION.md", "README.md"]


def _sources():
    pats = ["classical_speech_enhancement_amd/*.py", "classical_speech_enhancement_amd/csrc/*",
            "include/*.h", "oracle/*.py", "bench.py", "__graft_entry__.py", "tools/*.py",
            "tests/*.py"] + DOCS
    for p in pats:
        for path in sorted(glob.glob(os.path.join(REPO, p))):
            if os.path.basename(path) != "test_citations.py":
                yield path


def _paragraphs(text):
    """(offset, paragraph) pieces split at blank lines."""
    pos = 0
    for piece in re.split(r"(\n\s*\n)", text):
        yield pos, piece
        pos += len(piece)


def citations(text):
    """(file, lo, hi, start offset, explicit) for every explicit citation and
    every bare one attributed to the file last named in its paragraph."""
    out = []
    for base, para in _paragraphs(text):
        spans = []
        for m in CITE.finditer(para):
            if m.group(1) in REFERENCE_LINES:
                lo = int(m.group(2))
                out.append((m.group(1), lo, int(m.group(3)) if m.group(3) else lo, base + m.start(), True))
            spans.append((m.start(), m.end()))
        names = [(m.start(), m.group(1)) for m in NAMED.finditer(para)]
        for m in BARE.finditer(para):
            if any(a <= m.start() < b for a, b in spans):
                continue
            prev = [n for s, n in names if s < m.start()]
            if not prev or prev[-1] not in REFERENCE_LINES:
                continue
            lo = int(m.group(1))
            out.append((prev[-1], lo, int(m.group(2)) if m.group(2) else lo, base + m.start(), False))
    return out


def _scan():
    bad, seen, bare = [], 0, 0
    for path in _sources():
        text = open(path, encoding="utf-8").read()
        rel = os.path.relpath(path, REPO)
        for name, lo, hi, at, explicit in citations(text):
            seen += 1
            bare += not explicit
            n = REFERENCE_LINES[name]
            line = text.count("\n", 0, at) + 1
            if not (1 <= lo <= hi <= n):
                bad.append(f"{rel}:{line}: {name}:{lo}-{hi} outside the file ({n} lines)")
                continue
            before = text[max(0, at - NAME_WINDOW):at]
            for fn, (d0, d1) in REFERENCE_SPANS.get(name, {}).items():
                if not re.search(r"(?<![\w.])`?" + re.escape(fn) + r"\b", before):
                    continue
                # a citation of the whole function (both ends within NEAR lines
                # of its span) must be the span itself
                if abs(lo - d0) <= NEAR and abs(hi - d1) <= NEAR and (lo, hi) != (d0, d1):
                    bad.append(f"{rel}:{line}: {name}:{lo}-{hi} next to `{fn}` ({d0}-{d1})")
    return bad, seen, bare


def test_reference_citations_point_inside_the_files():
    bad, seen, bare = _scan()
    assert seen > 250 and bare > 50, (seen, bare)
    assert not bad, "\n".join(bad)


def test_bare_citations_are_attributed():
    text = ("The sweep (`speech_enhancement_comparison.py:109-252`) skips a cell whose\n"
            "PESQ is None (`:180-181`); `main` (`:375-473`) loops.\n\n"
            "A new paragraph: `:12` has no file and is not attributed.")
    got = [(n, lo, hi, e) for n, lo, hi, _, e in citations(text)]
    assert got == [("speech_enhancement_comparison.py", 109, 252, True),
                   ("speech_enhancement_comparison.py", 180, 181, False),
                   ("speech_enhancement_comparison.py", 375, 473, False)]


def test_r05_drift_fixed():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    assert "`speech_enhancement_comparison.py:180-181`" in text and "(`main`, `:375-473`)" in text
    assert ":182-183" not in text and ":378-474" not in text
    search = open(os.path.join(REPO, "classical_speech_enhancement_amd", "search.py")).read()
    assert "raises ValueError like :233-235" in search
    assert "speech_enhancement_comparison.py:375-473" in search
    assert "run_algorithm_on_pair :278-294 and main :440-455" in search
    assert "_fmt :273-276" in open(os.path.join(REPO, "classical_speech_enhancement_amd", "results.py")).read()
