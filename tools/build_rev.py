"""Build libcse.so from the sources of a git revision (A/B baselines).

    python tools/build_rev.py REV OUT.so

Exports classical_speech_enhancement_amd/csrc and include/ at REV into a
scratch directory and compiles them with this tree's build recipe
(__graft_entry__.build: same flags and per-file flags).  Experiments only.
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, REPO)


def main(rev, out):
    import __graft_entry__ as g
    tmp = tempfile.mkdtemp(prefix="cse_rev_")
    try:
        for d in ("classical_speech_enhancement_amd/csrc", "include"):
            os.makedirs(os.path.join(tmp, d), exist_ok=True)
            names = subprocess.run(["git", "ls-tree", "--name-only", rev, d + "/"], cwd=REPO,
                                   check=True, capture_output=True, text=True).stdout.split()
            for n in names:
                blob = subprocess.run(["git", "show", f"{rev}:{n}"], cwd=REPO, check=True,
                                      capture_output=True).stdout
                open(os.path.join(tmp, n), "wb").write(blob)
        csrc, pkg = g.CSRC, g.PKG
        g.CSRC = os.path.join(tmp, "classical_speech_enhancement_amd", "csrc")
        old_repo = g.REPO
        g.REPO = tmp
        try:
            g.build(out=os.path.abspath(out))
        finally:
            g.CSRC, g.REPO, g.PKG = csrc, old_repo, pkg
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
