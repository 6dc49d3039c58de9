"""Build a libcse variant from patched copies of the sources (experiments only).

    python tools/variant_build.py OUT.so FILE 'old' 'new' [FILE 'old' 'new' ...]

Each (FILE, old, new) replaces the one occurrence of ``old`` in csrc/FILE; the
patched tree lives in a scratch directory next to csrc/ and is removed after
the build.  The product sources are never touched.
"""
import os
import shutil
import sys
import tempfile

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, REPO)


def main(out, *edits):
    import __graft_entry__ as g
    if len(edits) % 3:
        raise SystemExit("edits come in (file, old, new) triples")
    tmp = tempfile.mkdtemp(prefix="cse_variant_", dir=g.PKG)
    try:
        for f in os.listdir(g.CSRC):
            shutil.copy(os.path.join(g.CSRC, f), tmp)
        for i in range(0, len(edits), 3):
            f, old, new = edits[i:i + 3]
            p = os.path.join(tmp, f)
            src = open(p).read()
            if src.count(old) != 1:
                raise SystemExit(f"{f}: anchor not found exactly once: {old!r}")
            open(p, "w").write(src.replace(old, new))
        csrc, g.CSRC = g.CSRC, tmp
        try:
            g.build(out=os.path.join(g.PKG, out))
        finally:
            g.CSRC = csrc
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main(*sys.argv[1:])
