"""Static instruction mix per frame-loop stage of enhance_kernel<512,false>.

Compiles cse_enhance.hip with -DCSE_MARKS (asm comment markers between the
stages), extracts the kernel's ISA and counts instructions between markers,
per (hop, algorithm) specialisation, by class.  Analysis only.

    python tools/isa_sections.py [kernel-substring [source]]
"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SRC = os.path.join(REPO, "classical_speech_enhancement_amd", "csrc", "cse_enhance.hip")
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def classify(op):
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op == "s_nop":
        return "nop"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(kname="enhance_kernelILi512ELb0E", src=SRC, extra=()):
    out = "/tmp/cse_marks.s"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(REPO, "include"),
                    "-I" + os.path.join(REPO, "classical_speech_enhancement_amd", "csrc"),
                    "-DCSE_MARKS", "-fno-slp-vectorize", "-S", "--cuda-device-only", src, "-o", out, *extra], check=True)
    lines = open(out).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith("_ZN3cse14" + kname.split("14", 1)[-1])
                 or (kname in l and l.endswith(":") is False and l.startswith("_Z") and ":" in l))
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        body.append(l)
    sections = []
    cur, counts = "prologue", collections.Counter()
    for l in body:
        m = re.search(r";#MARK (\w+)", l)
        if m:
            sections.append((cur, counts))
            cur, counts = m.group(1), collections.Counter()
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        counts[classify(t.split()[0])] += 1
    sections.append((cur, counts))
    cols = ["valu", "valu_pk", "trans", "lds", "vmem", "salu", "nop", "wait"]
    print(f"{'section':10s} " + " ".join(f"{c:>7s}" for c in cols))
    for name, c in sections:
        if sum(c.values()) == 0:
            continue
        print(f"{name:10s} " + " ".join(f"{c[k]:7d}" for k in cols))


if __name__ == "__main__":
    main(*(sys.argv[1:3] or []))
