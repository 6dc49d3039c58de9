"""Sample the GPU's shader clock while a command runs (analysis only).

    python tools/clock_trace.py OUT.json -- python3 tools/bench_sweep.py --pairs 20 --reps 1

The command runs as a child process (nothing is exec'd from this process,
which never touches the GPU); every ~50 ms the current SCLK level is read
from sysfs (pp_dpm_sclk, the line marked '*') or, failing that, from
`rocm-smi --showclocks`.  Writes the samples (seconds since start, MHz) and
their summary; the command's own stdout/stderr pass through.
"""
import glob
import json
import re
import subprocess
import sys
import time


def read_sysfs():
    vals = []
    for f in sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk")):
        try:
            for line in open(f):
                if "*" in line:
                    m = re.search(r"(\d+)\s*[Mm][Hh]z", line)
                    if m:
                        vals.append(int(m.group(1)))
        except OSError:
            pass
    return max(vals) if vals else None


def read_smi():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True, timeout=5).stdout
    except Exception:
        return None
    m = re.findall(r"sclk.*?\((\d+)\s*Mhz\)", out, flags=re.I)
    return max(int(x) for x in m) if m else None


def main():
    if "--" not in sys.argv:
        raise SystemExit(__doc__)
    k = sys.argv.index("--")
    out, cmd = sys.argv[1], sys.argv[k + 1:]
    reader = read_sysfs if read_sysfs() is not None else read_smi
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd)
    samples = []
    while p.poll() is None:
        v = reader()
        if v is not None:
            samples.append((round(time.perf_counter() - t0, 3), v))
        time.sleep(0.05)
    mhz = [v for _, v in samples]
    res = {"command": cmd, "reader": reader.__name__, "rc": p.returncode, "samples": samples,
           "summary": {"n": len(mhz), "min_mhz": min(mhz) if mhz else None,
                       "max_mhz": max(mhz) if mhz else None,
                       "mean_mhz": sum(mhz) / len(mhz) if mhz else None}}
    json.dump(res, open(out, "w"))
    print("clock_trace", json.dumps(res["summary"]))
    sys.exit(p.returncode)


if __name__ == "__main__":
    main()
