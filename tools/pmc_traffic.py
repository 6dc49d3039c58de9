"""Write profiles/pmc_traffic.json from a tools/profile.sh run (FETCH_SIZE and
WRITE_SIZE collected in separate rocprofv3 --pmc passes).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide streaming reads -> x2; both counters are in KiB -> x1024.

    python tools/pmc_traffic.py TAG UNITS_PER_LAUNCH [ROUND]
"""
import csv
import glob
import json
import sys


def main(tag, units, rnd="r01"):
    pmc = {}
    for f in glob.glob(f"gpurun_out/prof_{tag}/pmc_*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "enhance_kernel" in r["Kernel_Name"]:
                pmc[r["Counter_Name"]] = pmc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    fetch_kb, write_kb = pmc["FETCH_SIZE"], pmc["WRITE_SIZE"]
    traffic = (2 * fetch_kb + write_kb) * 1024
    d = {
        "kernel": "cse::enhance_kernel<512, false>",
        "round": rnd,
        "command": ("rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) -- "
                    "python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"),
        "units_per_launch": int(units),
        "fetch_size_kb_raw": fetch_kb, "write_size_kb_raw": write_kb,
        "correction": "gfx950: FETCH_SIZE x2 (half-counted streaming reads); KiB -> x1024",
        "hbm_bytes_per_launch": traffic,
        "algorithmic_bytes_per_launch": int(units) * 3084,
        "sq": {k: v for k, v in pmc.items() if k.startswith(("SQ_", "GRBM"))},
    }
    json.dump(d, open("profiles/pmc_traffic.json", "w"), indent=1)
    print(f"traffic {traffic / 1e6:.1f} MB per launch = {traffic / (int(units) * 3084):.4f} "
          f"of algorithmic")


if __name__ == "__main__":
    main(*sys.argv[1:])
