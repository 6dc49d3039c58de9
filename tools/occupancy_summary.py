"""Summarise tools/occupancy_probe.sh into profiles/r05_occupancy_probe.json:
per build the kernel trace's VGPRs / LDS / scratch / kernel ms and the SQ pass
per launch (wait shares of SQ_WAVE_CYCLES; mean resident waves per SIMD =
4 x SQ_WAVE_CYCLES (quad-cycles) / (1024 SIMDs x SQ_BUSY_CYCLES / 32))."""
import csv
import glob
import json
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
KN = "enhance_kernel<512"
# WG<512, false>::BYTES of each build (dynamic LDS: the kernel trace's
# LDS_Block_Size reads 0); from a host program printing the constant under the
# build's -D flags
LDS = {"libcse": 53600, "r04": 53600, "b3": 53600, "p3": 35136, "p4": 35136, "s3": 38496,
       "s4": 38496, "s4i": 38496}


def main(out="profiles/r05_occupancy_probe.json"):
    base = os.path.join(REPO, "gpurun_out", "occ")
    res = {}
    for d in sorted(glob.glob(os.path.join(base, "kt_*"))):
        if not os.path.isdir(d):
            continue
        n = os.path.basename(d)[3:]
        rows = [r for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))
                if KN in r["Kernel_Name"]]
        ms = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows)
        r0 = rows[0]
        e = {"kernel": r0["Kernel_Name"][:60], "launches": len(rows), "kernel_ms_median": ms[len(ms) // 2],
             # VGPR_Count is in units of 2 in this ROCm's trace (153 -> 80)
             "vgprs_alloc": 2 * int(r0["VGPR_Count"]), "lds_bytes": LDS.get(n),
             "scratch_bytes_per_lane": int(r0.get("Scratch_Size") or 0)}
        e["waves_per_simd_limit"] = min(512 // e["vgprs_alloc"], 163840 // e["lds_bytes"])
        acc, disp = {}, set()
        for r in csv.DictReader(open(os.path.join(base, f"pmc_{n}", "run_counter_collection.csv"))):
            if KN not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] = acc.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
        pmc = {k: v / len(disp) for k, v in acc.items()}
        w = pmc["SQ_WAVE_CYCLES"]
        e["pmc_per_launch"] = pmc
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            e["share_" + k[3:].lower()] = pmc[k] / w
        e["mean_waves_per_simd"] = 4 * w / (1024 * pmc["SQ_BUSY_CYCLES"] / 32)
        res[n] = e
        print(f"{n:7s} ms {e['kernel_ms_median']:7.2f} vgpr {e['vgprs_alloc']:3d} lds {e['lds_bytes']:6d} "
              f"scr {e['scratch_bytes_per_lane']:4d} lim {e['waves_per_simd_limit']} "
              f"mean_w {e['mean_waves_per_simd']:.2f} wait_any {e['share_wait_any']:.3f} "
              f"wait_inst {e['share_wait_inst_any']:.3f} active {e['share_active_inst_any']:.3f} "
              f"valu {pmc['SQ_INSTS_VALU']:.3e}")
    json.dump({"source": "tools/occupancy_probe.sh + tools/occupancy_summary.py (r05)",
               "workload": "tools/time_enhance.py: 13 pairs x 10 s, n_fft 512 half of the grid",
               "builds": res}, open(os.path.join(REPO, out), "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:])
