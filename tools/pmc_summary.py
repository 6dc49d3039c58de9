"""Summarise a tools/profile_all.sh run into profiles/ (committed evidence).

For every kernel of interest: rocprofv3 --kernel-trace --stats average duration
and calls, and the PMC counters of the separate --pmc passes, per launch
(counter sum over the profiled launches / launches).  HBM traffic per launch =
(2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 (gfx950 correction, MI355X_MICROARCH.md
HBM/rocprofv3 section: FETCH_SIZE counts half the bytes of wide streaming reads).
VALU issue fraction = (2 x (VALU - TRANS) + 4 x TRANS) SIMD cycles (fp64 FMA/MUL/ADD
at 4) over 1024 SIMDs x SQ_BUSY_CYCLES / 32 (per-shader-engine cycles with
waves resident, summed over the 32 SEs).  GRBM_GUI_ACTIVE / 8 read twice the
shader clock on the r02 boxes, so it is only recorded.

    python tools/pmc_summary.py TAG ROUND [UNITS_512 UNITS_1024]

Writes profiles/{ROUND}_kernels.json (all kernels) and, when the launch sizes
are given, profiles/pmc_enhance512_{ROUND}.json / pmc_enhance1024_{ROUND}.json,
which bench.py reads (matched by units_per_launch) for roofline.traffic/valu.
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
KERNELS = {"enhance512": "enhance_kernel<512, false>", "enhance1024": "enhance_kernel<1024, false>",
           "stoi": "stoi_cells_kernel", "xcorr_lag": "xcorr_lag_kernel"}
SIMDS, VALU_CYC, TRANS_CYC = 1024, 2, 4  # transcendental = 2x v_fma_f32 (tools/micro/valu_rate.hip)


# WG<NFFT, false>::BYTES (dynamic LDS: the trace's LDS_Block_Size reads 0)
LDS_BYTES = {"enhance_kernel<512, false>": 53600, "enhance_kernel<1024, false>": 52800}


def occupancy(trace, kname):
    """(VGPRs allocated, LDS bytes, waves per SIMD) of a kernel from a rocprofv3
    kernel trace: this ROCm's trace gives VGPR_Count in units of 2 registers
    (the 153-VGPR sweep kernel reads 80: 160 allocated, granule 8; 512 per lane
    and SIMD), and the LDS of the dynamically sized kernels comes from
    LDS_BYTES (160 KiB per CU shared by workgroups of 4 waves, one per SIMD)."""
    if not os.path.exists(trace):
        return None
    for r in csv.DictReader(open(trace)):
        if kname in r["Kernel_Name"]:
            v = 2 * (int(r["VGPR_Count"]) + int(r.get("Accum_VGPR_Count") or 0))
            lds = int(r["LDS_Block_Size"]) or LDS_BYTES.get(kname, 0)
            w = min(8, 512 // v)
            if lds:
                w = min(w, 163840 // lds)
            return {"vgprs": v, "lds_bytes": lds, "waves_per_simd": w}
    return None


def stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                          "pct": float(r["Percentage"])}
    return out


def counters(pattern, kname):
    """{counter: value per launch} over the matching dispatches of all pmc dirs:
    per pass (file) the sum over its dispatches / its dispatches, and a counter
    that several passes collected (GRBM_GUI_ACTIVE, SQ_INSTS_VALU, ...) is the
    mean of their per-launch values (r03's summaries summed such counters over
    the passes, e.g. GRBM_GUI_ACTIVE twice)."""
    per, disp = {}, {}
    for f in sorted(glob.glob(pattern)):
        acc, dd = {}, {}
        for r in csv.DictReader(open(f)):
            if kname not in r["Kernel_Name"]:
                continue
            c = r["Counter_Name"]
            acc[c] = acc.get(c, 0.0) + float(r["Counter_Value"])
            dd.setdefault(c, set()).add(r["Dispatch_Id"])
        for c, v in acc.items():
            per.setdefault(c, []).append(v / len(dd[c]))
            disp[c] = disp.get(c, 0) + len(dd[c])
    return {c: sum(v) / len(v) for c, v in per.items()}, disp


def derive(pmc, kernel_ms):
    d = {}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        d["hbm_bytes_per_launch"] = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
    vi, tr = pmc.get("SQ_INSTS_VALU"), pmc.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
    f64 = sum(pmc.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                         "SQ_INSTS_VALU_ADD_F64"))
    busy = pmc.get("SQ_BUSY_CYCLES")
    if vi and busy:
        need = VALU_CYC * (vi - tr - f64) + TRANS_CYC * tr + 2 * VALU_CYC * f64
        cyc = busy / 32
        d["valu_issue_cycles"] = need
        d["busy_cycles_per_se"] = cyc
        d["valu_frac"] = need / (SIMDS * cyc)
        d["clock_ghz_profiled"] = cyc / (kernel_ms / 1e3) / 1e9 if kernel_ms else None
    if "SQ_WAVE_CYCLES" in pmc:
        w = pmc["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS"):
            if k in pmc:
                d["share_" + k[3:].lower()] = pmc[k] / w
    if "SQ_LDS_IDX_ACTIVE" in pmc and busy:
        # LDS-array cycles (summed over the CUs) over the CU cycles of the launch
        d["lds_array_busy"] = pmc["SQ_LDS_IDX_ACTIVE"] / (256 * busy / 32)
        d["lds_cycles_per_lds_inst"] = pmc["SQ_LDS_IDX_ACTIVE"] / pmc["SQ_INSTS_LDS"]
    if "SQ_WAIT_INST_LDS" in pmc and "SQ_WAVE_CYCLES" in pmc:
        d["share_wait_inst_lds"] = pmc["SQ_WAIT_INST_LDS"] / pmc["SQ_WAVE_CYCLES"]
    if "SQ_LDS_BANK_CONFLICT" in pmc and "SQ_INSTS_LDS" in pmc:
        d["lds_conflict_cycles_per_lds_inst"] = pmc["SQ_LDS_BANK_CONFLICT"] / pmc["SQ_INSTS_LDS"]
    return d


def main(tag, rnd, units512=None, units1024=None):
    sys.path.insert(0, REPO)
    import bench
    src_sha = bench.kernel_src_sha()  # the sources the profiled .so was built from
    base = os.path.join(REPO, "gpurun_out", f"prof_{tag}")
    kt = {}
    for name in ("512", "1024", "sweep"):
        p = os.path.join(base, f"kt_{name}", "run_kernel_stats.csv")
        if os.path.exists(p):
            kt[name] = stats(p)
    summary = {"round": rnd, "tag": tag, "commands": {
        "kt512": "rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity",
        "kt1024": "... bench.py --nfft 1024 --steps 3 --warmup 1 --no-cpu-baseline --no-parity",
        "ktsweep": "... tools/bench_sweep.py --pairs 4 --reps 1",
        "pmc": "one rocprofv3 --pmc pass per counter group (tools/profile_all.sh), bench.py --steps 1 --warmup 0"},
        "kernel_stats": kt, "kernels": {}}
    src = {"enhance512": ("512", "512"), "enhance1024": ("1024", "1024"), "stoi": ("sweep", "stoi"),
           "xcorr_lag": ("sweep", "stoi")}
    for key, kname in KERNELS.items():
        ktname, pmcname = src[key]
        ms = None
        for n, v in kt.get(ktname, {}).items():
            if kname in n:
                ms = v["avg_ms"]
        pmc, nd = counters(os.path.join(base, f"pmc_{pmcname}_*", "run_counter_collection.csv"), kname)
        summary["kernels"][key] = {"kernel": kname, "kernel_ms_rocprof": ms, "pmc_per_launch": pmc,
                                   "pmc_launches": nd, **derive(pmc, ms)}
    # r05: the product binary's own counts are the basis (a packed v_pk_*
    # instruction counted once: it issues at the scalar rate); the SQPK pass
    # adds its FP32 FLOPs.  r04 priced the scalar build (CSE_PK=0) instead,
    # which counts instructions the product does not issue; that build's passes
    # are still summarised when present, as a record only.
    for key, name, pk in (("enhance512", "512", "pk512"), ("enhance1024", "1024", "pk1024")):
        k = summary["kernels"][key]
        occ = occupancy(os.path.join(base, f"kt_{name}", "run_kernel_trace.csv"), KERNELS[key])
        if occ:
            k.update(occ)
        ppk, _ = counters(os.path.join(base, f"pmc_{pk}", "run_counter_collection.csv"), KERNELS[key])
        if ppk:
            k["pmc_packed_counters_per_launch"] = ppk
            k["flops_fp32"] = ppk.get("SQ_INSTS_VALU_FLOPS_FP32")
    k512 = summary["kernels"]["enhance512"]
    spmc, _ = counters(os.path.join(base, "pmc_s512_sq1", "run_counter_collection.csv"), KERNELS["enhance512"])
    spk, _ = counters(os.path.join(base, "pmc_s512_pk", "run_counter_collection.csv"), KERNELS["enhance512"])
    ppk, _ = counters(os.path.join(base, "pmc_pk512", "run_counter_collection.csv"), KERNELS["enhance512"])
    if spmc:  # record only (see above)
        k512["pmc_scalar_build_per_launch"] = spmc
        k512["pmc_scalar_build_pk_pass_per_launch"] = spk
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    json.dump(summary, open(os.path.join(REPO, "profiles", f"{rnd}_kernels.json"), "w"), indent=1)
    for key, units in (("enhance512", units512), ("enhance1024", units1024)):
        if not units:
            continue
        k = summary["kernels"][key]
        pmc = k["pmc_per_launch"]
        out = {"kernel": "cse::" + k["kernel"], "round": rnd, "units_per_launch": int(units),
               "kernel_ms": k["kernel_ms_rocprof"],
               "hbm_bytes_per_launch": k.get("hbm_bytes_per_launch"),
               "sq_insts_valu": pmc.get("SQ_INSTS_VALU"), "sq_insts_valu_trans": pmc.get("SQ_INSTS_VALU_TRANS_F32"),
               "grbm_gui_active": pmc.get("GRBM_GUI_ACTIVE"),
               "sq_busy_cycles": pmc.get("SQ_BUSY_CYCLES"),
               "sq_insts_valu_flops_fp32": k.get("flops_fp32"),
               "valu_frac": k.get("valu_frac"), "clock_ghz_profiled": k.get("clock_ghz_profiled"),
               "valu_issue_cycles": k.get("valu_issue_cycles"),
               "valu_issue_cycles_source": "this build's own SQ_INSTS_VALU / _TRANS_F32 (packed counted once)",
               "vgprs": k.get("vgprs"), "lds_bytes": k.get("lds_bytes"),
               "waves_per_simd": k.get("waves_per_simd"),
               "share_wait_inst_any": k.get("share_wait_inst_any"),
               "share_wait_any": k.get("share_wait_any"),
               "share_active_inst_valu": k.get("share_active_inst_valu"),
               "share_active_inst_any": k.get("share_active_inst_any"),
               "lds_conflict_cycles_per_lds_inst": k.get("lds_conflict_cycles_per_lds_inst"),
               "lds_array_busy": k.get("lds_array_busy"),
               "share_wait_inst_lds": k.get("share_wait_inst_lds"),
               "kernel_src_sha": src_sha,
               "source": f"profiles/{rnd}_kernels.json (tools/profile_all.sh {tag})"}
        json.dump(out, open(os.path.join(REPO, "profiles", f"pmc_{key}_{rnd}.json"), "w"), indent=1)
    for key, k in summary["kernels"].items():
        print(key, "ms", k["kernel_ms_rocprof"], "valu_frac", k.get("valu_frac"),
              "hbm MB", (k.get("hbm_bytes_per_launch") or 0) / 1e6,
              "wait_inst", k.get("share_wait_inst_any"), "conf/lds", k.get("lds_conflict_cycles_per_lds_inst"))


if __name__ == "__main__":
    main(*sys.argv[1:])
