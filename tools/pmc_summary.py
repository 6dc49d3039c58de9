"""Summarise a tools/profile_all.sh run into profiles/ (committed evidence).

For every kernel of interest: rocprofv3 --kernel-trace --stats average duration
and calls, and the PMC counters of the separate --pmc passes, per launch
(counter sum over the profiled launches / launches).  HBM traffic per launch =
(2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 (gfx950 correction, MI355X_MICROARCH.md
HBM/rocprofv3 section: FETCH_SIZE counts half the bytes of wide streaming reads).
VALU cycles (r06 pricing, measured chip-wide by tools/micro/valu_cal.hip and
valu_mix.hip, see bench.py: a wave64 f32 VALU instruction 2 SIMD cycles, a
packed v_pk_*_f32 4, a transcendental 8, an fp64 FMA/MUL/ADD 4) over 1024
SIMDs x SQ_BUSY_CYCLES / 32 (per-shader-
engine cycles with waves resident, summed over the 32 SEs).  The packed
instructions are counted, not assumed: the F32 class counters
(SQ_INSTS_VALU_ADD/MUL/FMA_F32) count a v_pk_* once, so the scalar build of the
same sources (CSE_PK=0, every f32 operation its own instruction) minus the
product build gives the packed count per class; the FP32 FLOP counter (which
counts a packed instruction's two operations) checks it.  GRBM_GUI_ACTIVE / 8
read twice the shader clock on the r02 boxes, so it is only recorded.

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
SIMDS = 1024
VALU_CYC, PK_CYC, TRANS_CYC, F64_CYC = 2, 4, 8, 4  # SIMD cycles per wave64 instruction (see above)
F64_COUNTERS = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")


def valu_cycles(vi, tr, pk, f64):
    """SIMD cycles of a launch's VALU instructions: vi all VALU, of which tr
    transcendental, pk packed f32, f64 fp64 FMA/MUL/ADD."""
    return VALU_CYC * (vi - tr - pk - f64) + PK_CYC * pk + TRANS_CYC * tr + F64_CYC * f64


def packed_counts(prod, scalar):
    """Packed f32 instructions per class from the F32 class counters of the
    product build (a v_pk_* counted once) and the scalar build (CSE_PK=0: two
    instructions): {add, mul, fma, total, flop_check}.  flop_check compares the
    product's FLOP counter with what its class counters and these packed counts
    imply (FLOPS = ADD + MUL + 2 FMA + TRANS + pk_add + pk_mul + 2 pk_fma)."""
    if not prod or not scalar:
        return None
    out = {}
    for c, k in (("add", "SQ_INSTS_VALU_ADD_F32"), ("mul", "SQ_INSTS_VALU_MUL_F32"),
                 ("fma", "SQ_INSTS_VALU_FMA_F32")):
        if k not in prod or k not in scalar:
            return None
        out[c] = scalar[k] - prod[k]
    out["total"] = out["add"] + out["mul"] + out["fma"]
    fl = prod.get("SQ_INSTS_VALU_FLOPS_FP32")
    if fl:
        implied = (prod["SQ_INSTS_VALU_ADD_F32"] + prod["SQ_INSTS_VALU_MUL_F32"]
                   + 2 * prod["SQ_INSTS_VALU_FMA_F32"] + prod.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
                   + out["add"] + out["mul"] + 2 * out["fma"])
        out["flop_check"] = {"flops_counter": fl, "implied_by_class_counts": implied,
                             "ratio": implied / fl}
    if "SQ_INSTS_VALU" in prod and "SQ_INSTS_VALU" in scalar:
        out["valu_difference"] = scalar["SQ_INSTS_VALU"] - prod["SQ_INSTS_VALU"]
    return out


# WG<NFFT, false>::BYTES (dynamic LDS: the trace's LDS_Block_Size reads 0)
LDS_BYTES = {"enhance_kernel<512, false>": 53600, "enhance_kernel<1024, false>": 52960}


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


def derive(pmc, kernel_ms, packed=None):
    d = {}
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        d["hbm_bytes_per_launch"] = (2 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024
    vi, tr = pmc.get("SQ_INSTS_VALU"), pmc.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
    f64 = sum(pmc.get(k, 0.0) for k in F64_COUNTERS)
    busy = pmc.get("SQ_BUSY_CYCLES")
    if vi and busy:
        need = valu_cycles(vi, tr, packed or 0.0, f64)
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
                                   "pmc_launches": nd}
    # r06: the product build's counts priced per instruction kind, the packed
    # count from the F32 class counters of the product and of the scalar build
    # (CSE_PK=0; the n_fft 1024 kernel issues no packed instruction: its ISA
    # has no v_pk_*, `python tools/isa_sections.py enhance_kernelILi1024ELb0E`)
    for key, name, pk in (("enhance512", "512", "pk512"), ("enhance1024", "1024", "pk1024")):
        k = summary["kernels"][key]
        occ = occupancy(os.path.join(base, f"kt_{name}", "run_kernel_trace.csv"), KERNELS[key])
        if occ:
            k.update(occ)
        ppk, _ = counters(os.path.join(base, f"pmc_{pk}", "run_counter_collection.csv"), KERNELS[key])
        if ppk:
            k["pmc_packed_counters_per_launch"] = ppk
            k["flops_fp32"] = ppk.get("SQ_INSTS_VALU_FLOPS_FP32")
        spk, _ = counters(os.path.join(base, f"pmc_s{name}_pk", "run_counter_collection.csv"), KERNELS[key])
        if spk:
            k["pmc_scalar_build_pk_pass_per_launch"] = spk
        k["packed"] = packed_counts(ppk, spk) if name == "512" else {"total": 0.0, "source": "ISA"}
    for key, k in summary["kernels"].items():
        pk = (k.get("packed") or {}).get("total") if key.startswith("enhance") else 0.0
        k.update(derive(k["pmc_per_launch"], k["kernel_ms_rocprof"], pk))
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
               "valu_issue_cycles_source": ("this build's SQ_INSTS_VALU priced per kind: f32 VALU 2, "
                                            "packed v_pk_* 4, transcendental 8, f64 FMA/MUL/ADD 4 cycles"),
               "packed_insts": (k.get("packed") or {}).get("total"),
               "packed": k.get("packed"),
               "sq_insts_valu_f64": sum(pmc.get(c, 0.0) for c in F64_COUNTERS) if any(
                   c in pmc for c in F64_COUNTERS) else None,
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
