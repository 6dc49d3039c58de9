"""tools/micro/valu_cal output -> profiles/<round>_micro_valu_cal.json.

    python tools/valu_cal_summary.py gpurun_out/valu_cal.txt profiles/r06_micro_valu_cal.json [valu_mix.txt]

Keeps the printed table (as text) and the JSON rows, and states what the rows
say about the pricing bench.py's roofline uses: the f32 VALU and packed-f32
rates in FLOP/clk/SIMD at the held clock, and the SIMD cycles of one wave64
instruction of each kind with 8 waves per SIMD.
"""
import json
import sys


def parse_mix(path):
    """tools/micro/valu_mix output -> {"K1 + K2": {waves: SIMD cycles per instruction}}."""
    import re
    out = {}
    for line in open(path):
        if line.startswith("#") or "+" not in line:
            continue
        name = " + ".join(x.strip() for x in line.split("W=1")[0].split("+"))
        out[name] = {int(w): float(c) for w, c in re.findall(r"W=(\d+)\s+[\d.]+ ms\s+([\d.]+) cyc", line)}
    return out


def main(src, dst, mix=None):
    rows, table = [], []
    for line in open(src):
        if line.startswith("JSON "):
            rows.append(json.loads(line[5:]))
        elif line.strip():
            table.append(line.rstrip("\n"))
    out = {"source": "tools/micro/valu_cal.hip (chip-wide, HIP-event timed)", "table": table, "rows": rows}
    by = {(r["op"], r["waves_per_simd"]): r for r in rows}
    summ = {}
    for op in ("v_fma_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_add_f32", "v_exp_f32", "v_fma_f64"):
        r = by.get((op, 8))
        if r:
            flop_per_clk_simd = r["tflops"] * 1e12 / (r["clock_ghz"] * 1e9 * r["simds"])
            summ[op] = {"cycles_per_wave_inst_8w": r["cycles_per_wave_inst"],
                        "flop_per_clk_per_simd_8w": flop_per_clk_simd,
                        "tflops_8w": r["tflops"], "clock_ghz": r["clock_ghz"]}
    out["summary_8_waves"] = summ
    if mix:
        out["mix_source"] = "tools/micro/valu_mix.hip (" + mix + "), SIMD cycles per wave64 instruction at 2.4 GHz"
        out["mix"] = parse_mix(mix)
    json.dump(out, open(dst, "w"), indent=1)
    for k, v in summ.items():
        print(k, v)


if __name__ == "__main__":
    main(*sys.argv[1:4])
