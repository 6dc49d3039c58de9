"""Per enhance launch in a rocprofv3 kernel trace: its start/end and the
side-stream kernels that ran between its start and the next launch's start
(the analysis chain and what of it is left after the launch drains).

    python tools/gap_trace.py gpurun_out/<dir>/run_kernel_trace.csv [n_fft]
"""
import csv
import sys


def main(path, nfft="512"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    ms = lambda t: (int(t) - t0) / 1e6  # noqa: E731
    enh = [i for i, r in enumerate(rows) if f"enhance_kernel<{nfft}, false>" in r["Kernel_Name"]]
    for n, i in enumerate(enh):
        r = rows[i]
        nxt = rows[enh[n + 1]] if n + 1 < len(enh) else None
        gap = (ms(nxt["Start_Timestamp"]) - ms(r["End_Timestamp"])) if nxt else None
        print(f"enhance {ms(r['Start_Timestamp']):10.3f} -> {ms(r['End_Timestamp']):10.3f} ms"
              + (f"   gap to next {gap:.3f} ms" if gap is not None else ""))
        end = int(nxt["Start_Timestamp"]) if nxt else None
        after = 0.0
        for q in rows[i + 1:(enh[n + 1] if nxt else len(rows))]:
            s, e = ms(q["Start_Timestamp"]), ms(q["End_Timestamp"])
            if end is not None and int(q["Start_Timestamp"]) > end:
                continue
            tail = max(0.0, e - max(s, ms(r["End_Timestamp"])))
            after += tail if s >= ms(r["End_Timestamp"]) else 0.0
            print(f"    {q['Kernel_Name'][:58]:58s} {s:10.3f} {e:10.3f}  ({(e - s) * 1e3:8.1f} us)")


if __name__ == "__main__":
    main(*sys.argv[1:])
