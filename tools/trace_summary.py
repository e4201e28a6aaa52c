"""Per-kernel durations (last launch of each kernel) from rocprofv3 kernel-trace CSVs.

    python tools/trace_summary.py gpurun_out/trace_mixed_default [more dirs ...]
"""
import csv
import glob
import os
import sys


def summary(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "crr" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = {}
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crr::", "")
        last.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {n: sorted(v)[len(v) // 2] for n, v in last.items()}


if __name__ == "__main__":
    res = {d: summary(d) for d in sys.argv[1:]}
    names = sorted({n for r in res.values() for n in r})
    print("kernel".ljust(44) + "".join(os.path.basename(d)[-14:].rjust(16) for d in res))
    for n in names:
        print(n[:43].ljust(44) + "".join(f"{res[d].get(n, float('nan')):16.1f}" for d in res))
