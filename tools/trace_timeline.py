"""Start / end of each kernel of the last crr_replay launch group in a rocprofv3 kernel trace (us,
relative to the group's first start): which segment is the critical path when they run concurrently.

    python tools/trace_timeline.py gpurun_out/trace_mixed_x
"""
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "crr" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last group: from the last replay_retry_kernel back to the previous one
    idx = [i for i, r in enumerate(rows) if "replay_retry_kernel" in r["Kernel_Name"]]
    lo = idx[-2] + 1 if len(idx) > 1 else 0
    grp = rows[lo:idx[-1] + 1]
    t0 = min(int(r["Start_Timestamp"]) for r in grp)
    print(d)
    for r in grp:
        n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crr::", "")
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"  {n[:40]:40s} {s:9.1f} {e:9.1f} {e - s:9.1f}")
