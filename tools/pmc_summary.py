"""Summarise rocprofv3 --pmc CSVs under a directory: per kernel, per counter (min over dispatches)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for d in sorted(glob.glob(f"{root}/pmc*/pmc_counter_collection.csv")):
    rows = list(csv.DictReader(open(d)))
    agg = collections.defaultdict(float)
    for r in rows:
        if "replay" not in r["Kernel_Name"] and "checksum" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("crr::", "")
        agg[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (k, disp, name), v in agg.items():
        per[(k, name)].append(v)
    for (k, n), v in sorted(per.items()):
        print(f"{d.split('/')[-2]:6s} {k:22s} {n:22s} {min(v):16.0f} {max(v):16.0f}")
for d in sorted(glob.glob(f"{root}/pmc1/pmc_kernel_trace.csv")):
    for r in csv.DictReader(open(d)):
        if "replay" in r["Kernel_Name"]:
            print("trace", r["Kernel_Name"].split("(")[0], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us",
                  "vgpr", r["VGPR_Count"], "sgpr", r["SGPR_Count"], "lds", r["LDS_Block_Size"], "scratch", r["Scratch_Size"])
