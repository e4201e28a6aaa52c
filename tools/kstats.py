"""Top kernels of a rocprofv3 --stats run: python tools/kstats.py <dir-with-*_kernel_stats.csv> [n]."""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{r['Name'][:90]:90s} calls={int(r['Calls']):5d} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
          f"share={float(r['TotalDurationNs']) / tot:5.1%}")
