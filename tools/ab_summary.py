"""Median kernel times of scripts/r2_ab.sh logs: python tools/ab_summary.py [gpurun_out]"""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(d, "ab_c*_*.log"))):
    for line in open(f):
        if line.startswith("{") and "median_ms" in line:
            r = json.loads(line)
            print(f"{os.path.basename(f)[:-4]:28s} {r['median_ms']:8.3f} ms  {r['events_per_s']:.3e} ev/s  ok={r['ok']}")
