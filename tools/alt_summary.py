"""Per-run medians of scripts/r2_alt.sh logs: python tools/alt_summary.py [gpurun_out]"""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(d, "alt_c*_*.log"))):
    ms = [json.loads(l)["median_ms"] for l in open(f) if l.startswith("{") and "median_ms" in l]
    ok = [json.loads(l)["ok"] for l in open(f) if l.startswith("{") and "median_ms" in l]
    print(f"{os.path.basename(f)[:-4]:24s} " + " ".join(f"{m:8.3f}" for m in ms) + f"   ok={ok}")
