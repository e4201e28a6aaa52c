"""Per-kernel PMC report over the rocprofv3 --pmc passes of scripts/r2_profiles.sh.

    python tools/pmc_report.py gpurun_out/pmc_c3 [--events events.json] > profiles/round2/pmc_c3.md

Each pass directory p<i>/ holds pmc_counter_collection.csv (one row per dispatch x counter x
dimension instance).  Per kernel: the median over its dispatches of the per-dispatch sums.  Derived:
instructions and wave cycles per wavefront, SQ_WAIT_ANY share of wave cycles, LDS bank-conflict share
of LDS-active cycles, HBM bytes (FETCH_SIZE x 2 -- the gfx950 correction of MI355X_MICROARCH.md
"HBM" -- and WRITE_SIZE, both in KB), and with --events (kernel -> events replayed per launch) the
instructions per event.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> [per dispatch]
    for f in sorted(glob.glob(os.path.join(root, "p*", "pmc_counter_collection.csv"))):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("crr::", "").strip()
            acc[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _d, c), v in acc.items():
            per[k][c].append(v)
    return {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in per.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("root")
    p.add_argument("--events", default=None, help="json: kernel name -> events per launch")
    p.add_argument("--min-waves", type=float, default=64)
    p.add_argument("--kernels", default="replay,widen,compact", help="comma-separated name fragments to report")
    a = p.parse_args()
    data = load(a.root)
    ev = json.load(open(a.events)) if a.events else {}
    print(f"PMC per kernel launch (median over dispatches), {a.root}\n")
    print("| kernel | waves | VALU/wave | SALU/wave | LDS/wave | VMEM rd/wave | wave cycles/wave | WAIT_ANY | "
          "LDS bank conflict | FETCHx2 MB | WRITE MB | L2 hit | VALU+SALU per event |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for k, c in sorted(data.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        waves = c.get("SQ_WAVES", 0)
        if waves < a.min_waves or not any(f in k for f in a.kernels.split(",")):
            continue
        w = max(waves, 1)
        wait = c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_LDS_IDX_ACTIVE", 1), 1)
        hit = c.get("TCC_HIT_sum", 0) / max(c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0), 1)
        per_ev = ""
        if k in ev and ev[k]:
            per_ev = f"{(c.get('SQ_INSTS_VALU', 0) + c.get('SQ_INSTS_SALU', 0)) / ev[k]:.0f}"
        print(f"| {k} | {waves:.0f} | {c.get('SQ_INSTS_VALU', 0) / w:.0f} | {c.get('SQ_INSTS_SALU', 0) / w:.0f} | "
              f"{c.get('SQ_INSTS_LDS', 0) / w:.0f} | {c.get('SQ_INSTS_VMEM_RD', 0) / w:.0f} | "
              f"{c.get('SQ_WAVE_CYCLES', 0) / w:.0f} | {wait:.2f} | {conf:.2f} | "
              f"{2 * c.get('FETCH_SIZE', 0) / 1024:.1f} | {c.get('WRITE_SIZE', 0) / 1024:.1f} | {hit:.2f} | {per_ev} |")


if __name__ == "__main__":
    main()
