#!/bin/bash
# Config 4: the long-history threshold (lane per workflow below it, a wavefront per run above) swept.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python tools/prof_longtail.py --native --n 2000 --thresholds ${THR:-256,192,128,96,64} --reps 3 \
  > gpurun_out/lt_thr.log 2>&1 || { tail -5 gpurun_out/lt_thr.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/lt_thr.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["threshold"], round(d["median_ms"], 3), "%.3g" % d["events_per_s"], d["wave_tail"], d["same_as_first"], d["ok"],
              [round(x, 3) for x in d["phase_ms"]])
PY
