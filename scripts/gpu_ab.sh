#!/bin/bash
# Alternating A/B of library variants (tools/variants/<name>.so; "product" = cadence_amd/libcadence_replay.so)
# over workloads: WORK="c2 c3 c4 repl" (config-2 / config-3 kernels via tools/prof_kernel.py, config 4 via
# tools/prof_longtail.py, passive replication via tools/prof_replication.py), REPS rounds.  Prints one
# line per run with the median kernel time.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
for r in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-product}; do
    L=cadence_amd/libcadence_replay.so; [ "$V" != product ] && L=tools/variants/$V.so
    for W in ${WORK:-c2}; do
      case $W in
        c2) CMD="python tools/prof_kernel.py --reps 10 --lib $L" ;;
        c3) CMD="python tools/prof_kernel.py --native --wf 1250000 --reps 5 --lib $L" ;;
        c4) CMD="python tools/prof_longtail.py --native --n 2000 --thresholds 256 --reps 3 --lib $L" ;;
        repl) CMD="python tools/prof_replication.py --reps 5 --lib $L" ;;
      esac
      timeout -k 10 300 $CMD > gpurun_out/ab_${W}_${V}_$r.log 2>&1
      rc=$?; log "$W $V $r rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_${W}_${V}_$r.log; exit $rc; }
      echo "$W $V $(grep -o '"median_ms": [0-9.]*' gpurun_out/ab_${W}_${V}_$r.log | tail -1) $(grep -o '"mismatches": [0-9]*' gpurun_out/ab_${W}_${V}_$r.log | head -1)"
    done
  done
done
exit 0
