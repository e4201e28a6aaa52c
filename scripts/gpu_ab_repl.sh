#!/bin/bash
# Passive-replication kernel time (tools/prof_replication.py) for the variant libraries in VARIANTS
# (tools/variants/<name>.so; "product" = cadence_amd/libcadence_replay.so; "hbm" = the product on the
# round-3 HBM-row path), alternating, REPS rounds.  No tests: variants may be wrong by design.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
for r in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-product}; do
    L=cadence_amd/libcadence_replay.so; X=""
    [ "$V" = hbm ] && X="--hbm-rows"
    [ "$V" != product ] && [ "$V" != hbm ] && L=tools/variants/$V.so
    timeout -k 10 300 python tools/prof_replication.py --reps 5 --lib $L $X ${WF:+--wf $WF} > gpurun_out/ab_repl_${V}_$r.log 2>&1
    rc=$?; log "repl $V $r rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_repl_${V}_$r.log; exit $rc; }
    echo "repl $V $(grep -o '"median_ms": [0-9.]*' gpurun_out/ab_repl_${V}_$r.log | head -1) $(grep -o '"mismatches": [0-9]*' gpurun_out/ab_repl_${V}_$r.log | head -1)"
  done
done
exit 0
