#!/bin/bash
# GPU suite on the current build, then config-4 (long tail) and config-3 kernel times for the variant
# libraries named in VARIANTS (tools/variants/<name>.so; "product" = cadence_amd/libcadence_replay.so),
# alternating, REPS rounds.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; log "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_ab.log | head -30; exit $rc; }
fi
for r in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-product}; do
    L=cadence_amd/libcadence_replay.so; [ "$V" != product ] && L=tools/variants/$V.so
    if [ -n "${C4-1}" ]; then
      timeout -k 10 300 python tools/prof_longtail.py --native --n 2000 --thresholds 256 --reps 3 --lib $L > gpurun_out/ab_c4_${V}_$r.log 2>&1
      rc=$?; log "c4 $V $r rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_c4_${V}_$r.log; exit $rc; }
      echo "c4 $V $(grep -o '"median_ms": [0-9.]*' gpurun_out/ab_c4_${V}_$r.log | head -1) $(grep -o '"ok": [0-9]*' gpurun_out/ab_c4_${V}_$r.log | head -1)"
    fi
    if [ -n "${C3:-}" ]; then
      timeout -k 10 300 python tools/prof_kernel.py --native --wf 1250000 --reps 5 --lib $L > gpurun_out/ab_c3_${V}_$r.log 2>&1
      rc=$?; log "c3 $V $r rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_c3_${V}_$r.log; exit $rc; }
      echo "c3 $V $(tail -c 300 gpurun_out/ab_c3_${V}_$r.log | tr '\n' ' ')"
    fi
  done
done
exit 0
