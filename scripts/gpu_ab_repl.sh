#!/bin/bash
# Resume / loaded-state GPU tests, then alternating passive-replication step times (tools/prof_replication.py)
# for the libraries named in VARIANTS ("product" = cadence_amd/libcadence_replay.so).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_resume.py tests/test_gpu_kats.py tests/test_state_builder.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_repl.log 2>&1
  rc=$?; log "pytest rc=$rc"; tail -3 gpurun_out/pytest_repl.log; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-product}; do
    L=cadence_amd/libcadence_replay.so; [ "$V" != product ] && L=tools/variants/$V.so
    timeout -k 10 300 python tools/prof_replication.py --lib $L > gpurun_out/ab_repl_${V}_$r.log 2>&1
    rc=$?; log "repl $V $r rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ab_repl_${V}_$r.log; exit $rc; }
    echo "repl $V $(grep -o '"median_ms": [0-9.]*' gpurun_out/ab_repl_${V}_$r.log) $(grep -o '"mismatches": [0-9]*' gpurun_out/ab_repl_${V}_$r.log)"
  done
done
exit 0
