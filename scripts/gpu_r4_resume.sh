#!/bin/bash
# Round 4: the resume path in the compact tiers -- its GPU tests, then the passive-replication probe in
# both modes (compact tiers / the round-3 HBM-row path), each step under its own time limit.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_resume.py tests/test_gpu_kats.py tests/test_state_builder.py} \
  -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_resume.log 2>&1
rc=$?; log "pytest resume rc=$rc"; tail -5 gpurun_out/pytest_resume.log; [ $rc -ne 0 ] && exit $rc
for mode in "" "--hbm-rows" ""; do
  timeout -k 10 300 python -u tools/prof_replication.py --reps 5 $mode >> gpurun_out/repl_ab.jsonl 2>> gpurun_out/repl_ab.err
  rc=$?; log "prof_replication $mode rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/repl_ab.err; exit $rc; }
done
cat gpurun_out/repl_ab.jsonl
exit 0
