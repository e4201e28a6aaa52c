#!/bin/bash
# GPU suite (the device-ingest tests last, in their own step), then the headline bench (config 2 only);
# each step under its own time limit, stopping at the first failure.  NO_BENCH=1 skips the bench,
# ONLY=<pytest args> runs just those tests.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
run_tests() {   # name, pytest args...
  local name=$1; shift
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_$name.log 2>&1
  local rc=$?; log "pytest $name rc=$rc"
  tail -4 gpurun_out/pytest_$name.log
  return $rc
}
if [ -n "${ONLY:-}" ]; then
  run_tests only $ONLY || exit $?
else
  run_tests main tests --ignore tests/test_gpu_ingest.py || exit $?
  run_tests ingest tests/test_gpu_ingest.py || exit $?
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 300 python -u bench.py --headline-only --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_headline.log 2>&1
  rc=$?; log "bench rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/bench_headline.log; exit $rc; }
  tail -c 1200 gpurun_out/bench_headline.log
fi
exit 0
