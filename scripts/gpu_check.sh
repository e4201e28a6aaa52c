#!/bin/bash
# GPU suite then the headline bench (config 2 only), each step under its own time limit; stops at the
# first failure.  TESTS=<pytest node ids> narrows the suite; NO_BENCH=1 skips the bench.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; log "pytest rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_gpu.log; exit $rc; }
tail -3 gpurun_out/pytest_gpu.log
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 300 python -u bench.py --headline-only --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_headline.log 2>&1
  rc=$?; log "bench rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/bench_headline.log; exit $rc; }
  tail -c 1500 gpurun_out/bench_headline.log
fi
exit 0
