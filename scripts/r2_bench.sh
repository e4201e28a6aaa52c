#!/bin/bash
# GPU tests (TESTS=1), then the default bench line.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/status.log; exit $rc
