#!/bin/bash
# Round 6: the GPU test suite (or the tests named in $TESTS), smoke, then the full bench line (driver
# contract, N = 1) unless NO_BENCH is set.  Each step under its own limit; stops at the first failure.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
TAG="${TAG:-r6}"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full_$TAG.json 2> gpurun_out/bench_full_$TAG.err || { tail -20 gpurun_out/bench_full_$TAG.err; exit 1; }
tail -c 3000 gpurun_out/bench_full_$TAG.json
