#!/bin/bash
# Round-5 end: the GPU test suite, smoke, the full bench line (driver contract, N = 1), then the
# rocprofv3 kernel stats and traffic passes (scripts/profiles_r5.sh).  Each step under its own limit.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_r5.log 2>&1 || { tail -5 gpurun_out/pytest_gpu_r5.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r5.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5.log 2>&1 || { tail -5 gpurun_out/smoke_r5.log; exit 1; }
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full_r5.json 2> gpurun_out/bench_full_r5.err || { tail -5 gpurun_out/bench_full_r5.err; exit 1; }
tail -c 600 gpurun_out/bench_full_r5.json
[ -n "${NO_PROFILES:-}" ] || bash scripts/profiles_r5.sh
