#!/bin/bash
# Kernel-trace breakdown of the full-size mixed (config 3 per-GPU shard, 1.25M workflows) and long-tail
# (config 4) workloads from the native generator; optional GPU tests first.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/nprof" -o run --output-format csv \
  -- python3 "$R/tools/prof_kernel.py" --native --wf ${WF:-1250000} --reps 3 > "$R/gpurun_out/nprof.log" 2>&1
rc=$?; echo "native mixed prof rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/nltprof" -o lt --output-format csv \
  -- python3 "$R/tools/prof_longtail.py" --native --n ${LT_N:-2000} --thresholds 256 --reps 2 > "$R/gpurun_out/nltprof.log" 2>&1
rc=$?; echo "native longtail prof rc=$rc" >> "$R/gpurun_out/status.log"; exit $rc
