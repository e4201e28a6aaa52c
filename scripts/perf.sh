#!/bin/bash
# Unprofiled kernel times (HIP events) of the full-size native mixed shard (config 3) and long tail
# (config 4); optional GPU tests first (TESTS=1) and variant libraries (LIBS).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
for L in default ${LIBS:-}; do
  b=$(basename $L .so); arg=""; [ "$L" != "default" ] && arg="--lib $L"
  timeout -k 10 300 python tools/prof_kernel.py --native --wf ${WF:-1250000} --reps 5 $arg > gpurun_out/perf_mixed_$b.log 2>&1
  rc=$?; echo "mixed $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python tools/prof_longtail.py --native --n ${LT_N:-2000} --thresholds 256 --reps 3 $arg > gpurun_out/perf_lt_$b.log 2>&1
  rc=$?; echo "longtail $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
