#!/bin/bash
# Long-tail tail-kernel check: GPU tests (optional), then the native long tail with the default
# library and variant builds given in LIBS (space separated).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python tools/prof_longtail.py --native --n ${LT_N:-2000} --thresholds 256 --reps 3 > gpurun_out/lt_default.log 2>&1
rc=$?; echo "lt default rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
for L in ${LIBS:-}; do
  b=$(basename $L .so)
  timeout -k 10 300 python tools/prof_longtail.py --native --n ${LT_N:-2000} --thresholds 256 --reps 3 --lib $L > gpurun_out/lt_$b.log 2>&1
  rc=$?; echo "lt $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
if [ -n "${PROF:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/tltprof" -o lt --output-format csv \
    -- python3 "$R/tools/prof_longtail.py" --native --n ${LT_N:-2000} --thresholds 256 --reps 2 > "$R/gpurun_out/tltprof.log" 2>&1
  rc=$?; echo "tail prof rc=$rc" >> "$R/gpurun_out/status.log"; exit $rc
fi
exit 0
