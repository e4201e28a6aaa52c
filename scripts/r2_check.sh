#!/bin/bash
# Round 2: GPU parity tests, then per-kernel breakdown (rocprofv3 kernel trace) of the mixed
# (config-3 shape) and long-tail (config-4 shape) workloads, then PMC passes on the mixed workload.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/mprof" -o run --output-format csv \
  -- python3 "$R/tools/prof_kernel.py" --mixed --wf ${WF:-100000} --reps 3 > "$R/gpurun_out/mprof.log" 2>&1
rc=$?; echo "mixed prof rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ltprof" -o lt --output-format csv \
  -- python3 "$R/tools/prof_longtail.py" --n ${LT_N:-200} --thresholds 256 --reps 2 > "$R/gpurun_out/ltprof.log" 2>&1
rc=$?; echo "longtail prof rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && exit $rc
if [ -n "${PMC:-}" ]; then
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/mpmc$i" -o pmc --output-format csv \
      -- python3 "$R/tools/prof_kernel.py" --mixed --wf ${WF:-100000} --reps 1 > "$R/gpurun_out/mpmc$i.log" 2>&1
    rc=$?; echo "mixed pmc pass $i ($line) rc=$rc" >> "$R/gpurun_out/status.log"
    [ $rc -ne 0 ] && exit $rc
  done < "$R/scripts/pmc_passes.txt"
fi
exit 0
