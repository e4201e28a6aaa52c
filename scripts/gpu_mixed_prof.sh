#!/bin/bash
# kernel-trace breakdown of the mixed (config-3-like) workload
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/mprof" -o run --output-format csv \
  -- python3 "$R/tools/prof_kernel.py" --mixed --wf ${WF:-200000} --reps 3 ${PROF_ARGS:-} > "$R/gpurun_out/mprof.log" 2>&1
rc=$?; echo "mixed prof rc=$rc" >> "$R/gpurun_out/status.log"; exit $rc
