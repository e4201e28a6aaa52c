#!/bin/bash
# One PMC pass (instruction mix) over the native long tail for each library in LIBS ("default" = in-tree).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in ${LIBS:-default}; do
  b=$(basename $L .so); arg=""; [ "$L" != "default" ] && arg="--lib $R/$L"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH \
    -d "$R/gpurun_out/pmc_$b" -o pmc --output-format csv \
    -- python3 "$R/tools/prof_longtail.py" --native --n ${LT_N:-2000} --thresholds 256 --reps 1 $arg > "$R/gpurun_out/pmc_$b.log" 2>&1
  rc=$?; echo "pmc $b rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && exit $rc
done
exit 0
