#!/bin/bash
# Native long tail, unprofiled, with several replay_big_kernel thresholds (CAPS: "default 64 1000000").
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for C in ${CAPS:-default 64 1000000}; do
  arg=""; [ "$C" != "default" ] && arg="--big-caps $C"
  timeout -k 10 300 python tools/prof_longtail.py --native --n ${LT_N:-2000} --thresholds 256 --reps 3 $arg > gpurun_out/ltc_$C.log 2>&1
  rc=$?; echo "lt caps $C rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
