#!/bin/bash
# Alternating A/B (ROUNDS times) of the libraries in LIBS on the config-3 shard and the config-4 long
# tail (NO_LT=1: config 3 only), one box.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for L in ${LIBS}; do
    b=$(basename $L .so)
    timeout -k 10 300 python tools/prof_kernel.py --native --wf ${WF:-1250000} --reps 5 --lib $L >> gpurun_out/alt_c3_$b.log 2>&1
    rc=$?; echo "c3 $b $r rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
    if [ -z "${NO_LT:-}" ]; then
      timeout -k 10 300 python tools/prof_longtail.py --native --n 2000 --thresholds 256 --reps 3 --lib $L >> gpurun_out/alt_c4_$b.log 2>&1
      rc=$?; echo "c4 $b $r rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
    fi
  done
done
exit 0
