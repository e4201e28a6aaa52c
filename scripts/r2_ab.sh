#!/bin/bash
# A/B of variant libraries (LIBS) against the in-tree build: config 2 (1M x 29), the config-3 mixed
# shard and the config-4 long tail (HIP-event kernel times), then optionally (SOLO=1) solo per-kernel
# times of the mixed shard under one hardware queue.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for L in default ${LIBS:-}; do
  b=$(basename $L .so); arg=""; [ "$L" != "default" ] && arg="--lib $L"
  if [ -z "${NO_C23:-}" ]; then
    timeout -k 10 200 python tools/prof_kernel.py --reps 10 $arg > gpurun_out/ab_c2_$b.log 2>&1
    rc=$?; echo "c2 $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python tools/prof_kernel.py --native --wf ${WF:-1250000} --reps 5 $arg > gpurun_out/ab_c3_$b.log 2>&1
    rc=$?; echo "c3 $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
    for m in ${MERGE:-}; do
      timeout -k 10 300 python tools/prof_kernel.py --native --wf ${WF:-1250000} --reps 5 --merge $m $arg > gpurun_out/ab_c3m${m}_$b.log 2>&1
      rc=$?; echo "c3 merge $m $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
    done
  fi
  if [ -z "${NO_LT:-}" ]; then
    timeout -k 10 300 python tools/prof_longtail.py --native --n ${LT_N:-2000} --thresholds 256 --reps 3 $arg > gpurun_out/ab_c4_$b.log 2>&1
    rc=$?; echo "c4 $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
  fi
done
if [ -n "${SOLO:-}" ]; then PRE=GPU_MAX_HW_QUEUES=1 bash scripts/r2_trace_mixed.sh || exit $?; fi
exit 0
