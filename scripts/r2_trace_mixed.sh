#!/bin/bash
# Kernel trace (start / end timestamps) of the full-size mixed shard, default library and variants
# (LIBS): which tier kernel is the critical path of the concurrent segment launches; with
# PRE=GPU_MAX_HW_QUEUES=1 every kernel runs alone (solo durations).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp; cd "$R"
for L in default ${LIBS:-}; do
  b=$(basename $L .so); arg=""; [ "$L" != "default" ] && arg="--lib $L"
  env ${PRE:-} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_mixed_$b -o run -- \
    python tools/prof_kernel.py --native --wf ${WF:-1250000} --reps 3 $arg ${ARGS:-} > gpurun_out/trace_mixed_$b.log 2>&1
  rc=$?; echo "trace $b rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
