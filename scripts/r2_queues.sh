#!/bin/bash
# Mixed shard (config 3) kernel time against the number of hardware queues HIP gives the process
# (tier segments on side streams share a queue once there are more streams than queues).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for q in ${QS:-1 4 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/prof_kernel.py --native --wf ${WF:-1250000} --reps 5 ${ARGS:-} > gpurun_out/queues_$q.log 2>&1
  rc=$?; echo "q=$q rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
