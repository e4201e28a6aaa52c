#!/bin/bash
# Round 6: the GPU suite, then CRR_IN_STARTED_AUX on / off (the layout's ActivityTaskStarted -> scheduled side
# record join), alternated on one box: the config-3 shard and passive replication.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-sab}
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
fi
for r in 1 2 3; do
  for v in on off; do
    X=""; [ $v = off ] && X="--no-started-aux"
    timeout -k 10 300 python -u tools/prof_kernel.py --native --wf 1250000 --reps 5 $X > gpurun_out/${TAG}_c3_${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_c3_${v}_$r.log; exit 1; }
    echo c3 $v $r $(grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/${TAG}_c3_${v}_$r.log)
    timeout -k 10 300 python -u tools/prof_replication.py --reps 5 $X > gpurun_out/${TAG}_repl_${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_repl_${v}_$r.log; exit 1; }
    echo repl $v $r $(grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/${TAG}_repl_${v}_$r.log | tail -1)
  done
done
