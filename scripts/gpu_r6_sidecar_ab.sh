#!/bin/bash
# Round 6: the live-ID sidecar's price on the replay (config-3 shard, passive replication), alternated on one box.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for r in 1 2; do
  for v in side noside; do
    F=""; [ $v = noside ] && F="--no-live-ids"
    timeout -k 10 300 python -u tools/prof_kernel.py --native --wf 1250000 --reps 5 $F > gpurun_out/sideab_c3_${v}_$r.log 2>&1 || { tail -5 gpurun_out/sideab_c3_${v}_$r.log; exit 1; }
    timeout -k 10 300 python -u tools/prof_replication.py --reps 5 $F > gpurun_out/sideab_repl_${v}_$r.log 2>&1 || { tail -5 gpurun_out/sideab_repl_${v}_$r.log; exit 1; }
    echo $v $r c3 $(tail -1 gpurun_out/sideab_c3_${v}_$r.log | cut -c1-200) repl $(tail -1 gpurun_out/sideab_repl_${v}_$r.log | cut -c1-200)
  done
done
