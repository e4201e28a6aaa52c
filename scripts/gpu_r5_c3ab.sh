#!/bin/bash
# Round 5: config-3 kernel-group A/B (tools/prof_kernel.py --native, the bench's 1.25M-workflow shard) of
# variant libraries against the in-tree one, alternated on one box.
set -u
for r in 1 2 3; do
  for v in product ${VARIANTS:-}; do
    L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
    timeout -k 10 300 python -u tools/prof_kernel.py --native --wf 1250000 --reps 5 --lib $L > gpurun_out/c3ab_${v}_$r.log 2>&1 || exit 1
    echo $v $r $(grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/c3ab_${v}_$r.log)
  done
done
