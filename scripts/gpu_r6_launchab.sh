#!/bin/bash
# Round 6: launch-order A/B (VARIANTS: libraries under tools/variants built from capi.hip with -DCRR_SMALL_FIRST=...,
# "product" = the in-tree library), alternated on one box: the config-3 shard (with its segment finish times),
# passive replication and config 4.  Ship the variants with scripts/gpurun_with_variants.sh.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-lab}
for r in 1 2 3; do
  for v in product ${VARIANTS:-sf1 sf3}; do
    L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
    timeout -k 10 300 python -u tools/prof_kernel.py --native --wf 1250000 --reps 5 --segments --lib $L > gpurun_out/${TAG}_c3_${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_c3_${v}_$r.log; exit 1; }
    echo c3 $v $r $(grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/${TAG}_c3_${v}_$r.log)
    if [ -z "${C3_ONLY:-}" ]; then
    timeout -k 10 300 python -u tools/prof_replication.py --reps 5 --lib $L > gpurun_out/${TAG}_repl_${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_repl_${v}_$r.log; exit 1; }
    echo repl $v $r $(grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/${TAG}_repl_${v}_$r.log | tail -1)
    timeout -k 10 300 python -u tools/prof_c4_segments.py --lib $L --only all --reps 3 > gpurun_out/${TAG}_c4_${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_c4_${v}_$r.log; exit 1; }
    echo c4 $v $r $(grep -o "\"group_ms\": \[[^]]*\]" gpurun_out/${TAG}_c4_${v}_$r.log)
    fi
  done
done
