#!/bin/bash
# Round 6: instruction / wait counters of the wavefront path (config 4's big segment alone, and the 256
# longest tail runs alone) for the product library and the round-5 walk (tools/variants/r5wave.so).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for v in product r5wave; do
  L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
  for only in big tailtop; do
    NAME=walk_${v}_$only PASSES=pmc_passes_walk.txt PASS_LIMIT=120 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_c4_segments.py" --lib "$R/$L" --only $only --top 256 --reps 1 > gpurun_out/walkpmc_${v}_$only.txt 2>&1 || { tail -5 gpurun_out/walkpmc_${v}_$only.txt; exit 1; }
  done
done
