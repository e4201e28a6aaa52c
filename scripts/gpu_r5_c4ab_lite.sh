#!/bin/bash
# config-4 A/B (whole group and the 256 longest runs), alternated, no tests
set -u
for r in 1 2 3; do
  for v in ${VARIANTS:-product}; do
    L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
    timeout -k 10 300 python -u tools/prof_c4_segments.py --lib $L --only all,tailtop --top 256 --reps 3 > gpurun_out/c4l_${v}_$r.log 2>&1 || exit 1
    echo $v $r $(grep -o "\"run\": \"[a-z]*\", \"group_ms\": \[[^]]*\]" gpurun_out/c4l_${v}_$r.log)
  done
done
