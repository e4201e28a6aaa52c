#!/bin/bash
# Round 5: config-4 A/B of library variants (VARIANTS: names under tools/variants, "product" = the in-tree
# library), alternated on one box; then the parity tests (wave path included) and a wave profile.
set -u
VARIANTS=${VARIANTS:-"base16 product"}
for r in 1 2 3; do
  for v in $VARIANTS; do
    L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
    timeout -k 10 300 python -u tools/prof_c4_segments.py --lib $L --only all,tailtop --top 256 --reps 3 > gpurun_out/c4ab_${v}_$r.log 2>&1 || exit 1
    echo $v $r $(grep -o "\"run\": \"[a-z]*\", \"group_ms\": \[[^]]*\]" gpurun_out/c4ab_${v}_$r.log)
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resume.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_c4ab.log 2>&1 || { tail -5 gpurun_out/pytest_c4ab.log; exit 1; }
tail -2 gpurun_out/pytest_c4ab.log
if [ -f tools/variants/waveprof.so ]; then
  timeout -k 10 300 python -u tools/prof_c4_segments.py --lib tools/variants/waveprof.so --only tailtop --top 256 --wave-prof > gpurun_out/c4_waveprof4.log 2>&1 || exit 1
  tail -1 gpurun_out/c4_waveprof4.log | cut -c1-2500
fi
