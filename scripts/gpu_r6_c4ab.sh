#!/bin/bash
# Round 6: the wave-path GPU tests, then a config-4 A/B of library variants (VARIANTS: names under
# tools/variants, "product" = the in-tree library), alternated on one box: the whole launch group, the
# big segment alone and the 256 longest tail runs alone.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-c4ab}
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_kats.py tests/test_tasks.py tests/test_gpu_pipeline.py} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
fi
VARIANTS=${VARIANTS:-"r5wave product"}
for r in 1 2; do
  for v in $VARIANTS; do
    L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
    timeout -k 10 300 python -u tools/prof_c4_segments.py --lib $L --only all,big,tailtop --top 256 --reps 3 > gpurun_out/${TAG}_${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_$r.log; exit 1; }
    echo $v $r $(grep -o "\"run\": \"[a-z]*\", \"group_ms\": \[[^]]*\]" gpurun_out/${TAG}_${v}_$r.log)
  done
done
