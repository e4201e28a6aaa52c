#!/bin/bash
# Round 6: the GPU suite, then config 4 with the tail kernel's work list at several grid sizes
# (CRR_TAIL_WAVES_PER_SIMD, read per call by crr_replay; 0 = one wavefront per run, the round-5 grid),
# alternated on one box: the whole launch group and the 256 longest tail runs alone.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-tg}
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
fi
for r in 1 2; do
  for v in ${GRIDS:-0 1 2 3}; do
    CRR_TAIL_WAVES_PER_SIMD=$v timeout -k 10 300 python -u tools/prof_c4_segments.py --only ${ONLY:-all,tailtop} --top 256 --reps 3 > gpurun_out/${TAG}_w${v}_$r.log 2>&1 || { tail -5 gpurun_out/${TAG}_w${v}_$r.log; exit 1; }
    echo w$v $r $(grep -o "\"run\": \"[a-z]*\", \"group_ms\": \[[^]]*\]" gpurun_out/${TAG}_w${v}_$r.log)
  done
done
