#!/bin/bash
# Config-2 headline A/B: bench.py --headline-only with each library in LIBS (path or "default"),
# alternated ROUNDS times on one box.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for L in ${LIBS:-default}; do
    b=$(basename $L .so)
    if [ "$L" = "default" ]; then unset CRR_LIB_PATH; else export CRR_LIB_PATH="$R/$L"; fi
    timeout -k 10 200 python bench.py --headline-only --steps 20 --warmup 3 --no-cpu-baseline >> gpurun_out/c2ab_$b.log 2>&1
    rc=$?; echo "c2ab $b round $r rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
