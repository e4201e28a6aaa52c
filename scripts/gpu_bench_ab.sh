#!/bin/bash
# A/B of whole-step time: bench.py through build/variants/lib_${PREV:-prev}.so and the in-tree library, alternated
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for i in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export CRR_LIB_PATH="$R/build/variants/lib_${PREV:-prev}.so"; else unset CRR_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --steps ${STEPS:-100} --no-cpu-baseline > gpurun_out/ab_${v}_${i}.tmp 2>&1
    rc=$?; echo "bench $v $i rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
    echo "{\"lib\": \"$v\", \"line\": $(tail -1 gpurun_out/ab_${v}_${i}.tmp)}" >> gpurun_out/bench_ab.jsonl
  done
done
exit 0
