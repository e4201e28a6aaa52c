#!/bin/bash
# long-tail (config 4) timing of variant libraries, wave-tail layout only
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  timeout -k 10 300 python -u tools/prof_longtail.py --n ${LT_N:-200} --thresholds 256 --lib build/variants/lib_$v.so >> gpurun_out/lt_ab.jsonl 2>> gpurun_out/lt_ab.err
  rc=$?; echo "lt $v rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
