#!/bin/bash
# kernel-only timing (config 2) of the in-tree library, then build/variants/lib_<v>.so ($VARIANTS), then in-tree again
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_kernel.py --reps 7 >> gpurun_out/tv.jsonl 2>> gpurun_out/tv.err || exit $?
for v in ${VARIANTS:-}; do
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 7 >> gpurun_out/tv.jsonl 2>> gpurun_out/tv.err
  rc=$?; echo "timing $v rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/prof_kernel.py --reps 7 >> gpurun_out/tv.jsonl 2>> gpurun_out/tv.err
