#!/bin/bash
# parity tests, C2 A/B timing of variants, then the config-4 long-tail probe
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in ${VARIANTS:-}; do
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 7 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  rc=$?; echo "variant $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python tools/prof_longtail.py ${LT_ARGS:-} > gpurun_out/longtail.jsonl 2> gpurun_out/longtail.err
rc=$?; echo "longtail rc=$rc" >> gpurun_out/status.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/prof_longtail.py ${LT_ARGS:-} --unbounded >> gpurun_out/longtail.jsonl 2>> gpurun_out/longtail.err
rc=$?; echo "longtail-unbounded rc=$rc" >> gpurun_out/status.log
exit $rc
