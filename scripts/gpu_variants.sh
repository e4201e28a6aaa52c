#!/bin/bash
# for each variant library: GPU parity tests through it, then kernel-only timing
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for v in ${VARIANTS:-}; do
  CRR_LIB_PATH="$R/build/variants/lib_$v.so" timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 7 ${PROF_ARGS:-} >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  rc=$?; echo "timing $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 5 --mixed --wf 200000 >> gpurun_out/ab_mixed.jsonl 2>> gpurun_out/ab.err
  rc=$?; echo "timing-mixed $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
