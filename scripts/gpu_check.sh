#!/bin/bash
# GPU parity tests of the in-tree library, kernel timing of config 2 and of the mixed workload,
# then kernel timing of build/variants/lib_<v>.so ($VARIANTS)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/prof_kernel.py --reps 7 >> gpurun_out/check.jsonl 2>> gpurun_out/check.err
rc=$?; echo "config2 timing rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/prof_kernel.py --mixed --wf ${MIXED_WF:-200000} --reps 5 >> gpurun_out/check.jsonl 2>> gpurun_out/check.err
rc=$?; echo "mixed timing rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
if [ -n "${LT_N:-}" ]; then
  timeout -k 10 400 python -u tools/prof_longtail.py --n $LT_N --thresholds 256 >> gpurun_out/check_lt.jsonl 2>> gpurun_out/check.err
  rc=$?; echo "longtail timing rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
bash scripts/gpu_exp.sh
