#!/bin/bash
# Round 5: NDC stage-size A/B (product = 512 items), the NDC GPU tests, the 2-rank-on-one-GPU digest check.
set -u
for v in product ndc384 ndc256 ndc384b128 product ndc384 ndc256 ndc384b128; do
  L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
  timeout -k 10 300 python -u tools/prof_ndc.py --lib $L > gpurun_out/ndc2_$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"median_ms\": [0-9.]*\|bit_exact_sample\": [a-z]*" gpurun_out/ndc2_$v.log)
done
timeout -k 10 600 python -u -m pytest tests/test_ndc.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ndc.log 2>&1 || { tail -5 gpurun_out/pytest_ndc.log; exit 1; }
tail -2 gpurun_out/pytest_ndc.log
bash scripts/gpu_r4_multirank.sh || exit 1
# config-3 time of the two re-read removals (results wrong by design; time only)
for v in product noreread2 nofinread product noreread2 nofinread; do
  L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
  timeout -k 10 300 python -u tools/prof_kernel.py --native --wf 1250000 --reps 5 --lib $L > gpurun_out/c3t_$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/c3t_$v.log)
done
