#!/bin/bash
# Round 5, last A/B: phase 0 without the long-tail kernels (CRR_IN_NEW_RUN_LANES) against the previous
# library, the wave minimum's scalar threshold (CRR_WAVE_MIN_SCALAR 4 / 8), after the parity tests.
set -u
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_last.log 2>&1 || { tail -8 gpurun_out/pytest_last.log; exit 1; }
tail -2 gpurun_out/pytest_last.log
for v in product prephase0 product prephase0; do
  L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
  timeout -k 10 300 python -u tools/prof_c4_phases.py --reps 10 --lib $L > gpurun_out/phases_$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"median_ms\": {[^}]*}" gpurun_out/phases_$v.log)
done
VARIANTS="product wmin4 wmin8" bash scripts/gpu_r5_c4ab_lite.sh
