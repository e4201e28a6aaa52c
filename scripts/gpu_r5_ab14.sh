#!/bin/bash
# Round 5 A/B batch: NDC staging variants, config-4 launch order, parity, config-3 attribution, wave profile.
# Every GPU step under its own time limit; stops at the first failure.
set -u
for v in product ndcold ndc512 product ndcold ndc512; do
  L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
  timeout -k 10 300 python -u tools/prof_ndc.py --lib $L > gpurun_out/ndc_$v.log 2>&1 || exit 1
  echo $v $(grep -o "\"median_ms\": [0-9.]*\|bit_exact_sample\": [a-z]*" gpurun_out/ndc_$v.log)
done
for r in 1 2 3; do
  timeout -k 10 300 python -u tools/prof_c4_segments.py --only all --reps 5 > gpurun_out/c4_order_$r.log 2>&1 || exit 1
  grep -o "\"run\": \"[a-z]*\", \"group_ms\": \[[^]]*\]" gpurun_out/c4_order_$r.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_order.log 2>&1 || { tail -5 gpurun_out/pytest_order.log; exit 1; }
tail -2 gpurun_out/pytest_order.log
bash scripts/gpu_r5_c3attr.sh || exit 1
timeout -k 10 300 python -u tools/prof_c4_segments.py --lib tools/variants/waveprof.so --only tailtop --top 256 --wave-prof > gpurun_out/c4_waveprof3.log 2>&1 || exit 1
tail -1 gpurun_out/c4_waveprof3.log | cut -c1-2500
