#!/bin/bash
# Round 5: the big-before-tail gate -- 30 whole-group config-4 launches of the in-tree library (none should
# take the ~9.4-ms path), A/B against the ungated variant, the GPU suites that cover the wave path, resume
# and tiers, then the wave-path profile with sub-buckets.
set -u
for r in 1 2 3; do
  for v in product sidepfnohbm; do
    L=cadence_amd/libcadence_replay.so; [ $v != product ] && L=tools/variants/$v.so
    timeout -k 10 300 python -u tools/prof_c4_segments.py --lib $L --only all,tailtop --top 256 --reps 10 > gpurun_out/gate_${v}_$r.log 2>&1 || exit 1
    echo $v $r $(grep -o "\"run\": \"[a-z]*\", \"group_ms\": \[[^]]*\]" gpurun_out/gate_${v}_$r.log)
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resume.py tests/test_gpu_pipeline.py tests/test_tasks.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gate.log 2>&1 || { tail -5 gpurun_out/pytest_gate.log; exit 1; }
tail -2 gpurun_out/pytest_gate.log
[ -n "${WAVEPROF:-}" ] || exit 0
timeout -k 10 300 python -u tools/prof_c4_segments.py --lib tools/variants/waveprof.so --only tailtop --top 256 --wave-prof > gpurun_out/c4_waveprof5.log 2>&1 || exit 1
tail -1 gpurun_out/c4_waveprof5.log | cut -c1-3500
timeout -k 10 300 python -u tools/prof_c4_segments.py --lib tools/variants/waveprof.so --only big --wave-prof > gpurun_out/c4_waveprof5_big.log 2>&1 || exit 1
tail -1 gpurun_out/c4_waveprof5_big.log | cut -c1-3500
