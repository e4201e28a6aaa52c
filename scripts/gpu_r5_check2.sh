#!/bin/bash
# Round 5: the digest pointers read late (kernel-argument segment), the host-placed resumed workflows:
# digest + resume + pipeline GPU tests first, then config-2 digest on/off, passive replication, config 3.
set -u
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_resume.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_check2.log 2>&1 || { tail -8 gpurun_out/pytest_check2.log; exit 1; }
tail -2 gpurun_out/pytest_check2.log
for r in 1 2 3; do
  for x in "" --digest; do
    timeout -k 10 300 python -u tools/prof_kernel.py --reps 10 $x > gpurun_out/c2d_${r}${x}.log 2>&1 || exit 1
    echo c2 $r "$x" $(grep -o "\"median_ms\": [0-9.]*" gpurun_out/c2d_${r}${x}.log)
  done
done
timeout -k 10 300 python -u tools/prof_replication.py --reps 5 > gpurun_out/repl_check2.log 2>&1 || { tail -5 gpurun_out/repl_check2.log; exit 1; }
tail -2 gpurun_out/repl_check2.log | cut -c1-600
timeout -k 10 300 python -u tools/prof_kernel.py --native --wf 1250000 --reps 5 > gpurun_out/c3_check2.log 2>&1 || exit 1
grep -o "\"kernel_ms\": \[[^]]*\]" gpurun_out/c3_check2.log
