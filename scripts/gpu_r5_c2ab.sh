#!/bin/bash
# Round 5: config-2 kernel A/B (tools/prof_kernel.py, 1M x 29): the in-tree library with and without the
# fused digest, and variant libraries (VARIANTS under tools/variants), alternated; then the resume tests.
set -u
for r in 1 2 3; do
  for v in product product_digest ${VARIANTS:-}; do
    L=cadence_amd/libcadence_replay.so; X=""
    case $v in product) ;; product_digest) X=--digest ;; *) L=tools/variants/$v.so; X=--digest ;; esac
    timeout -k 10 300 python -u tools/prof_kernel.py --lib $L --reps 10 $X > gpurun_out/c2ab_${v}_$r.log 2>&1 || exit 1
    echo $v $r $(grep -o "\"median_ms\": [0-9.]*" gpurun_out/c2ab_${v}_$r.log)
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_resume.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_resume_r5.log 2>&1 || { tail -5 gpurun_out/pytest_resume_r5.log; exit 1; }
tail -2 gpurun_out/pytest_resume_r5.log
