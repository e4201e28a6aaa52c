#!/bin/bash
# Round 5: the digest's cost on config 2's kernel (tools/prof_kernel.py, 1M x 29): the in-tree library
# with and without the digest, and the variants (with it), alternated.
set -u
for r in 1 2 3; do
  for v in product product_digest ${VARIANTS:-}; do
    L=cadence_amd/libcadence_replay.so; X=""
    case $v in product) ;; product_digest) X=--digest ;; *) L=tools/variants/$v.so; X=--digest ;; esac
    timeout -k 10 300 python -u tools/prof_kernel.py --lib $L --reps 10 $X > gpurun_out/c2dig_${v}_$r.log 2>&1 || exit 1
    echo $v $r $(grep -o "\"median_ms\": [0-9.]*" gpurun_out/c2dig_${v}_$r.log)
  done
done
