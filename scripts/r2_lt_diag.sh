#!/bin/bash
# Long-tail wave-path diagnosis: per-event-type cycles (CRR_EXP=128 build in build_exp/), then one PMC
# pass (instruction mix and wave cycles) over the default build.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1
timeout -k 10 300 python tools/prof_longtail.py --native --n ${LT_N:-2000} --thresholds 256 --reps 2 \
  --lib build_exp/libexp128.so > gpurun_out/lt128.log 2>&1
rc=$?; echo "lt128 rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc ${PMC_LT:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY} \
  -d "$R/gpurun_out/ltpmc" -o pmc --output-format csv \
  -- python3 "$R/tools/prof_longtail.py" --native --n ${LT_N:-2000} --thresholds 256 --reps 1 > "$R/gpurun_out/ltpmc.log" 2>&1
rc=$?; echo "ltpmc rc=$rc" >> "$R/gpurun_out/status.log"; exit $rc
