#!/bin/bash
# Timing of experiment variants (build/variants/lib_<v>.so, no parity: CRR_EXP builds skip work),
# then calibrated FETCH_SIZE / WRITE_SIZE passes on PMC_LIBS.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for v in ${VARIANTS:-}; do
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 7 ${PROF_ARGS:-} >> gpurun_out/exp.jsonl 2>> gpurun_out/exp.err
  rc=$?; echo "timing $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
for v in ${PMC_LIBS:-}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/pmc_$v/$c" -o pmc --output-format csv \
      -- python3 "$R/tools/prof_kernel.py" --lib "$R/build/variants/lib_$v.so" --calib --reps 2 > "$R/gpurun_out/pmc_${v}_$c.log" 2>&1
    rc=$?; echo "pmc $v $c rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
