#!/bin/bash
# kernel-only timing of variant libraries (no parity), then PMC passes on PROF_LIB
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
for v in ${VARIANTS:-}; do
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 7 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  rc=$?; echo "timing $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
[ -z "${PROF_LIB:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/pmc$i" -o pmc --output-format csv -- python3 "$R/tools/prof_kernel.py" --lib "$R/$PROF_LIB" --reps 2 > "$R/gpurun_out/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc" >> "$R/gpurun_out/status.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < "$R/scripts/pmc_passes.txt"
exit 0
