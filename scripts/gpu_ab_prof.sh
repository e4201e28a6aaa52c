#!/bin/bash
# A/B kernel variants + PMC counter passes (each pass its own rocprofv3 run, kernel-trace only)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
VARIANTS="${VARIANTS:-v1 v2 v2lb3}"
PROF_LIB="${PROF_LIB:-build/variants/lib_v2.so}"
for v in $VARIANTS; do
  timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_$v.so --reps 7 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err
  rc=$?; echo "variant $v rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1 || true
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/pmc$i" -o pmc --output-format csv -- python3 "$R/tools/prof_kernel.py" --lib "$R/$PROF_LIB" --reps 2 > "$R/gpurun_out/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($line) rc=$rc" >> "$R/gpurun_out/status.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done < "$R/scripts/pmc_passes.txt"
exit 0
