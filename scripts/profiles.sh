#!/bin/bash
# Round-2 profiles: kernel-trace stats of the headline bench, then PMC passes (one rocprofv3 run per
# pass, scripts/pmc_passes.txt) over config 2 (with the stream calibration), the config-3 mixed shard
# and the config-4 long tail.  WHICH="c2 c3 c4" selects the PMC workloads.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
cd /tmp && export TMPDIR=/tmp
if [ -z "${NO_STATS:-}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r2stats" -o run --output-format csv \
    -- python3 "$R/bench.py" --headline-only --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/r2stats.log" 2>&1
  rc=$?; log "stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
for W in ${WHICH:-c2 c3 c4}; do
  case $W in
    c2) CMD="$R/tools/prof_kernel.py --calib --reps 2";;
    c3) CMD="$R/tools/prof_kernel.py --native --wf 1250000 --reps 1";;
    c4) CMD="$R/tools/prof_longtail.py --native --n 2000 --thresholds 256 --reps 1";;
  esac
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/pmc_$W/p$i" -o pmc --output-format csv \
      -- python3 $CMD > "$R/gpurun_out/pmc_${W}_p$i.log" 2>&1
    rc=$?; log "pmc $W pass $i ($line) rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done < "$R/scripts/${PASSES:-pmc_passes.txt}"
done
exit 0
