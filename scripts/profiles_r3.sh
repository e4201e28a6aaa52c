#!/bin/bash
# Round-3 profiles: rocprofv3 kernel-trace stats of the headline bench, of the config-3 shard and of the
# config-4 long tail; the device-ingest kernels (config-2 chains, config-3 mixed); then PMC passes
# (scripts/${PASSES:-pmc_passes.txt}, one rocprofv3 run each) over the config-3 shard.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
cd /tmp && export TMPDIR=/tmp
stats() {  # name, command...
  local n=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3stats_$n" -o run --output-format csv \
    -- "$@" > "$R/gpurun_out/r3stats_$n.log" 2>&1
  local rc=$?; log "stats $n rc=$rc"; return $rc
}
if [ -z "${NO_STATS:-}" ]; then
  stats headline python3 "$R/bench.py" --headline-only --steps 20 --warmup 3 --no-cpu-baseline || exit $?
  stats c3 python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 5 --segments || exit $?
  stats c4 python3 "$R/tools/prof_longtail.py" --native --n 2000 --thresholds 256 --reps 3 || exit $?
  stats ingest_chain python3 "$R/tools/prof_ingest.py" --kind chain || exit $?
  stats ingest_mixed python3 "$R/tools/prof_ingest.py" --kind mixed || exit $?
fi
if [ -z "${NO_PMC:-}" ]; then
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/pmc_c3/p$i" -o pmc --output-format csv \
      -- python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 1 > "$R/gpurun_out/pmc_c3_p$i.log" 2>&1
    rc=$?; log "pmc c3 pass $i ($line) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_c3_p$i.log"; exit $rc; }
  done < "$R/scripts/${PASSES:-pmc_passes.txt}"
fi
exit 0
