#!/bin/bash
# Round-5 profiles: rocprofv3 kernel-trace stats of the headline bench, the config-3 shard, the config-4
# long tail, passive replication and the device ingest (config-2 chains, config-3 mixed); then the HBM
# traffic passes (FETCH_SIZE, WRITE_SIZE) of config 3 and config 4 at the bench's sizes (the replication
# and config-5 ones: scripts/gpu_traffic_lines.sh).  Each step under its own limit, stopping at a failure.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
cd /tmp && export TMPDIR=/tmp
stats() {  # name, command...
  local n=$1; shift
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5stats_$n" -o run --output-format csv \
    -- "$@" > "$R/gpurun_out/r5stats_$n.log" 2>&1
  local rc=$?; log "stats $n rc=$rc"; return $rc
}
pmc() {  # name, counter, command...
  local n=$1 c=$2; shift 2
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/pmc_$n/$c" -o pmc --output-format csv \
    -- "$@" > "$R/gpurun_out/pmc_${n}_$c.log" 2>&1
  local rc=$?; log "pmc $n $c rc=$rc"; [ $rc -ne 0 ] && tail -5 "$R/gpurun_out/pmc_${n}_$c.log"; return $rc
}
if [ -z "${NO_STATS:-}" ]; then
  stats headline python3 "$R/bench.py" --headline-only --steps 20 --warmup 3 --no-cpu-baseline || exit $?
  stats c3 python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 5 --segments || exit $?
  stats c4 python3 "$R/tools/prof_longtail.py" --native --n 2000 --thresholds 256 --reps 3 || exit $?
  stats repl python3 "$R/tools/prof_replication.py" --reps 5 || exit $?
  stats ingest_chain python3 "$R/tools/prof_ingest.py" --kind chain || exit $?
  stats ingest_mixed python3 "$R/tools/prof_ingest.py" --kind mixed || exit $?
fi
if [ -z "${NO_PMC:-}" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    pmc r5c3 $c python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 1 || exit $?
    pmc r5c4 $c python3 "$R/tools/prof_longtail.py" --native --n 2000 --thresholds 256 --reps 1 || exit $?
  done
fi
exit 0
