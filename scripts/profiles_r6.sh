#!/bin/bash
# Round-6 profiles on the round's final library: rocprofv3 --kernel-trace --stats of the headline bench, the
# config-3 shard, the config-4 long tail and passive replication; then the PMC passes -- the headline's
# counters (scripts/pmc_passes.txt over tools/prof_kernel.py --calib, for profiles/traffic.json), FETCH_SIZE /
# WRITE_SIZE of config 3 and config 4, and of passive replication and config 5 (scripts/gpu_traffic_lines.sh).
# Each step under its own limit, stopping at the first failure.  The summaries are computed here afterwards
# from the merged gpurun_out (tools/traffic.py, tools/traffic_configs.py).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
stats() {  # name, command...
  local n=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6stats_$n" -o run \
    --output-format csv -- "$@" > "$R/gpurun_out/r6stats_$n.log" 2>&1)
  local rc=$?; log "stats $n rc=$rc"; [ $rc -ne 0 ] && tail -5 "$R/gpurun_out/r6stats_$n.log"; return $rc
}
pmc() {  # name, counter, command...
  local n=$1 c=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c -d "$R/gpurun_out/pmc_$n/$c" -o pmc \
    --output-format csv -- "$@" > "$R/gpurun_out/pmc_${n}_$c.log" 2>&1)
  local rc=$?; log "pmc $n $c rc=$rc"; [ $rc -ne 0 ] && tail -5 "$R/gpurun_out/pmc_${n}_$c.log"; return $rc
}
if [ -z "${NO_STATS:-}" ]; then
  stats headline python3 "$R/bench.py" --headline-only --steps 20 --warmup 3 --no-cpu-baseline || exit $?
  stats c3 python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 5 --segments || exit $?
  stats c4 python3 "$R/tools/prof_longtail.py" --native --n 2000 --thresholds 256 --reps 3 || exit $?
  stats repl python3 "$R/tools/prof_replication.py" --reps 5 || exit $?
fi
if [ -z "${NO_PMC:-}" ]; then
  NAME=r6c2 PASSES=pmc_passes.txt PASS_LIMIT=200 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_kernel.py" --calib --reps 3 \
    > gpurun_out/traffic_r6c2.txt 2>&1 || { tail -5 gpurun_out/traffic_r6c2.txt; exit 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    pmc r6c3 $c python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 1 || exit $?
    pmc r6c4 $c python3 "$R/tools/prof_longtail.py" --native --n 2000 --thresholds 256 --reps 1 || exit $?
  done
  NAME=r6repl PASSES=pmc_passes_traffic.txt PASS_LIMIT=400 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_replication.py" --reps 3 \
    > gpurun_out/traffic_r6repl.txt 2>&1 || { tail -5 gpurun_out/traffic_r6repl.txt; exit 1; }
  NAME=r6c5 PASSES=pmc_passes_traffic.txt PASS_LIMIT=500 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_config5.py" --steps 3 \
    > gpurun_out/traffic_r6c5.txt 2>&1 || { tail -5 gpurun_out/traffic_r6c5.txt; exit 1; }
fi
exit 0
