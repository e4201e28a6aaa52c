#!/bin/bash
# The full bench line (driver contract), then the rocprofv3 kernel-trace stats of the headline.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
timeout -k 10 1000 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; log "bench rc=$rc"; tail -5 gpurun_out/bench_full.err; [ $rc -ne 0 ] && exit $rc
tail -c 3000 gpurun_out/bench_full.json
exit 0
