#!/bin/bash
# Config-3 HBM traffic attribution: one FETCH_SIZE pass per library variant (product, compact tiers without
# ActivityTaskStarted's re-read of its scheduled event, finalize without re-reading the scheduled / started
# events), tools/prof_kernel.py --native at the bench's shard size.  Each pass under its own limit.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-product noreread2 nofinread}; do
  L="$R/cadence_amd/libcadence_replay.so"; [ "$v" != product ] && L="$R/tools/variants/$v.so"
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$R/gpurun_out/c3attr_$v" -o pmc --output-format csv \
    -- python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 1 --lib "$L" > "$R/gpurun_out/c3attr_$v.log" 2>&1
  rc=$?; echo "$(date +%T) c3attr $v rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/c3attr_$v.log"; exit $rc; }
done
exit 0
