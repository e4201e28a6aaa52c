#!/bin/bash
# Round-5 probe: config-4 segment split (tools/prof_c4_segments.py), then an alternating A/B of variant
# libraries on config 2 (scripts/gpu_ab.sh).  Each step under its own limit, stopping at a failure.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
if [ -z "${NO_C4:-}" ]; then
  timeout -k 10 400 python -u tools/prof_c4_segments.py ${C4ARGS:-} > gpurun_out/c4_segments.log 2>&1
  rc=$?; log "c4 segments rc=$rc"; cat gpurun_out/c4_segments.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${VARIANTS:-}" ]; then
  bash scripts/gpu_ab.sh || exit $?
fi
exit 0
