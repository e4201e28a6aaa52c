#!/bin/bash
# Round-3 session check: GPU suite + headline bench (scripts/gpu_check.sh), then the wavefront path's
# per-workflow phase records on config 4 (tools/wave_dbg.so, built by tools/instrument_wave.py).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
bash scripts/gpu_check.sh || exit $?
timeout -k 10 300 python tools/prof_longtail.py --native --n 2000 --thresholds 256 --reps 2 --lib tools/wave_dbg.so \
  > gpurun_out/wave_dbg.log 2>&1
rc=$?; log "wave dbg rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/wave_dbg.log; exit $rc; }
tail -c 3000 gpurun_out/wave_dbg.log
exit 0
