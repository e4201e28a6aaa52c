#!/bin/bash
# Probes: device-ingest kernel split (rocprofv3 kernel trace) and the wavefront path's per-workflow
# records (tools/wave_dbg.so, built by tools/instrument_wave.py).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ingest_prof" -o run --output-format csv \
  -- python3 "$R/tools/prof_ingest.py" --kind chain > "$R/gpurun_out/ingest_chain.log" 2>&1
rc=$?; log "ingest chain rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$R/gpurun_out/ingest_chain.log"; exit $rc; }
grep ingest_events "$R/gpurun_out/ingest_chain.log"
cd "$R"
timeout -k 10 300 python tools/prof_longtail.py --native --n 2000 --thresholds 256 --reps 2 --lib tools/wave_dbg.so \
  > gpurun_out/wave_dbg.log 2>&1
rc=$?; log "wave dbg rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/wave_dbg.log; exit $rc; }
cat gpurun_out/wave_dbg.log | tail -c 3000
exit 0
