#!/bin/bash
# Device-ingest tests, then its kernel split under rocprofv3 (one config-2 chunk and one config-3 chunk).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_ingest.log 2>&1
rc=$?; log "ingest tests rc=$rc"; tail -4 gpurun_out/pytest_ingest.log; [ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_ingest.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp
for K in chain mixed; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ingest_prof_$K" -o run --output-format csv \
    -- python3 "$R/tools/prof_ingest.py" --kind $K > "$R/gpurun_out/ingest_$K.log" 2>&1
  rc=$?; log "ingest $K rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$R/gpurun_out/ingest_$K.log"; exit $rc; }
  grep ingest_events "$R/gpurun_out/ingest_$K.log"
done
exit 0
