#!/bin/bash
# Round-3 check: the whole GPU suite; the device-ingest kernel split (config-2 / config-3 chunks); config-3
# and config-4 kernel times; the config-3 HBM traffic (FETCH_SIZE / WRITE_SIZE passes per kernel).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?; log "pytest rc=$rc"; tail -3 gpurun_out/pytest_all.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/pytest_all.log | head -30; exit $rc; }
timeout -k 10 300 python tools/prof_kernel.py --native --wf 1250000 --reps 5 > gpurun_out/perf_c3.log 2>&1
rc=$?; log "c3 rc=$rc"; tail -c 600 gpurun_out/perf_c3.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for K in chain mixed; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ingest_prof_$K" -o run --output-format csv \
    -- python3 "$R/tools/prof_ingest.py" --kind $K > "$R/gpurun_out/ingest_$K.log" 2>&1
  rc=$?; log "ingest $K rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$R/gpurun_out/ingest_$K.log"; exit $rc; }
  grep ingest_events "$R/gpurun_out/ingest_$K.log"
done
i=0
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/pmc_c3/p$i" -o pmc --output-format csv \
    -- python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 1 > "$R/gpurun_out/pmc_c3_p$i.log" 2>&1
  rc=$?; log "pmc c3 $C rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_c3_p$i.log"; exit $rc; }
done
exit 0
