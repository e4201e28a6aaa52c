#!/bin/bash
# PMC passes (scripts/pmc_passes.txt, one rocprofv3 run each) over the config-4 long tail with the
# library named by LIB (default: the product build).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
L="$R/${LIB:-cadence_amd/libcadence_replay.so}"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/${OUT:-pmc_c4}/p$i" -o pmc --output-format csv \
    -- python3 "$R/tools/prof_longtail.py" --native --n 2000 --thresholds 256 --reps 1 --lib "$L" > "$R/gpurun_out/${OUT:-pmc_c4}_p$i.log" 2>&1
  rc=$?; log "pmc c4 pass $i ($line) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/${OUT:-pmc_c4}_p$i.log"; exit $rc; }
done < "$R/scripts/${PASSES:-pmc_passes.txt}"
exit 0
