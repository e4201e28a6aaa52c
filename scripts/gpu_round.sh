#!/bin/bash
# One GPU call: parity tests, bench (N=1), rocprof kernel-trace stats of the bench, then PMC passes
# (one rocprofv3 run per pass) over tools/prof_kernel.py --calib.  Every GPU step has its own time
# limit; the script stops at the first failing step.
#   STEPS="tests bench stats pmc" (default: all)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
STEPS="${STEPS:-tests bench stats pmc}"
log() { echo "$(date +%T) $*" | tee -a "$R/gpurun_out/status.log"; }
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }

if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; log "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if has bench; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
  rc=$?; log "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
if has stats; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof_bench.log" 2>&1
  rc=$?; log "rocprof stats rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if has pmc; then
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/pmc/p$i" -o pmc --output-format csv \
      -- python3 "$R/tools/prof_kernel.py" --calib --reps 2 > "$R/gpurun_out/pmc_p$i.log" 2>&1
    rc=$?; log "pmc pass $i ($line) rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done < "$R/scripts/pmc_passes.txt"
fi
exit 0
