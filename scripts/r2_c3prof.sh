#!/bin/bash
# Config-3 shard profiles of the current build: rocprofv3 kernel-trace stats (kernels serialised by the
# profiler: per-kernel times, not the concurrent launch group), then the PMC passes.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/c3stats" -o run --output-format csv \
  -- python3 "$R/tools/prof_kernel.py" --native --wf 1250000 --reps 3 > "$R/gpurun_out/c3stats.log" 2>&1
rc=$?; echo "c3 stats rc=$rc" >> "$R/gpurun_out/status.log"; [ $rc -ne 0 ] && exit $rc
cd "$R" && NO_STATS=1 WHICH=c3 bash scripts/r2_profiles.sh
