#!/bin/bash
# rocprofv3 kernel-trace stats of one command: NAME=<tag> bash scripts/gpu_stats.sh python3 <script> [args]
# -> gpurun_out/stats_<tag>/ (kernel stats + trace csv) and the top kernels on stdout.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
N="${NAME:-run}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/stats_$N" -o run --output-format csv \
  -- "$@" > "$R/gpurun_out/stats_$N.log" 2>&1
rc=$?; echo "$(date +%T) stats $N rc=$rc" >> "$R/gpurun_out/status.log"
[ $rc -ne 0 ] && { tail -20 "$R/gpurun_out/stats_$N.log"; exit $rc; }
cd "$R"
python3 tools/kstats.py "$(dirname "$(ls gpurun_out/stats_$N/*/*kernel_stats.csv gpurun_out/stats_$N/*kernel_stats.csv 2>/dev/null | head -1)")" 14
exit 0
