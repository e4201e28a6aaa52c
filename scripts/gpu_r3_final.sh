#!/bin/bash
# Round-3 evidence: the whole GPU suite, then the full bench line (driver contract, every config).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
NO_BENCH=1 bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_bench.sh || exit $?
exit 0
