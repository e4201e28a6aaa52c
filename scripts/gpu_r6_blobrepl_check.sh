#!/bin/bash
# Round 6: the resume-ingest tests, then the blob replication step's time and kernel stats (scripts/gpu_r6_blobrepl.sh)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resume.py \
  tests/test_gpu_ingest.py > gpurun_out/r6_blobrepl.log 2>&1 || { tail -30 gpurun_out/r6_blobrepl.log; exit 1; }
tail -2 gpurun_out/r6_blobrepl.log
bash scripts/gpu_r6_blobrepl.sh
