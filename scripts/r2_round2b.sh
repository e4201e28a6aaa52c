#!/bin/bash
# GPU tests, then solo kernel times (one hardware queue: every kernel alone) of the full-size mixed
# shard for the default library and the variants in LIBS, then the unprofiled config-3 / config-4
# replay times of the default library.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [ $rc -ne 0 ] && exit $rc
fi
PRE=GPU_MAX_HW_QUEUES=1 bash scripts/r2_trace_mixed.sh || exit $?
LIBS= bash scripts/r2_perf.sh
