#!/bin/bash
# Round 6 final pass: the JSON device-ingest tests, then the full bench line (default arguments).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_json_ingest.py \
  > gpurun_out/pytest_json.log 2>&1 &&
timeout -k 10 1000 python -u bench.py > gpurun_out/bench_full_r6f.json 2> gpurun_out/bench_full_r6f.err
rc=$?
tail -3 gpurun_out/pytest_json.log
tail -c 2500 gpurun_out/bench_full_r6f.json
exit $rc
