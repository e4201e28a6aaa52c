#!/bin/bash
# Round 6: JSON-encoded blobs on the device (crr_ingest_transcode_*): the parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_json_ingest.py \
  > gpurun_out/pytest_json.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_json.log
exit $rc
