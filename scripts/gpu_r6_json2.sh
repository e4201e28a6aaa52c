#!/bin/bash
# Round 6: the staged one-walk JSON transcode: parity tests, then its timing and kernel stats.
set -o pipefail
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_json_ingest.py \
  > gpurun_out/pytest_json.log 2>&1 &&
timeout -k 10 300 python -u tools/prof_json.py --kind mixed --wf 125000 > gpurun_out/json_mixed.json 2> gpurun_out/json_mixed.err &&
timeout -k 10 300 python -u tools/prof_json.py --kind chain --wf 125000 > gpurun_out/json_chain.json 2> gpurun_out/json_chain.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_json2" -o json \
   --output-format csv -- python3 "$R/tools/prof_json.py" --kind mixed --wf 125000 --reps 2 > "$R/gpurun_out/json_prof2.log" 2>&1)
rc=$?
tail -3 gpurun_out/pytest_json.log
cat gpurun_out/json_mixed.json gpurun_out/json_chain.json
exit $rc
