#!/bin/bash
# Round 6: device JSON ingest timing (config-3 shard shape and config-2 chains, 125k workflows each) and
# its rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/prof_json.py --kind mixed --wf 125000 > gpurun_out/json_mixed.json 2> gpurun_out/json_mixed.err &&
timeout -k 10 300 python -u tools/prof_json.py --kind chain --wf 125000 > gpurun_out/json_chain.json 2> gpurun_out/json_chain.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_json -o json -- python3 tools/prof_json.py --kind mixed --wf 125000 --reps 2 > gpurun_out/json_prof.log 2>&1
rc=$?
cat gpurun_out/json_mixed.json gpurun_out/json_chain.json
find gpurun_out/prof_json -name "*kernel_stats.csv" | head -3
exit $rc
