#!/bin/bash
# Round 6: passive replication from the tasks' blobs (device resume ingest + replay): step wall time and the
# rocprofv3 kernel stats of the same run (config-3 shard, 1.25M workflows).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out/blobrepl
timeout -k 10 300 python -u tools/prof_replication.py --blobs --reps 5 > gpurun_out/blobrepl/plain.log 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/blobrepl/prof" -o run \
  --output-format csv -- python3 "$R/tools/prof_replication.py" --blobs --reps 5 > "$R/gpurun_out/blobrepl/prof.log" 2>&1) || exit 1
