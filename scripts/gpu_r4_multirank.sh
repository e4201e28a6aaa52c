#!/bin/bash
# The bench's N > 1 code path on one GPU: two ranks (torchrun, gloo for the collective) sharing device 0,
# each replaying its history shards of one 2M-workflow config-2 workload; then N = 1 over the same 2M
# workload.  The reduced digests must be equal (shard split, per-step exchange, max-over-ranks timing).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --headline-only --backend gloo --device 0 --steps 10 --warmup 2 \
  --no-cpu-baseline > gpurun_out/multirank_n2.json 2> gpurun_out/multirank_n2.err
rc=$?; log "n2 rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/multirank_n2.err; exit $rc; }
timeout -k 10 300 python -u bench.py --headline-only --workflows 2000000 --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/multirank_n1.json 2> gpurun_out/multirank_n1.err
rc=$?; log "n1 rc=$rc"; [ $rc -ne 0 ] && { tail -30 gpurun_out/multirank_n1.err; exit $rc; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/multirank_n2.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/multirank_n1.json").read().strip().splitlines()[-1])
print(json.dumps({"n2_digest": a["digest"], "n1_digest": b["digest"], "equal": a["digest"] == b["digest"],
                  "n2_value": a["value"], "n2_ms_per_step": a["ms_per_step"], "n2_parallelism": a["config"]["parallelism"],
                  "n1_value": b["value"], "n1_ms_per_step": b["ms_per_step"]}))
PY
