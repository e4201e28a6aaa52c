#!/bin/bash
# Round 6: the bench's N > 1 path on one GPU, every line: two ranks (torchrun, gloo for the collectives)
# sharing device 0, each replaying its history shards of one workload (config 2: 2 x 400k, config 3: 2 x 300k,
# config 5: 2 x 200k), then N = 1 over the same workloads.  The reduced digests of configs 2, 3 and 5 must be
# equal (shard split, fused digest, per-step all-reduce).  Config 4's keys are rank-qualified (its runs share
# workflow IDs), so its digest is compared by counts only.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
A="--steps 5 --warmup 1 --config-steps 3 --no-cpu-baseline --no-e2e --c4-workflows 200"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --device 0 --workflows 400000 --c3-workflows 300000 \
  --c5-workflows 200000 $A > gpurun_out/multirank6_n2.json 2> gpurun_out/multirank6_n2.err || { tail -30 gpurun_out/multirank6_n2.err; exit 1; }
timeout -k 10 900 python -u bench.py --workflows 800000 --c3-workflows 600000 --c5-workflows 400000 $A \
  --c4-workflows 400 > gpurun_out/multirank6_n1.json 2> gpurun_out/multirank6_n1.err || { tail -30 gpurun_out/multirank6_n1.err; exit 1; }
python3 - <<'PY'
import json
a = json.loads(open("gpurun_out/multirank6_n2.json").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/multirank6_n1.json").read().strip().splitlines()[-1])
out = {"config2": {"n2": a["digest"], "n1": b["digest"], "equal": a["digest"] == b["digest"]}}
for k, path in (("config3", ("configs", "config3_mixed", "digest", "digest")),
                ("config5", ("configs", "config5_ndc", "rebuild", "digest", "digest"))):
    x, y = a, b
    for p in path:
        x, y = x[p], y[p]
    out[k] = {"n2": x, "n1": y, "equal": x == y}
c4a, c4b = a["configs"]["config4_long_tail"]["digest"]["digest"], b["configs"]["config4_long_tail"]["digest"]["digest"]
out["config4_counts"] = {"n2": c4a[:3] + [c4a[5]], "n1": c4b[:3] + [c4b[5]], "equal": c4a[:3] + [c4a[5]] == c4b[:3] + [c4b[5]]}
out["host_digest_checks"] = {"n2": [a["configs"]["config3_mixed"]["digest"]["matches_host_digest"],
                                    a["configs"]["config5_ndc"]["rebuild"]["digest"]["matches_host_digest"]]}
print(json.dumps(out))
PY
