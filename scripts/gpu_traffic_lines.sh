#!/bin/bash
# PMC HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, one pass each) of the passive-replication and config-5 lines
# at the bench's sizes -> gpurun_out/pmc_{repl,c5}; the summaries go to profiles/traffic_configs.json (bench.py's
# config_traffic reads it) -- rerun the python part here on the merged gpurun_out to keep them.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
NAME=repl PASSES=pmc_passes_traffic.txt PASS_LIMIT=400 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_replication.py" --reps 3 > gpurun_out/traffic_repl.txt 2>&1 || { tail -5 gpurun_out/traffic_repl.txt; exit 1; }
NAME=c5 PASSES=pmc_passes_traffic.txt PASS_LIMIT=500 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_config5.py" --steps 3 > gpurun_out/traffic_c5.txt 2>&1 || { tail -5 gpurun_out/traffic_c5.txt; exit 1; }
python3 - <<'PY'
import json, subprocess
def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
r = last_json("gpurun_out/pmc_repl_p1.log")
# the resume step's kernels: the probe's one-shot and prefix replays are the fresh compact instantiations
subprocess.run(["python3", "tools/traffic_configs.py", "passive_replication", "gpurun_out/pmc_repl",
                "--exclude", "<false, false>", "--workflows", str(r["workflows"]), "--events", str(r["events"])], check=True)
c = last_json("gpurun_out/pmc_c5_p1.log")
for name, pref in (("config5_rebuild", "replay_"), ("config5_ndc_prepare", "ndc_prepare"),
                   ("config5_checksum_verify", "checksum_kernel")):
    subprocess.run(["python3", "tools/traffic_configs.py", name, "gpurun_out/pmc_c5", "--kernels", pref,
                    "--workflows", str(c[name]["workflows"]), "--events", str(c[name]["events"])], check=True)
PY
