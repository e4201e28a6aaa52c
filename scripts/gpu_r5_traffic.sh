#!/bin/bash
# Round-5 PMC passes: the headline (config 2, tools/prof_kernel.py --calib: FETCH / WRITE, LDS bank conflicts,
# VALU counters -> profiles/traffic.json via tools/traffic.py), the config-5 lines (rebuild, ndc_prepare,
# checksum_verify) and the access-width calibration kernels (tools/calib.py, row-field gathers included).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
NAME=c2 PASSES=pmc_passes.txt PASS_LIMIT=200 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_kernel.py" --calib --reps 3 > gpurun_out/traffic_c2.txt 2>&1 || { tail -5 gpurun_out/traffic_c2.txt; exit 1; }
NAME=c5 PASSES=pmc_passes_traffic.txt PASS_LIMIT=500 bash scripts/gpu_pmc.sh python3 "$R/tools/prof_config5.py" --steps 3 > gpurun_out/traffic_c5.txt 2>&1 || { tail -5 gpurun_out/traffic_c5.txt; exit 1; }
NAME=calib PASSES=pmc_passes_traffic.txt PASS_LIMIT=200 bash scripts/gpu_pmc.sh python3 "$R/tools/calib.py" --mib 1024 --reps 2 > gpurun_out/traffic_calib.txt 2>&1 || { tail -5 gpurun_out/traffic_calib.txt; exit 1; }
tail -3 gpurun_out/traffic_c2.txt
exit 0
