#!/bin/bash
# rocprofv3 PMC passes (one run per line of scripts/${PASSES:-pmc_passes.txt}) over one command:
#   NAME=<tag> bash scripts/gpu_pmc.sh python3 /root/repo/tools/<script> [args]
# -> gpurun_out/pmc_<tag>/p<i>/ ; then the per-kernel report (tools/pmc_report.py).
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
N="${NAME:-run}"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL ${PASS_LIMIT:-200} rocprofv3 --kernel-trace --pmc $line -d "$R/gpurun_out/pmc_$N/p$i" -o pmc \
    --output-format csv -- "$@" > "$R/gpurun_out/pmc_${N}_p$i.log" 2>&1
  rc=$?; echo "$(date +%T) pmc $N pass $i ($line) rc=$rc" >> "$R/gpurun_out/status.log"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/pmc_${N}_p$i.log"; exit $rc; }
done < "$R/scripts/${PASSES:-pmc_passes.txt}"
cd "$R"
python3 tools/pmc_report.py "gpurun_out/pmc_$N" > "gpurun_out/pmc_$N.md" && cat "gpurun_out/pmc_$N.md"
exit 0
