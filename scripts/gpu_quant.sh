set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for wf in 786432 983040 1000000 1048576 1179648 1228800; do
  timeout -k 10 200 python tools/prof_kernel.py --wf $wf --reps 5 >> gpurun_out/quant.jsonl 2>>gpurun_out/quant.err || exit 1
done
