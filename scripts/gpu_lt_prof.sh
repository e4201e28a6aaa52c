set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_kernel.py --lib build/variants/lib_v7b.so --reps 7 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit $?
timeout -k 10 300 python tools/prof_longtail.py --n 200 --thresholds 256 > gpurun_out/longtail.jsonl 2> gpurun_out/longtail.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_lt" -o lt --output-format csv -- python3 "$R/tools/prof_longtail.py" --n 200 --thresholds 256 --reps 2 > "$R/gpurun_out/prof_lt.log" 2>&1
