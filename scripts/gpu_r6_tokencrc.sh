#!/bin/bash
# Round 6: crr_inputs.token_crc -- its GPU tests and the golden / full-size parity tests, then the headline
# alternated with and without the splice (3 rounds, --headline-only).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out/tokcrc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  tests/test_gpu_parity.py tests/test_golden.py > gpurun_out/tokcrc/pytest.log 2>&1 || { tail -30 gpurun_out/tokcrc/pytest.log; exit 1; }
tail -2 gpurun_out/tokcrc/pytest.log
for i in 1 2 3; do
  for v in on off; do
    a=""; [ $v = off ] && a="--no-token-crc"
    timeout -k 10 300 python -u bench.py --headline-only --steps 20 --warmup 3 --no-cpu-baseline $a > gpurun_out/tokcrc/c2_${v}_$i.json 2> gpurun_out/tokcrc/c2_${v}_$i.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/tokcrc/c2_${v}_$i.json $v$i
  done
done
