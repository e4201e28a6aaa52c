#!/bin/bash
# Round-5 config-4 study: the NDC tests, then the tail kernel alone / with only its longest runs, and the
# cycle split of the wavefront path (tools/wave_prof.py variant).  Each step under its own limit.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"; mkdir -p gpurun_out
log() { echo "$(date +%T) $*" >> "$R/gpurun_out/status.log"; }
step() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1
  local rc=$?; log "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-12}; return $rc
}
if [ -n "${TESTS:-}" ]; then
  step pytest_r5 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread || exit $?
fi
step c4_top256 400 python -u tools/prof_c4_segments.py --only tail,tailtop --top 256 || exit $?
step c4_top1024 400 python -u tools/prof_c4_segments.py --only tailtop --top 1024 || exit $?
if [ -f tools/variants/waveprof.so ]; then
  step c4_waveprof 400 python -u tools/prof_c4_segments.py --lib tools/variants/waveprof.so --only tail,tailtop --top 256 --wave-prof || exit $?
fi
exit 0
