#!/bin/bash
# Local helper (runs HERE, not on the GPU box): one gpurun call that also ships tools/variants/*.so (the A/B
# variant libraries), which .gpurunignore otherwise keeps off every box -- the driver's round-end push
# included.  The ignore line is restored on exit, whatever happens.
#   scripts/gpurun_with_variants.sh <gpurun timeout s> '<command>'
set -u
cd "$(dirname "$0")/.."
cp .gpurunignore /tmp/.gpurunignore.keep
trap 'cp /tmp/.gpurunignore.keep .gpurunignore' EXIT
grep -v '^\./tools/variants$' /tmp/.gpurunignore.keep > .gpurunignore
/usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
