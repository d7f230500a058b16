#!/bin/bash
# Tile sweep of the split-at-stash conv kernels + PMC passes on l1 fwd/dgrad/wgrad.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_bench.py --variants "FLR_CONV_TILE=11;FLR_CONV_TILE=12;FLR_CONV_TILE=21;FLR_CONV_TILE=22" > gpurun_out/tiles2.txt 2>&1 || exit 1
LAYER=l1 bash tools/archive/pmc_conv3.sh || exit 1
LAYER=l3b bash tools/archive/pmc_conv3.sh || exit 1
