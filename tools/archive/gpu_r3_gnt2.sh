#!/bin/bash
# Round 3: Gram DMA policy at the C4 / C5 shapes (K = 256 / 512: cross groups re-read rows): FLR_GRAM_NT 1 vs 2.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in 1 2 1 2; do
  echo "FLR_GRAM_NT=$v"
  GRAM_ALL=1 FLR_GRAM_NT=$v timeout -k 10 300 python -u tools/agg_c4c5.py 2>&1 | grep -i "gram\|pairwise\|krum" || exit 1
done
