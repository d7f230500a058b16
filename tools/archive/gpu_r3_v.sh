#!/bin/bash
# Round 3: split-at-stash main-loop ablations (tools build, timing only): which phase sets the K-tile time.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V="FLR_SG_ABL=1;FLR_SG_ABL=2;FLR_SG_ABL=3;FLR_SG_ABL=4;FLR_SG_ABL=8;FLR_SG_ABL=10;FLR_SG_ABL=16;FLR_SG_ABL=11;FLR_SG_ABL=15;FLR_SG_ABL=23"
for L in l2b l3b; do
  FLR_LIB=$PWD/abl/abl/libflr.so timeout -k 10 300 python -u tools/conv_bench.py --only $L --variants "$V" > gpurun_out/r3v_conv_$L.txt 2>&1 || exit 1
done
FLR_LIB=$PWD/abl/abl/libflr.so ONLY=vit timeout -k 10 300 python -u tools/bgemm_bench.py --variants "$V" > gpurun_out/r3v_bgemm.txt 2>&1 || exit 1
