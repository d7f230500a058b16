#!/bin/bash
# round 6: co-resident workgroup controls of the split-at-stash GEMMs (guide:
# two waves per SIMD, items 4 and 9): odd-XCD-slot workgroups started late
# (FLR_GEMM_STAGGER=n x 512 cycles) and/or at static priority 1
# (FLR_GEMM_SPRIO=1); per-layer conv and encoder-GEMM timings, variants
# interleaved in one process
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 400 python -u tools/conv_bench.py --reps 20 --variants "FLR_GEMM_STAGGER=4;FLR_GEMM_STAGGER=8;FLR_GEMM_SPRIO=1;FLR_GEMM_STAGGER=8,FLR_GEMM_SPRIO=1" > $O/conv.txt 2>&1 || { echo "conv failed"; tail -5 $O/conv.txt; exit 1; }
tail -16 $O/conv.txt
timeout -k 10 400 python -u tools/bgemm_bench.py --variants "FLR_GEMM_STAGGER=8;FLR_GEMM_SPRIO=1" > $O/bgemm.txt 2>&1 || { echo "bgemm failed"; tail -5 $O/bgemm.txt; exit 1; }
tail -8 $O/bgemm.txt
