#!/bin/bash
# Round 3: swizzled (unpadded) split-at-stash LDS images — bit-identity of the
# conv / batched-GEMM tests, then same-box A/B: main (swizzle, 2 waves/SIMD) vs
# occ3 (swizzle, 3 waves/SIMD) vs noswz (padded rows): conv_bench, bgemm_bench, C3 bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_bgemm.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3h_tests.log 2>&1 || exit 1
for n in main occ3 noswz; do
  if [ "$n" = main ]; then lib=$PWD/multimodal-fl-security_amd/lib/libflr.so; else lib=$PWD/abl/$n/libflr.so; fi
  FLR_LIB=$lib timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/r3h_conv_$n.txt 2>&1 || exit 1
  FLR_LIB=$lib timeout -k 10 300 python -u tools/bgemm_bench.py > gpurun_out/r3h_bgemm_$n.txt 2>&1 || exit 1
  FLR_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r3h_bench_$n.json 2> gpurun_out/r3h_bench_$n.err || exit 1
done
