#!/bin/bash
# reference-exact chain kernel: timing-only ablations (abl/abl1..5, wrong results)
set -o pipefail
mkdir -p gpurun_out/r5l
for v in default abl1 abl2 abl3 abl4 abl5; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $v != default ] && lib=abl/$v/libflr.so
  FLR_LIB=$lib timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 0 > gpurun_out/r5l/bench_$v.json 2> gpurun_out/r5l/bench_$v.err || { echo "bench failed"; tail -5 gpurun_out/r5l/bench_$v.err; exit 1; }
  echo "$v $(cut -c1-120 gpurun_out/r5l/bench_$v.json)"
done
