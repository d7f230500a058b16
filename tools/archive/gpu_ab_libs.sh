#!/bin/bash
# Same-box A/B of library builds: conv_bench + C3 bench per FLR_LIB.
# usage: tools/archive/gpu_ab_libs.sh name1 name2 ...  (names under abl/, "main" = the in-tree lib)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in "$@"; do
  if [ "$n" = main ]; then lib=$PWD/multimodal-fl-security_amd/lib/libflr.so; else lib=$PWD/abl/$n/libflr.so; fi
  FLR_LIB=$lib timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/ab_conv_$n.txt 2>&1 || exit 1
  FLR_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench_$n.json 2> gpurun_out/ab_bench_$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],2), 'ms/round', 'conv sum', open('gpurun_out/ab_conv_$n.txt').read().strip().splitlines()[-1])"
done
