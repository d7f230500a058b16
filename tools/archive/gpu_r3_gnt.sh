#!/bin/bash
# Round 3: Gram DMA with default vs non-temporal policy (FLR_GRAM_NT), C3 bench roofline, alternating runs.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_krum_c3.py tests/test_gpu_aggregation.py > gpurun_out/gnt_tests.txt 2>&1 || exit 1
tail -1 gpurun_out/gnt_tests.txt
for i in 1 2; do
  for v in 0 1; do
    FLR_GRAM_NT=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/gnt_$v.json 2> gpurun_out/gnt_$v.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/gnt_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('nt=$v', round(d['ms_per_step'],2), 'ms/round agg', round(d['aggregate_ms'],3), 'gram_ms', round(r['kernel_ms'],4), 'frac', round(r['frac'],4))"
  done
done
