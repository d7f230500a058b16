#!/bin/bash
# Gram kernel changes: aggregation / Krum GPU tests, C4/C5 aggregation timings, C3 bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_krum_c3.py tests/test_gpu_shard.py -m gpu -x -q -rf -s --timeout 300 --timeout-method thread > gpurun_out/gram_tests.log 2>&1 || { tail -40 gpurun_out/gram_tests.log; exit 1; }
grep "2-term Gram\|passed\|failed" gpurun_out/gram_tests.log | tail -6
timeout -k 10 400 python -u tools/agg_c4c5.py > gpurun_out/agg_c4c5.txt 2>&1 || { tail gpurun_out/agg_c4c5.txt; exit 1; }
cat gpurun_out/agg_c4c5.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gram_bench.json 2> gpurun_out/gram_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/gram_bench.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), 'ms/round', d['roofline']['kernel_ms'], d['roofline']['frac'])"
