#!/bin/bash
# C3 Gram kernel timing (pairwise_only at the bench shape) + C5 Gram.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=128 P=11800394 timeout -k 10 200 python -u tools/pairwise_only.py > gpurun_out/pw_only.txt 2>&1 || { tail gpurun_out/pw_only.txt; exit 1; }
tail -3 gpurun_out/pw_only.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gram_bench.json 2> gpurun_out/gram_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/gram_bench.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],2), 'ms/round', d['roofline']['kernel_ms'], d['roofline']['frac'])"
