#!/bin/bash
# reference-exact distances through the training-order coordinate map: parity
# tests (kernel, rounds, shards, configs) and the default C3 bench line
set -o pipefail
mkdir -p gpurun_out/r5q
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_round.py tests/test_gpu_shard.py tests/test_gpu_configs.py > gpurun_out/r5q/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r5q/tests.log | head -20; tail -30 gpurun_out/r5q/tests.log; exit 1; }
tail -2 gpurun_out/r5q/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5q/bench.json 2> gpurun_out/r5q/bench.err || { echo "bench failed"; tail -20 gpurun_out/r5q/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5q/bench.json'))
print({k: d[k] for k in ('value','ms_per_step','global_sha256','aggregate_ms','train_ms_per_round')}); print(d['distance_phase']); print(d['roofline']); print(d['aggregate_ms_by_defense'])"
