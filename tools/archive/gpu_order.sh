#!/bin/bash
# Training-order rounds: the affected GPU tests, then the C3 bench (both orders).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_round.py tests/test_gpu_train.py tests/test_gpu_shard.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/order_tests.log 2>&1 || { tail -30 gpurun_out/order_tests.log; exit 1; }
tail -2 gpurun_out/order_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/order_bench.json 2> gpurun_out/order_bench.err || exit 1
FLR_ORDER=torch timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/order_bench_torch.json 2>> gpurun_out/order_bench.err || exit 1
python - <<'PY'
import json
for f in ("gpurun_out/order_bench.json", "gpurun_out/order_bench_torch.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms", "train", round(d["train_ms_per_round"], 2), "agg", round(d["aggregate_ms"], 3))
PY
