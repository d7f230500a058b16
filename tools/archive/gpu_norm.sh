#!/bin/bash
# Fused clip norm: conv / train / round GPU tests, then the C3 bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_train.py tests/test_gpu_round.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/norm_tests.log 2>&1 || { tail -40 gpurun_out/norm_tests.log; exit 1; }
tail -2 gpurun_out/norm_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/norm_bench.json 2> gpurun_out/norm_bench.err || exit 1
FLR_FUSED_NORM=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/norm_bench0.json 2>> gpurun_out/norm_bench.err || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/norm_bench.json", "gpurun_out/norm_bench0.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms")
PY
