#!/bin/bash
# Shared first-step weights: round / native-trainer tests, then a same-box bench A/B (FLR_SHARED_FIRST=1 vs 0).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_round.py tests/test_gpu_native_trainer.py tests/test_gpu_train.py > gpurun_out/t_shared.log 2>&1
rc=$?; tail -3 gpurun_out/t_shared.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  FLR_SHARED_FIRST=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/b_sf$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/b_sf$v.json'));print('shared_first=$v', round(d['ms_per_step'],2), round(d['train_ms_per_round'],2))"
done
