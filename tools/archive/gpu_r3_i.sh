#!/bin/bash
# Round 3: optimizer update on a side stream under the next step's forward —
# bit-identity (phase split, native vs Python trainer, rounds), then the C3 bench
# with the overlap on / off (FLR_SGD_OVERLAP=0), same box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgd_phase.py tests/test_gpu_native_trainer.py tests/test_gpu_round.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 || exit 1
for v in 1 0 1 0; do
  FLR_SGD_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
    >> gpurun_out/r3i_bench_ov$v.json 2>> gpurun_out/r3i_bench.err || exit 1
done
