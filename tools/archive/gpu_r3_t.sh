#!/bin/bash
# Round 3: GRU step kernels with the ordered one-slot reduction ("8,2s": two / three workgroups
# per CU) — bit-identity and timing against the 8-slot form; unrolled sum-of-squares pass (tests);
# C3 bench with each GRU form, same box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gru_bench.py > gpurun_out/r3t_gru.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_native_trainer.py tests/test_gpu_sgd_phase.py \
  tests/test_gpu_gru.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1 || exit 1
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export FLR_GRU_FW=8,2s FLR_GRU_BW=8,2s; else unset FLR_GRU_FW FLR_GRU_BW; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline >> gpurun_out/r3t_bench_$v.json 2>/dev/null || exit 1
done
