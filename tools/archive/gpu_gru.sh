#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests/test_gpu_gru.py tests/test_gpu_train.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gru_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/gru_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gru -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_gru.log 2>&1
timeout -k 10 300 python -u tools/round_ab.py FLR_GRU_FUSED=0 > gpurun_out/round_ab.txt 2>&1
