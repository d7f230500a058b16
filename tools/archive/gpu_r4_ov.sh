#!/bin/bash
# side-stream optimizer together with the text / weight-gradient streams: bit-identity, then K=16/32/128 A/B
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_native_trainer.py::test_native_trainer_bit_identical_to_python_trainer" tests/test_gpu_round.py > gpurun_out/r4ov_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4ov_tests.log; exit 1; }
tail -1 gpurun_out/r4ov_tests.log
timeout -k 10 300 python3 -u tools/lib_identity.py 2>&1 | grep -v amdgpu.ids
for V in FLR_X=0; do
  for KK in 16 32 128; do
    ( export "$V"; timeout -k 10 300 python3 -u bench.py --clients $KK --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4ov_bench.log 2>&1 ) || { echo "bench rc=$?"; tail -5 gpurun_out/r4ov_bench.log; exit 1; }
    echo "K=$KK $V $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4ov_bench.log)"
  done
done
