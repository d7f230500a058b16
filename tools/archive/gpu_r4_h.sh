#!/bin/bash
# fp64 step diagnostic; fill tiles + text stream: bit-identity (tests, library identity), K=16 / K=128 timing A/B
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/diag_step0_fp64.py 32 0 3 > gpurun_out/r4h_step0_fp64.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4h_step0_fp64.txt | tail -14
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py -k "fill or narrow or forms" "tests/test_gpu_native_trainer.py::test_native_trainer_bit_identical_to_python_trainer" tests/test_gpu_round.py > gpurun_out/r4h_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -1 gpurun_out/r4h_tests.log
timeout -k 10 300 python3 -u tools/lib_identity.py 2>&1 | grep -v amdgpu.ids
for V in "base" "FLR_CONV_FILL=0" "FLR_TEXT_STREAM=0" "FLR_CONV_FILL=0,FLR_TEXT_STREAM=0"; do
  for KK in 16 128; do
    ( if [ "$V" != base ]; then for kv in ${V//,/ }; do export "$kv"; done; fi
      timeout -k 10 300 python3 -u bench.py --clients $KK --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4h_bench.log 2>&1 ) || { echo "bench rc=$?"; tail -5 gpurun_out/r4h_bench.log; exit 1; }
    echo "K=$KK $V $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4h_bench.log)"
  done
done
