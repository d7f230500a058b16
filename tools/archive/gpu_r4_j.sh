#!/bin/bash
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/diag_layer_grads.py 32 0 3 > gpurun_out/r4j_layer_grads.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4j_layer_grads.txt | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread "tests/test_gpu_native_trainer.py::test_native_trainer_matches_reference_loop" > gpurun_out/r4j_test.log 2>&1 || { echo "test failed"; tail -20 gpurun_out/r4j_test.log; exit 1; }
tail -1 gpurun_out/r4j_test.log
