#!/bin/bash
# After the GEMM epilogue refactor / force-inlined plans: library identity hashes (vs round 3),
# conv + trainer tests, and the C3 bench line.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/lib_identity.py > gpurun_out/r4e_lib_identity.txt 2>&1 || { echo "identity rc=$?"; tail -20 gpurun_out/r4e_lib_identity.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4e_lib_identity.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_native_trainer.py tests/test_gpu_bgemm.py tests/test_gpu_bgemm_dma.py > gpurun_out/r4e_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4e_bench_c3.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r4e_bench_c3.log; exit 1; }
grep '^{"metric' gpurun_out/r4e_bench_c3.log | cut -c1-400
