#!/bin/bash
# round 4 first GPU pass: reference-exact mode, refine rework, bench launcher, one bench line
set -o pipefail
mkdir -p gpurun_out
export FLR_RECORD_DIR=gpurun_out/records
timeout -k 10 120 python -u tools/diag_norm_host.py > gpurun_out/r4a_diag_norm.txt 2>&1; cat gpurun_out/r4a_diag_norm.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_aggregation.py > gpurun_out/r4a_ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4a_ref_tests.log; exit 1; }
tail -3 gpurun_out/r4a_ref_tests.log
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread tests/test_bench_launch.py > gpurun_out/r4a_launch.log 2>&1 || { echo "launch test failed"; tail -40 gpurun_out/r4a_launch.log; exit 1; }
tail -5 gpurun_out/r4a_launch.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { echo "bench failed"; tail -20 gpurun_out/r4a_bench.err; exit 1; }
cat gpurun_out/r4a_bench.json
