#!/bin/bash
# pipelined DPP reference-exact kernel: bit-exact tests, timing, kernel summary
set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5g/ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5g/ref_tests.log; exit 1; }
tail -2 gpurun_out/r5g/ref_tests.log
timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 32 > gpurun_out/r5g/bench.json 2> gpurun_out/r5g/bench.err || { echo "bench failed"; tail -5 gpurun_out/r5g/bench.err; exit 1; }
cat gpurun_out/r5g/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5g/prof -o p -- python3 -u tools/ref_bench.py --reps 3 --check 0 > gpurun_out/r5g/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5g/prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5g/prof/p_results.db | head -5
