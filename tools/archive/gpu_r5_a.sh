#!/bin/bash
# round 5 first GPU pass: the reworked reference-exact distance kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5b_ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5b_ref_tests.log; exit 1; }
tail -3 gpurun_out/r5b_ref_tests.log
timeout -k 10 240 python -u tools/ref_bench.py --reps 5 --check 48 > gpurun_out/r5b_ref_bench.json 2> gpurun_out/r5b_ref_bench.err || { echo "ref bench failed"; tail -20 gpurun_out/r5b_ref_bench.err; exit 1; }
cat gpurun_out/r5b_ref_bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b_prof -o r5a -- python3 -u tools/ref_bench.py --reps 3 --check 0 > gpurun_out/r5b_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5b_prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5b_prof/r5b_results.db | head -8
