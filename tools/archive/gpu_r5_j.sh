#!/bin/bash
# reference-exact distances: chain-major rows padded off the L2 channel stride
# (FLR_REF_ROW_MOD sweep), bit-exact tests, timing, kernel summary
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5j/ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5j/ref_tests.log; exit 1; }
tail -2 gpurun_out/r5j/ref_tests.log
for m in -1 2304 256 1280 3328; do
  FLR_REF_ROW_MOD=$m timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 8 > gpurun_out/r5j/bench_$m.json 2> gpurun_out/r5j/bench_$m.err || { echo "bench failed"; tail -5 gpurun_out/r5j/bench_$m.err; exit 1; }
  echo "ROW_MOD=$m $(cat gpurun_out/r5j/bench_$m.json)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5j/prof -o p -- python3 -u tools/ref_bench.py --reps 3 --check 0 > gpurun_out/r5j/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5j/prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5j/prof/p_results.db > gpurun_out/r5j/stats.txt && head -5 gpurun_out/r5j/stats.txt
