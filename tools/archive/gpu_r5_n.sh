#!/bin/bash
# reference-exact chain kernel: one-wave tiles (4 I x 16 J rows), no barrier
# , bit-exact tests on the default, timing, kernel summary
set -o pipefail
mkdir -p gpurun_out/r5n
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5n/ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5n/ref_tests.log; exit 1; }
tail -2 gpurun_out/r5n/ref_tests.log
for v in default; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $v != default ] && lib=abl/$v/libflr.so
  FLR_LIB=$lib timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 8 > gpurun_out/r5n/bench_$v.json 2> gpurun_out/r5n/bench_$v.err || { echo "bench failed"; tail -5 gpurun_out/r5n/bench_$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r5n/bench_$v.json)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5n/prof -o p -- python3 -u tools/ref_bench.py --reps 3 --check 0 > gpurun_out/r5n/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5n/prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5n/prof/p_results.db > gpurun_out/r5n/stats.txt && head -5 gpurun_out/r5n/stats.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d gpurun_out/r5n/pmc -o p -- python3 -u tools/ref_bench.py --reps 1 --check 0 > gpurun_out/r5n/pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r5n/pmc.log; exit 1; }
python3 tools/pmc_stats.py gpurun_out/r5n/pmc/p_results.db | grep -E "kernel  |chain_kernel"
