#!/bin/bash
# reference-exact distances: SGPR-operand chain kernel (default) vs the DPP form; tests
set -o pipefail
mkdir -p gpurun_out/r5c
for v in default ref_dpp_cs64; do
  if [ $v = default ]; then L=multimodal-fl-security_amd/lib/libflr.so; else L=abl/$v/libflr.so; fi
  FLR_LIB=$L timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 24 > gpurun_out/r5c/$v.json 2> gpurun_out/r5c/$v.err || { echo "$v failed"; tail -5 gpurun_out/r5c/$v.err; exit 1; }
  echo "$v $(cat gpurun_out/r5c/$v.json)"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5c/ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5c/ref_tests.log; exit 1; }
tail -2 gpurun_out/r5c/ref_tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5c/prof -o p -- python3 -u tools/ref_bench.py --reps 3 --check 0 > gpurun_out/r5c/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5c/prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5c/prof/p_results.db | head -6
