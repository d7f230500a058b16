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
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_round.py tests/test_gpu_aggregation.py "tests/test_gpu_train.py::test_c2_round_fedavg_matches_reference" "tests/test_gpu_native_trainer.py::test_native_trainer_matches_reference_loop" tests/test_gpu_conv.py tests/test_gpu_bgemm_dma.py tests/test_gpu_xfmr.py tests/test_gpu_krum_c3.py > gpurun_out/r5c/tests2.log 2>&1 || { echo "tests2 failed"; tail -60 gpurun_out/r5c/tests2.log; exit 1; }
tail -3 gpurun_out/r5c/tests2.log
