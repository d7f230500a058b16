#!/bin/bash
# reference-exact distances: transpose of segment s+1 on a side stream under the
# chain kernel of segment s; segment-size sweep, bit-exact tests, kernel summary
set -o pipefail
mkdir -p gpurun_out/r5h
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5h/ref_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r5h/ref_tests.log; exit 1; }
tail -2 gpurun_out/r5h/ref_tests.log
for cfg in "FLR_REF_OVERLAP=0" "FLR_REF_SEG_MB=1024" "FLR_REF_SEG_MB=512" "FLR_REF_SEG_MB=256" "FLR_REF_SEG_MB=128" "FLR_REF_SEG_MB=64"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 8 > gpurun_out/r5h/bench_$cfg.json 2> gpurun_out/r5h/bench_$cfg.err || { echo "bench failed"; tail -5 gpurun_out/r5h/bench_$cfg.err; exit 1; }
  cat gpurun_out/r5h/bench_$cfg.json
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r5h/prof -o p -- python3 -u tools/ref_bench.py --reps 3 --check 0 > gpurun_out/r5h/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5h/prof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5h/prof/p_results.db | head -5
