#!/bin/bash
# reference chain kernel: two waves per SIMD (4-stage ring) past 1024 waves;
# bit-exact tests, K = 512 timing both ways, C3 unchanged
set -o pipefail
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5v/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5v/tests.log; exit 1; }
tail -1 gpurun_out/r5v/tests.log
for w in 0 1; do
  FLR_REF_2W=$w timeout -k 10 200 python -u tools/ref_bench.py --K 512 --P 2000003 --reps 3 --check 4 > gpurun_out/r5v/k512_$w.json 2> gpurun_out/r5v/k512_$w.err || { echo "bench failed"; tail -5 gpurun_out/r5v/k512_$w.err; exit 1; }
  echo "K=512 2W=$w $(cut -c1-150 gpurun_out/r5v/k512_$w.json)"
done
timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 8 > gpurun_out/r5v/c3.json 2> gpurun_out/r5v/c3.err || { echo "bench failed"; tail -5 gpurun_out/r5v/c3.err; exit 1; }
echo "C3 $(cut -c1-150 gpurun_out/r5v/c3.json)"
