#!/bin/bash
# Round-4 closing check on the final library: full -m gpu suite + smoke, the C3 line (cpu_baseline), the
# C4 / C5 lines come from tools/archive/gpu_r4_bench.sh (CONFIGS="C4 C5") in a call of their own.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/final3
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/final3/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/final3/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final3/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final3/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final3/smoke.log; exit 1; }
tail -1 gpurun_out/final3/smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/final3/bench_c3.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/final3/bench_c3.log; exit 1; }
grep '^{"metric' gpurun_out/final3/bench_c3.log > gpurun_out/final3/r4_bench_c3_final.json
cut -c1-200 gpurun_out/final3/r4_bench_c3_final.json
