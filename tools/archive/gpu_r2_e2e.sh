#!/bin/bash
# C2/C3 end-to-end GPU tests, the C3 round profile, the C5 bench line
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -m gpu -q -rA --timeout 600 --timeout-method thread -k "c2_round" > gpurun_out/e2e_tests.log 2>&1
rc=$?
echo rc=$rc >> gpurun_out/e2e_tests.log
[ $rc -gt 1 ] && exit $rc
[ "${TESTS_ONLY:-0}" = 1 ] && exit 0
mkdir -p gpurun_out/prof_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3/bench.json 2> gpurun_out/prof_c3/bench.err || exit $?
timeout -k 10 600 python -u bench.py --config C5 --steps 1 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
echo rc=$? >> gpurun_out/bench_c5.err
