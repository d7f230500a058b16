#!/bin/bash
# Full GPU suite, the default C3 bench line, and a C3 kernel profile
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/ck_tests.log 2>&1
rc=$?
echo rc=$rc >> gpurun_out/ck_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/ck_bench.json 2> gpurun_out/ck_bench.err || exit $?
mkdir -p gpurun_out/prof_ck
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ck -o c3 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_ck/bench.json 2> gpurun_out/prof_ck/bench.err
