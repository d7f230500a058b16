#!/bin/bash
# Session check: GPU test suite, default bench line, rocprofv3 kernel summary of a short bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s3.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/gpu_tests_s3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_s3.json 2> gpurun_out/bench_s3.err || exit $?
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /root/repo/gpurun_out/prof_s3.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/prof_s3_stats.txt
