#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread > gpurun_out/gpu_tests4.log 2>&1
rc=$?
echo rc=$rc >> gpurun_out/gpu_tests4.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
