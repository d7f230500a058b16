#!/bin/bash
# GPU session: the full -m gpu suite, then (if no crash) one bench line.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
