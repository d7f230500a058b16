#!/bin/bash
# Quarter-split order statistics as the default: the aggregation / defense / config tests.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/q4b
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_defenses_ext.py tests/test_gpu_configs.py tests/test_gpu_round.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q4b/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/q4b/tests.log; exit 1; }
tail -1 gpurun_out/q4b/tests.log
