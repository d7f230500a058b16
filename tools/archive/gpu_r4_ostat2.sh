#!/bin/bash
# Row-subset order statistics with LDS-staged indices: the aggregation tests, then the C4 / C5 shapes
# (incl. the trimmed mean of 256 of 512 rows, the C5 defense's second half).
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ostat2
timeout -k 10 400 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_defenses_ext.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ostat2/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ostat2/tests.log; exit 1; }
tail -1 gpurun_out/ostat2/tests.log
timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/ostat2/agg.log 2>&1 || { echo "agg rc=$?"; tail -20 gpurun_out/ostat2/agg.log; exit 1; }
grep -h '"kernel"' gpurun_out/ostat2/agg.log | cut -c1-200
