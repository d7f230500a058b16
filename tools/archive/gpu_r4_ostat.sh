#!/bin/bash
# K = 256 / 512 order statistics at split vs whole load wait: the aggregation tests under each, then the C4 / C5 shapes.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ostat
timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/ostat/w2.log 2>&1 || { echo "w2 rc=$?"; tail -20 gpurun_out/ostat/w2.log; exit 1; }
FLR_OSTAT_NOSPLIT=1 timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/ostat/w3.log 2>&1 || { echo "w3 rc=$?"; tail -20 gpurun_out/ostat/w3.log; exit 1; }
grep -h '"kernel"' gpurun_out/ostat/w2.log gpurun_out/ostat/w3.log | cut -c1-200
timeout -k 10 400 python -u -m pytest tests/test_gpu_aggregation.py -m gpu -q -x -k "trimmed or median or order" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ostat/tests_w3.log 2>&1 || { echo "tests w3 failed"; tail -30 gpurun_out/ostat/tests_w3.log; exit 1; }
tail -1 gpurun_out/ostat/tests_w3.log
