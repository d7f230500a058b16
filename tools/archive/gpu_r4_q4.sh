#!/bin/bash
# K = 256 / 512 order statistics: halves (default) vs quarters (FLR_OSTAT_Q4) of the split load wait, plus the
# order-statistics tests under quarters.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/q4
timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/q4/halves.log 2>&1 || { echo "halves rc=$?"; tail -20 gpurun_out/q4/halves.log; exit 1; }
FLR_OSTAT_Q4=1 timeout -k 10 300 python -u tools/agg_c4c5.py > gpurun_out/q4/quarters.log 2>&1 || { echo "quarters rc=$?"; tail -20 gpurun_out/q4/quarters.log; exit 1; }
FLR_OSTAT_Q4=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregation.py -m gpu -q -x -k "order or trimmed or median" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q4/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/q4/tests.log; exit 1; }
tail -1 gpurun_out/q4/tests.log
for f in halves quarters; do echo "== $f"; grep -h '"kernel"' gpurun_out/q4/$f.log | grep -v gram | python3 -c "import sys,json; [print(d['config'], d['kernel'], round(d['ms'],3)) for d in map(json.loads, sys.stdin)]"; done
