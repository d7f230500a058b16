#!/bin/bash
# round 6: the dead-tap deferral gated on the defense (supports_dead_rows) — round tests
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_round.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
