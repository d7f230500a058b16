#!/bin/bash
# the committed library as shipped: reference / shard tests and smoke()
set -o pipefail
D=gpurun_out/r5last; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_shard.py tests/test_gpu_krum_c3.py > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
