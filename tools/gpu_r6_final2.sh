#!/bin/bash
# round 6 final (part 1): the -m gpu suite on the final library, in three
# pytest runs (each under its own limit), then smoke
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread --ignore=tests/test_gpu_shard.py --ignore=tests/test_gpu_configs.py > $O/gpu_tests_a.log 2>&1 || { echo "gpu tests a failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests_a.log | head -20; exit 1; }
tail -1 $O/gpu_tests_a.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_shard.log 2>&1 || { echo "shard tests failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests_shard.log | head -20; exit 1; }
tail -1 $O/gpu_tests_shard.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu --timeout 500 --timeout-method thread > $O/gpu_tests_configs.log 2>&1 || { echo "config tests failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests_configs.log | head -20; exit 1; }
tail -1 $O/gpu_tests_configs.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
