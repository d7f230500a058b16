#!/bin/bash
# Krum's default distances now reference-exact: the suites that build Krum
# defenses, smoke(), and the default C3 bench line
set -o pipefail
mkdir -p gpurun_out/r5t
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_pairwise_reference.py tests/test_gpu_defenses_ext.py tests/test_gpu_eval.py > gpurun_out/r5t/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r5t/tests.log | head -20; tail -30 gpurun_out/r5t/tests.log; exit 1; }
tail -1 gpurun_out/r5t/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5t/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5t/smoke.log; exit 1; }
tail -1 gpurun_out/r5t/smoke.log
