#!/bin/bash
# the driver's GPU tier: the whole -m gpu suite, then smoke()
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_full_gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r4_full_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -2 gpurun_out/r4_smoke.log
