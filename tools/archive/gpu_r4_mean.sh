#!/bin/bash
# Mean kernels with 8 row loads in flight: the aggregation tests, then the C3 line's aggregate_ms_by_defense.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/mean
timeout -k 10 400 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_defenses_ext.py tests/test_gpu_round.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mean/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/mean/tests.log; exit 1; }
tail -1 gpurun_out/mean/tests.log
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/mean/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/mean/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/mean/bench.log') if l.startswith('{\"metric')][-1]); print(d['value'], d['aggregate_ms'], d['aggregate_ms_by_defense'])"
