#!/bin/bash
# the tap-major blocks rewritten chain-major (training-order reference distances): timing at C3 (the
# bench's distance phase) + kernel summary
set -o pipefail
mkdir -p gpurun_out/r5s
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py > gpurun_out/r5s/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r5s/tests.log; exit 1; }
tail -1 gpurun_out/r5s/tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5s/prof -o p -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r5s/bench.json 2> gpurun_out/r5s/bench.err || { echo "bench failed"; tail -20 gpurun_out/r5s/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r5s/bench.json').read().strip().splitlines()[-1])
print({k: d[k] for k in ('value','ms_per_step','aggregate_ms','train_ms_per_round')}); print(d['distance_phase']['ms'])"
python3 tools/rocpd_stats.py gpurun_out/r5s/prof/p_results.db > gpurun_out/r5s/stats.txt && grep -E "pwref|kernel  " gpurun_out/r5s/stats.txt
