#!/bin/bash
# reference-exact distances over coordinate slices (chains handed rank to rank):
# shard tests (gloo ranks on one GPU), the remaining Krum suites, smoke, the default C3 bench
set -o pipefail
mkdir -p gpurun_out/r5u
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_defenses_ext.py tests/test_gpu_eval.py > gpurun_out/r5u/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" gpurun_out/r5u/tests.log | head -20; tail -30 gpurun_out/r5u/tests.log; exit 1; }
tail -1 gpurun_out/r5u/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5u/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r5u/smoke.log; exit 1; }
tail -1 gpurun_out/r5u/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5u/bench.json 2> gpurun_out/r5u/bench.err || { echo "bench failed"; tail -20 gpurun_out/r5u/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5u/bench.json'))
print({k: d[k] for k in ('value','ms_per_step','global_sha256','sha_matches_reference_run','aggregate_ms','train_ms_per_round')}); print(d['aggregate_ms_by_defense'], d['distance_phase']['ms'])"
