#!/bin/bash
# refine ring: aggregation / shard / reference / Krum C3 tests (records bit-identical), then the C3 aggregate timing
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_aggregation.py tests/test_gpu_shard.py tests/test_gpu_krum_c3.py > gpurun_out/r4rf_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r4rf_tests.log; exit 1; }
tail -1 gpurun_out/r4rf_tests.log
timeout -k 10 300 python3 -u tools/lib_identity.py 2>&1 | grep -v amdgpu.ids
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prf -o b -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r4rf_prof.log" 2>&1 || { echo "prof rc=$?"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/prf/b_results.db > gpurun_out/r4rf_stats.txt 2>&1
grep -E "refine|gram_partials|rows_mean" gpurun_out/r4rf_stats.txt | cut -c1-150
grep -o '"aggregate_ms": [0-9.]*, "aggregate_ms_by_defense": {[^}]*}' gpurun_out/r4rf_prof.log
