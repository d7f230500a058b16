#!/bin/bash
# round 4: refine compact mapping + reference-mode DMA ring: parity tests, the C3 trained round, stats
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
export FLR_RECORD_DIR=$R/gpurun_out/records
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_aggregation.py tests/test_gpu_shard.py tests/test_gpu_pairwise_reference.py tests/test_gpu_krum_c3.py "tests/test_gpu_configs.py::test_c3_trained_round_krum_indices_vs_reference_norms" > gpurun_out/r4d_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r4d_tests.log | head; tail -30 gpurun_out/r4d_tests.log; exit 1; }
tail -3 gpurun_out/r4d_tests.log
grep -o '"reference_mode[^,]*' gpurun_out/records/c3_krum_trained_round.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pc3 -o b -- python3 "$R/bench.py" --steps 8 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/r4d_prof_c3.log" 2>&1 || { echo "prof rc=$?"; tail -20 "$R/gpurun_out/r4d_prof_c3.log"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pc3/b_results.db > gpurun_out/r4d_c3_kernel_stats.txt 2>&1
grep -E "refine|gram_partials|rows_mean" gpurun_out/r4d_c3_kernel_stats.txt | cut -c1-150
grep -o "\"aggregate_ms_by_defense\": {[^}]*}" gpurun_out/r4d_prof_c3.log; grep -E "orderstat|pairwise_ref" gpurun_out/r4d_c3_kernel_stats.txt | cut -c1-150; tail -1 gpurun_out/r4d_prof_c3.log | cut -c1-300
