#!/bin/bash
# row-subset mean / FedAvg with 8 rows' loads in flight: aggregation tests, C3 line + summary
set -o pipefail
D=gpurun_out/r5mean; mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_aggregation.py tests/test_gpu_krum_c3.py tests/test_gpu_pairwise_reference.py -k "mean or fedavg or krum or c3" > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o p -- python3 -u bench.py --steps 3 --warmup 1 > $D/b.log 2>&1 || { echo "prof failed"; tail -20 $D/b.log; exit 1; }
python3 tools/rocpd_stats.py $D/prof/p_results.db > $D/stats.txt && grep -E "rows_mean|fedavg" $D/stats.txt | cut -c1-50,90-160
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/c3_25.json 2> $D/c3_25.err || { echo "bench25 failed"; tail -20 $D/c3_25.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c3_25.json').read().strip().splitlines()[-1]); print(d['value'], d['aggregate_ms'], d['aggregate_ms_by_defense'], d['global_sha256'][:12], d['sha_matches_reference_run'])"
