#!/bin/bash
# the kept tap form + the transpose over needed waves only: reference / shard /
# C3-config tests, the default C3 bench line, its kernel summary, the 25-round sha
set -o pipefail
D=gpurun_out/r5tap2; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_shard.py tests/test_gpu_configs.py > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 200 python -u tools/ref_bench.py --taps --reps 5 --check 8 > $D/ref_taps.json 2> $D/ref_taps.err || { echo "ref bench failed"; tail -20 $D/ref_taps.err; exit 1; }
cat $D/ref_taps.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/c3_25.json 2> $D/c3_25.err || { echo "bench25 failed"; tail -20 $D/c3_25.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c3_25.json').read().strip().splitlines()[-1]); print(d['value'], d['aggregate_ms'], d['distance_phase']['ms'], d['global_sha256'][:12], d['sha_matches_reference_run'])"
timeout -k 10 300 python -u bench.py > $D/c3_default.json 2> $D/c3_default.err || { echo "bench failed"; tail -20 $D/c3_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c3_default.json').read().strip().splitlines()[-1]); print(d['value'], d['aggregate_ms'], d['distance_phase']['ms'])"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/bprof -o p -- python3 -u bench.py --steps 3 --warmup 1 > $D/bprof.log 2>&1 || { echo "prof failed"; tail -20 $D/bprof.log; exit 1; }
python3 tools/rocpd_stats.py $D/bprof/p_results.db > $D/bench_stats.txt && grep -E "pwref" $D/bench_stats.txt | cut -c1-50,90-160
