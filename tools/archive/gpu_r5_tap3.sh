#!/bin/bash
# the tap kernel as persistent workgroups (next tile's loads under the current
# tile's writes): reference tests, --taps timing + check, kernel summary
set -o pipefail
D=gpurun_out/r5tap3; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pairwise_reference.py > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 200 python -u tools/ref_bench.py --taps --reps 5 --check 8 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 1; }
cat $D/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof -o p -- python3 -u tools/ref_bench.py --taps --reps 3 --check 0 > $D/prof.log 2>&1 || { echo "prof failed"; tail -20 $D/prof.log; exit 1; }
python3 tools/rocpd_stats.py $D/prof/p_results.db > $D/stats.txt && grep -E "tap_chain|transpose|ref_chain" $D/stats.txt | cut -c1-50,90-160
