#!/bin/bash
# round 6: persistent tap-rewrite workgroups (FLR_TAP_PERSIST=N per XCD and client)
# — parity, then the C3 training-order distance phase A/B and kernel traces
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
for v in 1 2; do
  FLR_TAP_PERSIST=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py -k "tap" > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; grep -E "^E |FAILED|passed|failed" $O/tests_$v.log | head -20; exit 1; }
  tail -1 $O/tests_$v.log
done
for v in 0 1 2 4 0 1 2 4; do
  FLR_TAP_PERSIST=$v timeout -k 10 200 python -u tools/ref_bench.py --taps --reps 5 --check 4 > $O/ref_$v.json 2> $O/ref_$v.err || { echo "ref $v failed"; tail -5 $O/ref_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/ref_$v.json')); print('persist=$v', round(d['ms_median'],3), d['mismatches'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 1 2; do
  FLR_TAP_PERSIST=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r6t_$v -o t -- python3 tools/ref_bench.py --taps --reps 3 --check 0 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  python3 tools/rocpd_stats.py $(ls /tmp/r6t_$v/*/t_results.db /tmp/r6t_$v/t_results.db 2>/dev/null | head -1) > $O/stats_$v.txt || exit 1
  echo "persist=$v"; grep -E "tap_chain" $O/stats_$v.txt | cut -c1-150
done
