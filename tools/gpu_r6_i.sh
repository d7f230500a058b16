#!/bin/bash
# round 6: the tap rewrite on 16 x 576 tiles (FLR_TAP_TILE=16) — parity, then
# the C3 training-order distance phase A/B (tools/ref_bench.py --taps) and a
# kernel trace of each form
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
FLR_TAP_TILE=64 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py -k "tap" > $O/tests64.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests64.log | head -20; exit 1; }
tail -1 $O/tests64.log
for v in 0 64 0 64; do
  FLR_TAP_TILE=$v timeout -k 10 200 python -u tools/ref_bench.py --taps --reps 5 --check 8 > $O/ref_$v.json 2> $O/ref_$v.err || { echo "ref $v failed"; tail -5 $O/ref_$v.err; exit 1; }
  echo "tile=$v $(cat $O/ref_$v.json)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 0 64; do
  FLR_TAP_TILE=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r6n_$v -o t -- python3 tools/ref_bench.py --taps --reps 3 --check 0 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  python3 tools/rocpd_stats.py $(ls /tmp/r6n_$v/*/t_results.db /tmp/r6n_$v/t_results.db 2>/dev/null | head -1) > $O/stats_$v.txt || exit 1
  grep -E "tap_chain|ref_chain|transpose" $O/stats_$v.txt | cut -c1-150
done
