#!/bin/bash
# round 6: 16-B stores in the tap rewrite's dense writes (tap_chain_kernel):
# parity (tap / reference tests), then the C3 training-order distance phase A/B
# against the previous library (abl/oldtap) and kernel traces of both
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for v in new old; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $v = old ] && lib=abl/oldtap/libflr.so
  FLR_LIB=$lib timeout -k 10 200 python -u tools/ref_bench.py --taps --reps 5 --check 4 > $O/ref_${v}_$r.json 2> $O/ref_${v}_$r.err || { echo "ref $v failed"; tail -5 $O/ref_${v}_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ref_${v}_$r.json')); print('$v', round(d['ms_median'],3), d['mismatches'])"
done; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in new old; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $v = old ] && lib=abl/oldtap/libflr.so
  FLR_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r6u_$v -o t -- python3 tools/ref_bench.py --taps --reps 3 --check 0 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  python3 tools/rocpd_stats.py $(ls /tmp/r6u_$v/*/t_results.db /tmp/r6u_$v/t_results.db 2>/dev/null | head -1) > $O/stats_$v.txt || exit 1
  echo "$v"; grep -E "tap_chain|ref_chain_kernel|chain_transpose" $O/stats_$v.txt | cut -c1-150
done
