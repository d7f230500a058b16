#!/bin/bash
# round 6: x_i by one LDS read + v_readlane (ref_chain_w_kernel<true, true>) against the broadcast form and DPP
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed|Error" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
run() {  # name K P reps env...
  local n=$1 K=$2 P=$3 reps=$4; shift 4
  env "$@" timeout -k 10 300 python -u tools/ref_bench.py --K $K --P $P --reps $reps --check 4 > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['ms_median'],3), d.get('mismatches'))"
}
for r in 1 2; do
  run k512_wg_$r 512 2000003 5 FLR_REF_SGPR=1 || exit 1
  run k512_dpp_$r 512 2000003 5 FLR_REF_SGPR=0 || exit 1
  run k512_rl_$r 512 2000003 5 FLR_REF_SGPR=1 FLR_REF_SGPR_FORM=readlane || exit 1
done




run c5_wg 512 32700000 3 FLR_REF_SGPR=1 || exit 1
run c5_dpp 512 32700000 3 FLR_REF_SGPR=0 || exit 1
run c5_rl 512 32700000 3 FLR_REF_SGPR=1 FLR_REF_SGPR_FORM=readlane || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FLR_REF_SGPR_FORM=readlane timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r6x -o t -- python3 tools/ref_bench.py --K 512 --P 2000003 --reps 3 --check 0 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
python3 tools/rocpd_stats.py $(ls /tmp/r6x/*/t_results.db /tmp/r6x/t_results.db 2>/dev/null | head -1) > $O/stats.txt || exit 1
head -6 $O/stats.txt | cut -c1-160
