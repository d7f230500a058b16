#!/bin/bash
# round 6: the SGPR-operand throughput form of the reference chains (K >= 480):
# parity (reference-distance tests), then K=512 A/B against the DPP kernel at
# P = 2M and at the C5 shape, and a kernel trace
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed|Error" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for v in 1 0 8 1 0 8; do
  FLR_REF_SGPR=$([ $v = 8 ] && echo 1 || echo $v) FLR_REF_SGPR_ROWS=$([ $v = 8 ] && echo 8 || echo 4) timeout -k 10 200 python -u tools/ref_bench.py --K 512 --P 2000003 --reps 5 --check 8 > $O/k512_2m_$v.json 2> $O/k512_2m_$v.err || { echo "ref $v failed"; tail -5 $O/k512_2m_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/k512_2m_$v.json')); print('K512 P2M sgpr=$v', round(d['ms_median'],3), d.get('mismatches'))"
done
for k in 256 384; do for v in 1 0; do
  FLR_REF_SGPR=$v timeout -k 10 200 python -u tools/ref_bench.py --K $k --P 4000037 --reps 3 --check 4 > $O/k${k}_$v.json 2> $O/k${k}_$v.err || { echo "k$k $v failed"; tail -5 $O/k${k}_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/k${k}_$v.json')); print('K$k P4M sgpr=$v', round(d['ms_median'],3), d.get('mismatches'))"
done; done
for v in 1 0; do
  FLR_REF_SGPR=$v timeout -k 10 300 python -u tools/ref_bench.py --K 512 --P 32700000 --reps 3 --check 2 > $O/k512_c5_$v.json 2> $O/k512_c5_$v.err || { echo "c5 $v failed"; tail -5 $O/k512_c5_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/k512_c5_$v.json')); print('K512 C5 sgpr=$v', round(d['ms_median'],3), d.get('mismatches'))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/r6o -o t -- python3 tools/ref_bench.py --K 512 --P 2000003 --reps 3 --check 0 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
python3 tools/rocpd_stats.py $(ls /tmp/r6o/*/t_results.db /tmp/r6o/t_results.db 2>/dev/null | head -1) > $O/stats.txt || exit 1
head -8 $O/stats.txt | cut -c1-160
