#!/bin/bash
# tap_chain_kernel (training-order C3 matrix): the write-phase forms (FLR_TAP_WR
# 0 / 1 / 2) timed and checked, a kernel summary each, HBM traffic passes of form 0
set -o pipefail
D=gpurun_out/r5tap; mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pairwise_reference.py > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for w in 0 2 4; do
  FLR_TAP_WR=$w timeout -k 10 200 python -u tools/ref_bench.py --taps --reps 5 --check 8 > $D/bench_$w.json 2> $D/bench_$w.err || { echo "bench $w failed"; tail -20 $D/bench_$w.err; exit 1; }
  echo "wr $w $(cat $D/bench_$w.json)"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in 0 2 4; do
  FLR_TAP_WR=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof$w -o p -- python3 -u tools/ref_bench.py --taps --reps 3 --check 0 > $D/prof$w.log 2>&1 || { echo "prof failed"; tail -20 $D/prof$w.log; exit 1; }
  python3 tools/rocpd_stats.py $D/prof$w/p_results.db > $D/stats$w.txt && grep -E "tap_chain|ref_chain|transpose" $D/stats$w.txt | cut -c1-40,90-160
done
run() {
  timeout -s KILL 120 rocprofv3 --pmc $2 -d $D/$1 -o p -- python3 -u tools/ref_bench.py --taps --reps 1 --check 0 > $D/$1.log 2>&1 || { echo "pmc $1 failed"; tail -5 $D/$1.log; exit 1; }
  python3 tools/pmc_stats.py $D/$1/p_results.db | grep -E "kernel  |pwref" > $D/$1.txt && cut -c1-40,70-170 $D/$1.txt
}
export FLR_TAP_WR=4
run f "FETCH_SIZE" && run w "WRITE_SIZE" &&
run l "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_BUSY_CYCLES"
