#!/bin/bash
# round 6 final artifacts: the -m gpu suite, smoke, the C3 bench line and its
# rocprofv3 kernel summary, the PMC traffic of the reference distance phase
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 850 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests.log | head -20; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail -5 $O/bench_c3.err; exit 1; }
tail -c 600 $O/bench_c3.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_$C -o p -- python3 tools/ref_bench.py --taps --reps 1 --check 0 > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $O/pmc_$C.log; exit 1; }
  db=$(ls $O/pmc_$C/*/p_results.db $O/pmc_$C/p_results.db 2>/dev/null | head -1)
  python3 tools/pmc_stats.py $db > $O/pmc_ref_$C.txt 2>&1 || { echo "pmc stats failed"; exit 1; }
  grep -E "pwref" $O/pmc_ref_$C.txt | head -8
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -5 $O/prof_c3.err; exit 1; }
ls $O/prof
