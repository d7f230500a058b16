#!/bin/bash
# Round-4 final artifacts: the C3 bench line (with cpu_baseline), its rocprofv3 kernel summary, the Gram PMC
# traffic passes, and the K=16 per-GPU share of C3 at G=8.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/final
timeout -k 10 600 python3 -u bench.py > gpurun_out/final/bench_c3.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/final/bench_c3.log; exit 1; }
grep '^{"metric' gpurun_out/final/bench_c3.log > gpurun_out/final/r4_bench_c3_final.json
cut -c1-300 gpurun_out/final/r4_bench_c3_final.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pfin -o b -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/final/prof_c3.log" 2>&1 || { echo "prof rc=$?"; tail -10 "$R/gpurun_out/final/prof_c3.log"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pfin/b_results.db > gpurun_out/final/r4_c3_kernel_stats_final.txt 2>&1
head -12 gpurun_out/final/r4_c3_kernel_stats_final.txt | cut -c1-150
for C in FETCH_SIZE WRITE_SIZE; do
  K=128 P=11800394 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d /tmp/pmc_$C -o p -- python3 tools/pairwise_only.py > gpurun_out/final/pmc_$C.log 2>&1 || { echo "pmc $C rc=$?"; exit 1; }
  python3 tools/pmc_stats.py /tmp/pmc_$C/p_results.db > gpurun_out/final/r4_gram_pmc_$C.txt 2>&1
  grep gram_partials gpurun_out/final/r4_gram_pmc_$C.txt | cut -c1-160
done
timeout -k 10 300 python3 -u bench.py --clients 16 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/final/bench_c3_k16.log 2>&1 || { echo "k16 rc=$?"; exit 1; }
grep '^{"metric' gpurun_out/final/bench_c3_k16.log > gpurun_out/final/r4_bench_c3_k16.json
grep -o '"ms_per_step": [0-9.]*' gpurun_out/final/r4_bench_c3_k16.json
