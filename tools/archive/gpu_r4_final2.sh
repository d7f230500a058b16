#!/bin/bash
# Round-4 final artifacts after the weight-gradient stream: full -m gpu suite + smoke, the C3 line (cpu_baseline),
# its rocprofv3 summary, a serial-stream summary (conv utilisation), the C2 line, and K=16/32/64 shares.
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/final2
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/final2/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/final2/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final2/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final2/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/final2/bench_c3.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/final2/bench_c3.log; exit 1; }
grep '^{"metric' gpurun_out/final2/bench_c3.log > gpurun_out/final2/r4_bench_c3_final.json
cut -c1-240 gpurun_out/final2/r4_bench_c3_final.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pf2 -o b -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/final2/prof_c3.log" 2>&1 || { echo "prof rc=$?"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pf2/b_results.db > gpurun_out/final2/r4_c3_kernel_stats_final.txt 2>&1
grep gram_partials gpurun_out/final2/r4_c3_kernel_stats_final.txt | cut -c1-150
cd /tmp && FLR_TEXT_STREAM=0 FLR_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pf3 -o b -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/final2/prof_c3_serial.log" 2>&1 || { echo "prof serial rc=$?"; exit 1; }
cd "$R" && python3 tools/rocpd_stats.py /tmp/pf3/b_results.db > gpurun_out/final2/r4_c3_kernel_stats_serial.txt 2>&1
timeout -k 10 500 python3 -u bench.py --config C2 --steps 10 --warmup 1 > gpurun_out/final2/bench_c2.log 2>&1 || { echo "c2 rc=$?"; exit 1; }
grep '^{"metric' gpurun_out/final2/bench_c2.log > gpurun_out/final2/r4_bench_c2.json
for KK in 16 32 64; do
  timeout -k 10 300 python3 -u bench.py --clients $KK --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/final2/k$KK.log 2>&1 || { echo "k$KK rc=$?"; exit 1; }
  grep '^{"metric' gpurun_out/final2/k$KK.log > gpurun_out/final2/r4_bench_c3_k$KK.json
  echo "K=$KK $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/final2/k$KK.log)"
done
grep -o '"value": [0-9.]*' gpurun_out/final2/r4_bench_c2.json | head -1
