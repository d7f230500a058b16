#!/bin/bash
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/diag_gate_flip.py 32 0 3 > gpurun_out/r4f_gate_flip.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4f_gate_flip.txt | tail -30
[ $rc -eq 0 ] || exit $rc
# the per-GPU share of C3 at G = 8 (16 clients on one GPU, no exchange): how the round scales down
timeout -k 10 300 python3 -u bench.py --clients 16 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r4f_bench_c3_k16.log 2>&1 || { echo "bench k16 rc=$?"; tail -5 gpurun_out/r4f_bench_c3_k16.log; exit 1; }
grep '^{"metric' gpurun_out/r4f_bench_c3_k16.log | cut -c1-300
