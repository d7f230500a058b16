#!/bin/bash
# C3 bench lines: reference-exact Krum distances and the Gram path, the
# driver's command shape (--steps 20 --warmup 5)
set -o pipefail
mkdir -p gpurun_out/r5o
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --pairwise reference > gpurun_out/r5o/bench_ref.json 2> gpurun_out/r5o/bench_ref.err || { echo "bench ref failed"; tail -20 gpurun_out/r5o/bench_ref.err; exit 1; }
cat gpurun_out/r5o/bench_ref.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --pairwise gram --no-cpu-baseline > gpurun_out/r5o/bench_gram.json 2> gpurun_out/r5o/bench_gram.err || { echo "bench gram failed"; tail -20 gpurun_out/r5o/bench_gram.err; exit 1; }
cat gpurun_out/r5o/bench_gram.json
