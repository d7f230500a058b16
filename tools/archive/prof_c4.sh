#!/bin/bash
# rocprofv3 kernel summary of C4-shaped rounds (fewer clients: same per-client kernels)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c4
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 -- \
  python3 bench.py --config C4 --clients ${CLIENTS:-64} --steps 1 --warmup 1 > gpurun_out/prof_c4/bench.json 2> gpurun_out/prof_c4/bench.err
echo rc=$? >> gpurun_out/prof_c4/bench.err
