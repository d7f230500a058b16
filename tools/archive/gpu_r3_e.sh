#!/bin/bash
# Round 3 checkpoint: the whole -m gpu suite, the default C3 bench line (incl. the CPU
# baseline), and a rocprofv3 kernel summary of the same bench.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3_bench_c3.json 2> gpurun_out/r3_bench_c3.err || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_c3.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/r3_c3_kernel_stats.txt
