#!/bin/bash
# Round 3: flr_train_vit_bert (the C4/C5 family's one-call trainer) — bit identity with
# the Python trainer and the oracle loop; C4/C5 round tests through it; the C4 bench
# line (native vs FLR_TRAINER=python) and its rocprofv3 kernel summary.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_trainer.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_vit_native_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_round.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r3_vit_round_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r3_bench_c4.json 2> gpurun_out/r3_bench_c4.err || exit 1
FLR_TRAINER=python timeout -k 10 400 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r3_bench_c4_python.json 2> gpurun_out/r3_bench_c4_python.err || exit 1
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/pc4 -o b -- python3 "$GRAFT_REPO_ROOT/bench.py" --config C4 --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_c4.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python3 tools/rocpd_stats.py /tmp/pc4/b_results.db > gpurun_out/r3_c4_kernel_stats.txt
