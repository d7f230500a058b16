#!/bin/bash
# Native-trainer round: focused GPU tests, then bench A/B (native vs python trainer) and a kernel profile.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_round.py tests/test_gpu_native_trainer.py "tests/test_gpu_conv.py::test_dgrad_addend_bit_identical" \
  > gpurun_out/gpu_native_tests.log 2>&1 || { tail -30 gpurun_out/gpu_native_tests.log; exit 1; }
tail -3 gpurun_out/gpu_native_tests.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_native.json 2> gpurun_out/bench_native.err || exit $?
FLR_TRAINER=python timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bench_python.json 2> gpurun_out/bench_python.err || exit $?
python3 -c "
import json
for n in ('native','python'):
    d=json.load(open('gpurun_out/bench_%s.json'%n)); print(n, round(d['value'],3), round(d['ms_per_step'],2), round(d['train_ms_per_round'],2))"
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench_native.txt 2>&1 || exit $?
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /root/repo/gpurun_out/prof_native.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/prof_native_stats.txt
head -30 gpurun_out/prof_native_stats.txt
