#!/bin/bash
# Round-2 final artifacts: GPU test suite, default bench line (CPU baseline), rocprofv3 kernel
# summary of a short bench, C2/C4/C5 lines, C4/C5 aggregation timings.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/gpu_tests_final.log; tail -2 gpurun_out/gpu_tests_final.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /root/repo/gpurun_out/prof_final.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/prof_final_stats.txt || exit $?
for c in C2 C4 C5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 > gpurun_out/bench_final_$c.json 2> gpurun_out/bench_final_$c.err || exit 1
done
timeout -k 10 400 python -u tools/agg_c4c5.py > gpurun_out/agg_final.txt 2>&1 || exit 1
python3 -c "
import json
for n in ('bench_final','bench_final_C2','bench_final_C4','bench_final_C5'):
    d=json.loads(open('gpurun_out/%s.json'%n).read().strip().splitlines()[-1]); print(n, round(d['value'],4), round(d['ms_per_step'],2))"
