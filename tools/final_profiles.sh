#!/bin/bash
# Round-end artifacts: the default bench line (with the CPU baseline) and a
# rocprofv3 kernel-trace summary of a short bench run.  Outputs under gpurun_out/.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pf -o f -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /root/repo/gpurun_out/prof_final.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pf/f_results.db > gpurun_out/prof_final_stats.txt || exit $?
head -5 gpurun_out/prof_final_stats.txt
