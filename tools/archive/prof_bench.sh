# rocprofv3 kernel trace of a short bench run -> per-kernel summary
# usage: CLIENTS=128 bash tools/archive/prof_bench.sh
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pb -o b -- python3 /root/repo/bench.py --steps 3 --warmup 1 --no-cpu-baseline --clients ${CLIENTS:-128} > /root/repo/gpurun_out/prof_bench.log 2>&1 || exit $?
cd /root/repo && python3 tools/rocpd_stats.py /tmp/pb/b_results.db > gpurun_out/prof_bench_stats.txt
head -45 gpurun_out/prof_bench_stats.txt
