#!/bin/bash
# the whole -m gpu suite on the zero-filled-stream chain kernel, then the default bench line and its kernel summary
set -o pipefail
sed 's#r5full#r5full2#g' tools/archive/gpu_r5_full.sh > /tmp/full2.sh && bash /tmp/full2.sh || exit $?
mkdir -p gpurun_out/r5z
timeout -k 10 300 python -u bench.py > gpurun_out/r5z/c3_default.json 2> gpurun_out/r5z/c3_default.err || { echo "bench failed"; tail -20 gpurun_out/r5z/c3_default.err; exit 1; }
cat gpurun_out/r5z/c3_default.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5z/bprof -o p -- python3 -u bench.py --steps 3 --warmup 1 > gpurun_out/r5z/bprof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r5z/bprof.log; exit 1; }
python3 tools/rocpd_stats.py gpurun_out/r5z/bprof/p_results.db > gpurun_out/r5z/bench_stats.txt && head -12 gpurun_out/r5z/bench_stats.txt
