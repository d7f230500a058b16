#!/bin/bash
# the per-GPU share at G = 8: C3 with 16 clients on one GPU — bench line and kernel trace
set -o pipefail
D=gpurun_out/r5k16; mkdir -p $D
timeout -k 10 300 python -u bench.py --clients 16 --no-cpu-baseline > $D/k16.json 2> $D/k16.err || { echo "bench failed"; tail -20 $D/k16.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/k16.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['train_ms_per_round'], d['aggregate_ms'])"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o p -- python3 -u bench.py --clients 16 --no-cpu-baseline --steps 3 --warmup 1 > $D/prof.log 2>&1 || { echo "prof failed"; tail -20 $D/prof.log; exit 1; }
python3 tools/rocpd_stats.py $D/prof/p_results.db > $D/stats.txt && head -20 $D/stats.txt | cut -c1-60,90-160
