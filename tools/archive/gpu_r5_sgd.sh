#!/bin/bash
# SGD workgroups per client (FLR_SGD_NWG): C3 bench line and the sgd kernel's time per form
set -o pipefail
D=gpurun_out/r5sgd; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for n in 256 64 128 512 1024; do
  FLR_SGD_NWG=$n timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/p$n -o p -- python3 -u bench.py --steps 3 --warmup 1 > $D/b$n.log 2>&1 || { echo "run $n failed"; tail -20 $D/b$n.log; exit 1; }
  python3 tools/rocpd_stats.py $D/p$n/p_results.db > $D/s$n.txt
  echo "nwg $n $(grep -E 'sgd_blocked' $D/s$n.txt | cut -c90-160) | $(grep -o '"value": [0-9.]*' $D/b$n.log)"
done
