#!/bin/bash
# FLR_WG_MAIN: the first N residual blocks' weight gradients on the caller's stream
# (beside the weight-gradient stream's backlog at the end of the backward): C3 timing + sha
set -o pipefail
D=gpurun_out/r5wgmain; mkdir -p $D
for i in 1 2; do
  for n in 0 1 2 3; do
    FLR_WG_MAIN=$n timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $D/n$n.$i.json 2> $D/n$n.$i.err || { echo "bench $n failed"; tail -20 $D/n$n.$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$D/n$n.$i.json').read().strip().splitlines()[-1]); print('wg_main $n', round(d['value'],3), round(d['train_ms_per_round'],2), d['global_sha256'][:12])"
  done
done
