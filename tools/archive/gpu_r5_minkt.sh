#!/bin/bash
# conv split-K floor (FLR_CONV_MINKT: fewest K-tiles per split part; 32 default) — C3 timing only
set -o pipefail
D=gpurun_out/r5minkt; mkdir -p $D
for v in 32 64 128 16; do
  FLR_CONV_MINKT=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8 --warmup 2 > $D/m$v.json 2> $D/m$v.err || { echo "bench $v failed"; tail -20 $D/m$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/m$v.json').read().strip().splitlines()[-1]); print('minkt $v', round(d['value'],3), round(d['train_ms_per_round'],2), round(d['aggregate_ms'],2))"
done
