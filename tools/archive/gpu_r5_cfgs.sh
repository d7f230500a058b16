#!/bin/bash
# C2 / C4 / C5 default bench lines on the final library
set -o pipefail
D=gpurun_out/r5cfgs; mkdir -p $D
for c in C2 C4 C5; do
  timeout -k 10 500 python -u bench.py --config $c > $D/$c.json 2> $D/$c.err || { echo "bench $c failed"; tail -20 $D/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d.get('aggregate_ms'), d.get('aggregate_ms_by_defense'))"
done
