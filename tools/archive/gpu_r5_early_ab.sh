#!/bin/bash
# early text/head clip partials: alternating A/B of the C3 round time (base = the previous library)
set -o pipefail
D=gpurun_out/r5earlyab; mkdir -p $D
for i in 1 2 3 4; do
  for v in base new; do
    lib=multimodal-fl-security_amd/lib/libflr.so; [ $v = base ] && lib=abl/base/libflr.so
    FLR_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $D/$v$i.json 2> $D/$v$i.err || { echo "bench $v failed"; tail -20 $D/$v$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$D/$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],3), round(d['train_ms_per_round'],2), round(d['aggregate_ms'],2))"
  done
done
