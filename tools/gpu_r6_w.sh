#!/bin/bash
# round 6: C3 rounds with FLR_GEMM_SPRIO=1 (odd-XCD-slot GEMM workgroups at static
# priority 1) against the default, alternating, sha checked
set -o pipefail
O=gpurun_out/r6w
mkdir -p $O
for r in 1 2 3; do for v in 0 1; do
  FLR_GEMM_SPRIO=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_sprio${v}_$r.json 2> $O/c3_sprio${v}_$r.err || { echo "bench $v failed"; tail -5 $O/c3_sprio${v}_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c3_sprio${v}_$r.json').read().strip().splitlines()[-1]); print('sprio=$v', round(d['value'],3), d.get('sha_matches_reference_run'))"
done; done
