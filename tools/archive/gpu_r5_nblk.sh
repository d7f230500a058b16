#!/bin/bash
# clip-norm partial blocks per client (NBLK 32 -> 128, a variant library): C3 25-round sha + timing, alternating
set -o pipefail
D=gpurun_out/r5nblk; mkdir -p $D
for v in base nblk base nblk; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $v = nblk ] && lib=abl/nblk/libflr.so
  FLR_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $D/$v.json 2> $D/$v.err || { echo "bench $v failed"; tail -20 $D/$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],3), round(d['train_ms_per_round'],2), d['global_sha256'][:12], d['sha_matches_reference_run'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
FLR_LIB=abl/nblk/libflr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o p -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/rocpd_stats.py $D/prof/p_results.db | grep -E "sumsq|clip_coef" | cut -c1-50,90-160
