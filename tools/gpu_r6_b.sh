#!/bin/bash
# round 6: conv / batched-GEMM fragment reads ahead (FLR_FRAG_AHEAD) — A/B against
# the per-k-step reads (abl/frag0), same box, alternating; then the C3 round both ways
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
for v in new old new old; do
  if [ $v = new ]; then L=multimodal-fl-security_amd/lib/libflr.so; else L=abl/frag0/libflr.so; fi
  FLR_LIB=$L timeout -k 10 150 python -u tools/conv_bench.py --reps 5 > $O/conv_$v.txt 2>&1 || { echo "conv $v failed"; tail -5 $O/conv_$v.txt; exit 1; }
  FLR_LIB=$L timeout -k 10 150 python -u tools/bgemm_bench.py > $O/bgemm_$v.txt 2>&1 || { echo "bgemm $v failed"; tail -5 $O/bgemm_$v.txt; exit 1; }
  echo "== $v"; tail -3 $O/conv_$v.txt; tail -3 $O/bgemm_$v.txt
done
for v in new old new old; do
  if [ $v = new ]; then L=multimodal-fl-security_amd/lib/libflr.so; else L=abl/frag0/libflr.so; fi
  FLR_LIB=$L timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms", "sha", d.get("global_sha256", "")[:16], d.get("sha_matches_reference_run"))
PY
done
