#!/bin/bash
# round 6: two chains per lane for K >= 256 (ref_chain2_kernel) — parity, then
# A/B against the one-chain form (FLR_REF_2I=0) at K = 512 and on the C5 round
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py > $O/tests_ref.log 2>&1 || { echo "ref tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests_ref.log | head -20; exit 1; }
tail -1 $O/tests_ref.log
for v in 1 0 1 0; do
  FLR_REF_2I=$v timeout -k 10 200 python -u tools/ref_bench.py --K 512 --P 2000003 --reps 3 --check 8 > $O/ref_K512_2i$v.json 2> $O/ref_K512_2i$v.err || { echo "K512 $v failed"; tail -5 $O/ref_K512_2i$v.err; exit 1; }
  echo "2I=$v $(cat $O/ref_K512_2i$v.json)"
done
for v in 1 0; do
  FLR_REF_2I=$v timeout -k 10 200 python -u tools/ref_bench.py --K 256 --P 4000037 --reps 3 --check 8 > $O/ref_K256_2i$v.json 2> $O/ref_K256_2i$v.err || { echo "K256 $v failed"; tail -5 $O/ref_K256_2i$v.err; exit 1; }
  echo "K256 2I=$v $(cat $O/ref_K256_2i$v.json)"
done
for v in 1 0; do
  FLR_REF_2I=$v timeout -k 10 500 python -u bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c5_2i$v.json 2> $O/bench_c5_2i$v.err || { echo "C5 $v failed"; tail -5 $O/bench_c5_2i$v.err; exit 1; }
  python - $O/bench_c5_2i$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C5 2I=" + sys.argv[2], round(d["value"], 4), "rounds/s", round(d["ms_per_step"], 1), "ms", "agg", round(d.get("aggregate_ms", 0), 1), "sha", d.get("global_sha256", "")[:16], "dist", (d.get("distance_phase") or {}).get("ms"))
PY
done
