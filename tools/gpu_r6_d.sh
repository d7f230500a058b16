#!/bin/bash
# round 6: training order at G > 1 for the reference-exact Krum distances
# (tap-block-aligned rank boundaries) — the sharded-round tests, then C3 at
# 2 and 4 gloo ranks on the one GPU (25 rounds: global_sha256 against the
# one-GPU reference run)
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_shard.py > $O/tests_shard.log 2>&1 || { echo "shard tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests_shard.log | head -30; exit 1; }
tail -1 $O/tests_shard.log
for n in 2 4; do
  timeout -k 10 600 python -u bench.py --gpus $n --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_n$n.json 2> $O/c3_n$n.err || { echo "n$n failed"; tail -30 $O/c3_n$n.err; exit 1; }
  python - $O/c3_n$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n", d["n_gpus"], round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 1), "ms", "sha", d["global_sha256"][:16], "match", d["sha_matches_reference_run"], "dist", (d.get("distance_phase") or {}).get("ms"))
PY
done
