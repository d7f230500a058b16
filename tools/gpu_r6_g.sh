#!/bin/bash
# round 6: the deferred dead-tap fill throttled (FLR_FILL_GRID workgroups per row)
# beside the Krum chains: C3 A/B against FLR_DEFER_DEAD=0, then a kernel trace
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
run() {
  env $1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_$2.json 2> $O/c3_$2.err || { echo "bench $2 failed"; tail -5 $O/c3_$2.err; exit 1; }
  python - $O/c3_$2.json $2 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms", "train", round(d["train_ms_per_round"], 2), "agg", round(d["aggregate_ms"], 2), "dist", round(d["distance_phase"]["ms"], 2), "sha", d["global_sha256"][:16], d["sha_matches_reference_run"])
PY
}
for r in 1 2; do
  run FLR_DEFER_DEAD=0 d0_$r || exit 1
  run FLR_FILL_GRID=1 g1_$r || exit 1
  run FLR_FILL_GRID=4 g4_$r || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FLR_FILL_GRID=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
