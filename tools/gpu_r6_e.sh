#!/bin/bash
# round 6: dead-tap slabs written beside the Krum chains (FLR_DEFER_DEAD) —
# parity, then C3 A/B against the slabs written last in training (=0), and a
# kernel-trace profile of the default
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_round.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  FLR_DEFER_DEAD=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_d$v.json 2> $O/c3_d$v.err || { echo "bench $v failed"; tail -5 $O/c3_d$v.err; exit 1; }
  python - $O/c3_d$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("defer=" + sys.argv[2], round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms", "train", round(d["train_ms_per_round"], 2), "agg", round(d["aggregate_ms"], 2), "dist", round(d["distance_phase"]["ms"], 2), "sha", d["global_sha256"][:16], d["sha_matches_reference_run"])
PY
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
