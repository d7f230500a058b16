#!/bin/bash
# round 6: dead-tap ranges never written (FLR_DEFER_DEAD=2; distances and the
# Multi-Krum mean read them from the round's global vector) — parity, then C3
# A/B against the slabs written in training (=0), and a kernel trace
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_aggregation.py -k "dead" tests/test_gpu_round.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
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
  run FLR_DEFER_DEAD=2 d2_$r || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FLR_DEFER_DEAD=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r6r_p -o t -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
python3 tools/rocpd_stats.py $(ls /tmp/r6r_p/*/t_results.db /tmp/r6r_p/t_results.db 2>/dev/null | head -1) > $O/stats_d2.txt || exit 1
grep -E "rows_mean|dead_mean|dead_ranges|tap_chain_kernel<9|ref_chain" $O/stats_d2.txt | cut -c1-150
