#!/bin/bash
# round 6: the optimizer's and clip-norm's float4 ranges in predicated 8-deep groups
# (no one-at-a-time tail) — C3 A/B against the previous library (abl/base), the
# global model's sha unchanged, and a kernel trace of each
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
run() {
  env $1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_$2.json 2> $O/c3_$2.err || { echo "bench $2 failed"; tail -5 $O/c3_$2.err; exit 1; }
  python - $O/c3_$2.json $2 <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms", "train", round(d["train_ms_per_round"], 2), "agg", round(d["aggregate_ms"], 2), "sha", d["global_sha256"][:16], d["sha_matches_reference_run"])
PY
}
for r in 1 2; do
  run FLR_LIB=abl/base/libflr.so base_$r || exit 1
  run FLR_SGD_PT=1 new_$r || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base new; do
  L=multimodal-fl-security_amd/lib/libflr.so; [ $v = base ] && L=abl/base/libflr.so
  FLR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r6o_$v -o t -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  python3 tools/rocpd_stats.py $(ls /tmp/r6o_$v/*/t_results.db /tmp/r6o_$v/t_results.db 2>/dev/null | head -1) > $O/stats_$v.txt || exit 1
  grep -E "sgd_blocked|sumsq_blocked" $O/stats_$v.txt | cut -c1-150
done
