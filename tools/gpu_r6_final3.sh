#!/bin/bash
# round 6 final (part 2): the C3 bench line (with its CPU baseline), its
# rocprofv3 kernel summary, and the C2 / C4 / C5 lines
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail -5 $O/bench_c3.err; exit 1; }
tail -c 400 $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r6z_c3 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -5 $O/prof_c3.err; exit 1; }
python3 tools/rocpd_stats.py $(ls /tmp/r6z_c3/*/c3_results.db /tmp/r6z_c3/c3_results.db 2>/dev/null | head -1) > $O/c3_kernel_stats.txt || exit 1
rm -rf /tmp/r6z_c3
head -6 $O/c3_kernel_stats.txt | cut -c1-140
for c in C2 C4 C5; do
  s=5; w=2; [ $c = C4 ] && s=3 && w=1; [ $c = C5 ] && s=2 && w=1
  timeout -k 10 500 python -u bench.py --config $c --steps $s --warmup $w --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
  python - $O/bench_$c.json $c <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"], 4), "rounds/s", round(d["ms_per_step"], 1), "ms", "agg", round(d.get("aggregate_ms") or 0, 1), "dist", (d.get("distance_phase") or {}).get("ms"))
PY
done
