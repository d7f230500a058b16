#!/bin/bash
# round 6: the software-pipelined GEMM loop (FLR_GEMM_PP=1) — per-layer conv and
# encoder-GEMM timings against the shipped loop, then C3 rounds (sha must not move)
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 300 python -u tools/conv_bench.py --reps 5 --variants "FLR_GEMM_PP=1;FLR_GEMM_PP=2" > $O/conv.txt 2>&1 || { echo "conv failed"; tail -5 $O/conv.txt; exit 1; }
cat $O/conv.txt | tail -20
timeout -k 10 300 python -u tools/bgemm_bench.py --variants "FLR_GEMM_PP=1;FLR_GEMM_PP=2" > $O/bgemm.txt 2>&1 || { echo "bgemm failed"; tail -5 $O/bgemm.txt; exit 1; }
cat $O/bgemm.txt | tail -16
for v in 2; do
  FLR_GEMM_PP=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { echo "bench $v failed"; tail -5 $O/c3_$v.err; exit 1; }
  python - $O/c3_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("pp=" + sys.argv[2], round(d["value"], 3), "rounds/s", round(d["ms_per_step"], 2), "ms", "train", round(d["train_ms_per_round"], 2), "sha", d["global_sha256"][:16], d["sha_matches_reference_run"])
PY
done
