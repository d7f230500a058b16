#!/bin/bash
# Round 3: PMC HBM traffic of the Gram kernel at the C3 bench shape (non-temporal DMA), separate FETCH_SIZE / WRITE_SIZE passes.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  K=128 P=11800394 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d /tmp/pmc_$C -o p -- python3 tools/pairwise_only.py > gpurun_out/pmc_$C.log 2>&1 || exit $?
  python3 tools/pmc_stats.py /tmp/pmc_$C/p_results.db > gpurun_out/pmc_gram_$C.txt 2>&1
  head -4 gpurun_out/pmc_gram_$C.txt
done
python3 - <<'PY'
import json, re
def val(path):
    for line in open(path):
        if "gram_partials_kernel" in line:
            return float(line.split()[-2])
f = val("gpurun_out/pmc_gram_FETCH_SIZE.txt"); w = val("gpurun_out/pmc_gram_WRITE_SIZE.txt")
json.dump({"kernel": "gram_partials_kernel", "K": 128, "P": 11800394, "fetch_kib": f, "write_kib": w,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tools/pairwise_only.py K=128 P=11800394"},
          open("gpurun_out/gram_traffic.json", "w"), indent=1)
print("traffic GB per launch:", (2 * f + w) * 1024 / 1e9)
