#!/bin/bash
# chain kernel over zero-filled streams (no per-chunk check): the small shapes,
# then the reference tests, timing, kernel summary and PMC pass (tools/archive/gpu_r5_n.sh)
set -o pipefail
mkdir -p gpurun_out/r5z
timeout -k 10 200 python -u tools/dbg_ref33.py > gpurun_out/r5z/dbg.log 2>&1 || { echo "dbg failed"; tail -20 gpurun_out/r5z/dbg.log; exit 1; }
grep "bad pairs" gpurun_out/r5z/dbg.log
grep -q "bad pairs [1-9]" gpurun_out/r5z/dbg.log && { echo "still bad"; exit 1; }
sed 's#r5n#r5z#g' tools/archive/gpu_r5_n.sh > gpurun_out/r5z/run.sh && bash gpurun_out/r5z/run.sh
