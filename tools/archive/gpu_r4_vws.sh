#!/bin/bash
# ViT weight-gradient stream: the ViT+BERT trainer tests and the C4 / C5 round tests, then C4 / C5 A/B
# (FLR_WGRAD_STREAM=0 vs on).
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/vws
timeout -k 10 600 python -u -m pytest tests/test_gpu_native_trainer.py tests/test_gpu_configs.py tests/test_gpu_xfmr.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/vws/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/vws/tests.log; exit 1; }
tail -1 gpurun_out/vws/tests.log
for C in C4 C5; do
  for W in 0 1; do
    FLR_WGRAD_STREAM=$W timeout -k 10 300 python3 -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/vws/b_${C}_$W.log 2>&1 || { echo "bench $C $W rc=$?"; tail -20 gpurun_out/vws/b_${C}_$W.log; exit 1; }
    echo "$C wgrad=$W $(grep -o '"value": [0-9.]*' gpurun_out/vws/b_${C}_$W.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/vws/b_${C}_$W.log)"
  done
done
