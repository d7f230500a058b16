#!/bin/bash
# the first residual blocks' weight gradients on the (idle) text stream: trainer /
# round tests, then alternating C3 timing for FLR_WG_TEXT = 0 / 1 / 2 with the sha
set -o pipefail
D=gpurun_out/r5wgtext3; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_native_trainer.py tests/test_gpu_round.py tests/test_gpu_configs.py -k "not c4 and not c5" > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for i in 1 2 3; do
  for n in 2 3 4; do
    FLR_WG_TEXT=$n timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 > $D/n$n.$i.json 2> $D/n$n.$i.err || { echo "bench $n failed"; tail -20 $D/n$n.$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$D/n$n.$i.json').read().strip().splitlines()[-1]); print('wg_text $n', round(d['value'],3), round(d['train_ms_per_round'],2), d['global_sha256'][:12])"
  done
done
