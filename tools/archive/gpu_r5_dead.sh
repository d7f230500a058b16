#!/bin/bash
# X's dead-tap ranges written on the weight-gradient stream under the first
# forward: trainer / round / config tests, the 25-round C3 sha, the default line
set -o pipefail
D=gpurun_out/r5dead; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_native_trainer.py tests/test_gpu_round.py tests/test_gpu_configs.py tests/test_gpu_train.py > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $D/c3_25.json 2> $D/c3_25.err || { echo "bench25 failed"; tail -20 $D/c3_25.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c3_25.json').read().strip().splitlines()[-1]); print(d['value'], d['train_ms_per_round'], d['aggregate_ms'], d['global_sha256'][:12], d['sha_matches_reference_run'])"
timeout -k 10 300 python -u bench.py > $D/c3_default.json 2> $D/c3_default.err || { echo "bench failed"; tail -20 $D/c3_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c3_default.json').read().strip().splitlines()[-1]); print(d['value'], d['train_ms_per_round'], d['aggregate_ms'])"
