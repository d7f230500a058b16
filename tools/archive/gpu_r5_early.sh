#!/bin/bash
# the text branch's and head's clip-norm partials on the text stream: trainer /
# round / config tests, the 25-round C3 sha and timing (alternating with the
# previous library, abl/base), the sumsq kernel's time
set -o pipefail
D=gpurun_out/r5early; mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_native_trainer.py tests/test_gpu_round.py tests/test_gpu_train.py tests/test_gpu_configs.py > $D/tests.log 2>&1 || { echo "tests failed"; tail -30 $D/tests.log; exit 1; }
tail -1 $D/tests.log
for v in new base new base; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $v = base ] && lib=abl/base/libflr.so
  FLR_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $D/$v.json 2> $D/$v.err || { echo "bench $v failed"; tail -20 $D/$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],3), round(d['train_ms_per_round'],2), d['global_sha256'][:12], d['sha_matches_reference_run'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o p -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/prof.log 2>&1 || { echo "prof failed"; exit 1; }
python3 tools/rocpd_stats.py $D/prof/p_results.db | grep -E "sumsq|clip_coef" | cut -c1-50,90-160
