#!/bin/bash
# C3 end to end at world 2 (gloo ranks on one GPU: the coordinate exchange and the
# reference-exact chains handed rank to rank) against world 1: the same global sha
set -o pipefail
mkdir -p gpurun_out/r5w
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r5w/n1.json 2> gpurun_out/r5w/n1.err || { echo "n1 failed"; tail -20 gpurun_out/r5w/n1.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r5w/n2.json 2> gpurun_out/r5w/n2.err || { echo "n2 failed"; tail -30 gpurun_out/r5w/n2.err; exit 1; }
python3 -c "
import json
a=json.loads(open('gpurun_out/r5w/n1.json').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/r5w/n2.json').read().strip().splitlines()[-1])
print('n1', a['value'], a['global_sha256'], a['config']['exchange']); print('n2', b['value'], b['global_sha256'], b['config']['exchange'], b['process_group'])
print('identical', a['global_sha256'] == b['global_sha256'])"
