#!/bin/bash
# round-5 final library: the whole -m gpu suite (two processes), smoke(), the default bench line
set -o pipefail
sed 's#r5full#r5final3#g' tools/archive/gpu_r5_full.sh > /tmp/final.sh && bash /tmp/final.sh || exit $?
D=gpurun_out/r5final3
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python -u bench.py > $D/c3_default.json 2> $D/c3_default.err || { echo "bench failed"; tail -20 $D/c3_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/c3_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['aggregate_ms'], d['roofline']['frac'], d['roofline'].get('one_wave_issue_frac'))"
