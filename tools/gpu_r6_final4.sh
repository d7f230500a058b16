#!/bin/bash
# round 6 final (the committed library): -m gpu suite, smoke, C3 and C5 bench lines, C3 kernel summary
set -o pipefail
O=gpurun_out/r6f4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread --ignore=tests/test_gpu_shard.py --ignore=tests/test_gpu_configs.py > $O/gpu_tests_a.log 2>&1 || { echo "gpu tests a failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests_a.log | head -20; exit 1; }
tail -1 $O/gpu_tests_a.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests_shard.log 2>&1 || { echo "shard tests failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests_shard.log | head -20; exit 1; }
tail -1 $O/gpu_tests_shard.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -m gpu --timeout 500 --timeout-method thread > $O/gpu_tests_configs.log 2>&1 || { echo "config tests failed"; grep -E "^E |FAILED|passed|failed" $O/gpu_tests_configs.log | head -20; exit 1; }
tail -1 $O/gpu_tests_configs.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/c3_bench.json 2> $O/c3_bench.err || { echo "c3 bench failed"; tail -5 $O/c3_bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c3_bench.json').read().strip().splitlines()[-1]); print('C3', d['value'], d.get('sha_matches_reference_run'), d['roofline']['frac'])"
timeout -k 10 500 python -u bench.py --config C5 --steps 2 --warmup 1 > $O/c5_bench.json 2> $O/c5_bench.err || { echo "c5 bench failed"; tail -5 $O/c5_bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c5_bench.json').read().strip().splitlines()[-1]); print('C5', d['value'], {k: v for k, v in d.items() if 'aggregate' in k or 'distance' in k})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r6f4_c3 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || { echo "prof failed"; tail -5 $O/prof_c3.err; exit 1; }
python3 tools/rocpd_stats.py $(ls /tmp/r6f4_c3/*/c3_results.db /tmp/r6f4_c3/c3_results.db 2>/dev/null | head -1) > $O/c3_kernel_stats.txt || exit 1
head -8 $O/c3_kernel_stats.txt | cut -c1-140
