#!/bin/bash
# GPU session driver: parity tests, then (only if pytest did not crash) the
# training-step timing and a rocprof kernel trace of one steady-state round.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider > gpurun_out/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ "${SKIP_PROFILE:-0}" = 1 ] && exit $rc
timeout -k 10 300 python tools/train_step_bench.py > gpurun_out/tsb.log 2>&1 || exit $?
cat gpurun_out/tsb.log
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/pr -o r -- python3 tools/profile_round.py > gpurun_out/prof_round.log 2>&1 || exit $?
python3 tools/rocpd_stats.py /tmp/pr/r_results.db --after-last orderstat_kernel > gpurun_out/prof_round_stats.txt
python3 tools/cgemm_calls.py /tmp/pr/r_results.db > gpurun_out/cgemm_calls.txt
exit $rc
