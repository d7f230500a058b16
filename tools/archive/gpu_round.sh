#!/bin/bash
# One GPU session: parity tests; then (unless pytest crashed) per-layer conv
# timing for both MFMA forms and the bench line.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?
tail -6 gpurun_out/pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ "${SKIP_BENCH:-0}" = 1 ] && exit $rc
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_x6.log 2>&1 || exit $?
FLR_GEMM=f32 timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_f32.log 2>&1 || exit $?
paste gpurun_out/conv_x6.log gpurun_out/conv_f32.log | tail -34
timeout -k 10 400 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
exit $rc
