#!/bin/bash
# round 6: the 8-wave ping-pong batched GEMM (ppgemm_kernel, FLR_GEMM_PP8=1):
# bit-identity against the 4-wave form, then the encoder-GEMM timings A/B
set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bgemm.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "^E |FAILED|passed|failed|Error" $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u tools/bgemm_bench.py --variants "FLR_GEMM_PP8=1;FLR_GEMM_PP8=2;FLR_GEMM_PP8=3" > $O/bgemm.txt 2>&1 || { echo "bgemm failed"; tail -5 $O/bgemm.txt; exit 1; }
cat $O/bgemm.txt | tail -30
