#!/bin/bash
# the whole -m gpu suite in two processes (as the driver runs it, split for the call limit), then smoke()
set -o pipefail
mkdir -p gpurun_out/r5full
A="tests/test_gpu_aggregation.py tests/test_gpu_bgemm.py tests/test_gpu_bgemm_dma.py tests/test_gpu_bn.py tests/test_gpu_conv.py tests/test_gpu_defenses_ext.py tests/test_gpu_eval.py tests/test_gpu_fltrust.py tests/test_gpu_gru.py tests/test_gpu_krum_c3.py"
B="tests/test_gpu_native_trainer.py tests/test_gpu_pairwise_reference.py tests/test_gpu_pool.py tests/test_gpu_round.py tests/test_gpu_sgd_phase.py tests/test_gpu_train.py tests/test_gpu_xfmr.py tests/test_gpu_shard.py tests/test_gpu_configs.py"
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 600 --timeout-method thread $A > gpurun_out/r5full/a.log 2>&1; ra=$?
tail -3 gpurun_out/r5full/a.log
[ $ra -eq 0 ] || [ $ra -eq 1 ] || exit $ra
timeout -k 10 1100 python -u -m pytest -m gpu -q --timeout 600 --timeout-method thread $B > gpurun_out/r5full/b.log 2>&1; rb=$?
tail -3 gpurun_out/r5full/b.log
[ $rb -eq 0 ] || [ $rb -eq 1 ] || exit $rb
grep -E "^FAILED|^ERROR" gpurun_out/r5full/a.log gpurun_out/r5full/b.log | head -20
exit $(( ra + rb ))
