#!/bin/bash
# round 6: the packed-subtraction chain kernel (A/B against the round-5 library),
# its parity tests, the trimmed-mean cascade and the C3/C4/C5 config tests
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export FLR_RECORD_DIR=$O/records
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_pairwise_reference.py tests/test_gpu_aggregation.py > $O/tests_ref_agg.log 2>&1 || { echo "ref/agg tests failed"; tail -30 $O/tests_ref_agg.log; exit 1; }
tail -2 $O/tests_ref_agg.log
for v in old new old new; do
  if [ $v = new ]; then L=multimodal-fl-security_amd/lib/libflr.so; else L=abl/ref_old/libflr.so; fi
  FLR_LIB=$L timeout -k 10 120 python -u tools/ref_bench.py --taps --reps 5 --check 16 > $O/ref_$v.json 2> $O/ref_$v.err || { echo "$v failed"; tail -5 $O/ref_$v.err; exit 1; }
  echo "$v $(cat $O/ref_$v.json)"
done
timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread tests/test_gpu_configs.py > $O/configs.log 2>&1 || { echo "configs failed"; grep -E "^E |FAILED|passed|failed" $O/configs.log | head -20; exit 1; }
tail -2 $O/configs.log
