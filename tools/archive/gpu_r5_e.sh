#!/bin/bash
# timing ablations of the DPP chain kernel (tools builds; wrong results), then the native trainer's step test
set -o pipefail
mkdir -p gpurun_out/r5e
for v in xi0_cs64_abl0 xi0_cs64_abl1 xi0_cs64_abl2 xi0_cs64_abl3 xi0_cs64_abl4 xi1_cs32_abl0; do
  FLR_LIB=abl/$v/libflr.so timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 0 > gpurun_out/r5e/$v.json 2> gpurun_out/r5e/$v.err || { echo "$v failed"; tail -5 gpurun_out/r5e/$v.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r5e/$v.json'));print(round(d['ms_median'],2))")"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread "tests/test_gpu_native_trainer.py::test_native_trainer_matches_reference_loop" > gpurun_out/r5e/native.log 2>&1 || { echo "native failed"; tail -5 gpurun_out/r5e/native.log; }
tail -2 gpurun_out/r5e/native.log
