#!/bin/bash
# x_i delivery variants of the reference-exact chain kernel (same box), then the
# native trainer's per-step parity test
set -o pipefail
mkdir -p gpurun_out/r5d
for v in default xi2_cs32 xi2_cs64 xi3_cs32 xi3_cs64 xi0_cs64; do
  if [ $v = default ]; then L=multimodal-fl-security_amd/lib/libflr.so; else L=abl/$v/libflr.so; fi
  FLR_LIB=$L timeout -k 10 120 python -u tools/ref_bench.py --reps 5 --check 16 > gpurun_out/r5d/$v.json 2> gpurun_out/r5d/$v.err || { echo "$v failed"; tail -5 gpurun_out/r5d/$v.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r5d/$v.json'));print(round(d['ms_median'],2), d['mismatches'])")"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread "tests/test_gpu_native_trainer.py::test_native_trainer_matches_reference_loop" > gpurun_out/r5d/native.log 2>&1 || { echo "native failed"; tail -30 gpurun_out/r5d/native.log; exit 1; }
tail -2 gpurun_out/r5d/native.log
