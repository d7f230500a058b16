#!/bin/bash
# Round 3: the half-phase split-at-stash schedule (abl/half, -DFLR_SG_HALF=1) against
# the in-tree library: bit-identity of a C3 and a C4-shaped round, conv / GEMM
# timings, the conv + GEMM GPU tests under the variant, C3 bench per library.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
MAIN=$PWD/multimodal-fl-security_amd/lib/libflr.so
ALT=$PWD/abl/${ALTNAME:-half}/libflr.so
FLR_LIB=$MAIN timeout -k 10 300 python -u tools/lib_identity.py > gpurun_out/y_id_main.txt 2>&1 || exit 1
FLR_LIB=$ALT timeout -k 10 300 python -u tools/lib_identity.py > gpurun_out/y_id_alt.txt 2>&1 || exit 1
grep -E "^c[34]" gpurun_out/y_id_main.txt gpurun_out/y_id_alt.txt
for n in main alt; do
  if [ $n = main ]; then lib=$MAIN; else lib=$ALT; fi
  FLR_LIB=$lib timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/y_conv_$n.txt 2>&1 || exit 1
  FLR_LIB=$lib ONLY=vit timeout -k 10 300 python -u tools/bgemm_bench.py > gpurun_out/y_bgemm_$n.txt 2>&1 || exit 1
done
FLR_LIB=$ALT timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py tests/test_gpu_bgemm.py > gpurun_out/y_tests_alt.txt 2>&1 || exit 1
tail -3 gpurun_out/y_tests_alt.txt
for n in main alt; do
  if [ $n = main ]; then lib=$MAIN; else lib=$ALT; fi
  FLR_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/y_bench_$n.json 2> gpurun_out/y_bench_$n.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/y_bench_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],2), 'ms/round')"
done
tail -1 gpurun_out/y_conv_main.txt gpurun_out/y_conv_alt.txt
