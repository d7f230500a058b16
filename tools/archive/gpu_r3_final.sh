#!/bin/bash
# Round 3 final artifacts: the whole -m gpu suite, smoke(), the C3 bench line and its rocprofv3 kernel summary.
export TMPDIR=/tmp
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python -u tools/lib_identity.py > gpurun_out/r3f_identity.txt 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3f_gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3f_smoke.log 2>&1 || exit 1
bash tools/archive/gpu_r3_n.sh
