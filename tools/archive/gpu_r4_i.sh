#!/bin/bash
export TMPDIR=/tmp
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for st in 1 2; do
  timeout -k 10 400 python3 -u tools/diag_step0_fp64.py 32 0 3 $st > gpurun_out/r4i_fp64_s$st.txt 2>&1 || { echo "diag rc=$?"; tail -5 gpurun_out/r4i_fp64_s$st.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/r4i_fp64_s$st.txt | tail -13
done
