#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u tools/diag_fc1b.py > gpurun_out/r4c_diag_fc1b.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4c_diag_fc1b.txt
exit $rc
