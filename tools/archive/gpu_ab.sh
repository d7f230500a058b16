#!/bin/bash
set -u
cd "$(dirname "$0")/.."
timeout -k 10 500 python -u tools/round_ab.py "$@" > gpurun_out/round_ab.txt 2>&1
