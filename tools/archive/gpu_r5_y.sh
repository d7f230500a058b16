#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u tools/dbg_ref33.py 2>&1 | tail -6
