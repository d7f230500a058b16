#!/bin/bash
# round 6 profiles of the shipped library: C3 with the side streams off (per-kernel
# durations for conv_mfma), C3 at K = 16 (one GPU's share at G = 8), C4.  The
# rocpd databases are summarised on the box and deleted (gpurun_out <= 64 MiB).
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
db() { ls $1/*/$2_results.db $1/$2_results.db 2>/dev/null | head -1; }
FLR_TEXT_STREAM=0 FLR_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r6l_serial -o s -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/serial.json 2> $O/serial.err || { echo "serial failed"; tail -5 $O/serial.err; exit 1; }
python3 tools/rocpd_stats.py $(db /tmp/r6l_serial s) > $O/c3_kernel_stats_serial.txt || exit 1
rm -rf /tmp/r6l_serial
timeout -k 10 300 python3 -u bench.py --clients 16 --steps 20 --warmup 5 --no-cpu-baseline > $O/k16.json 2> $O/k16.err || { echo "k16 failed"; tail -5 $O/k16.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r6l_k16 -o k -- python3 bench.py --clients 16 --steps 5 --warmup 2 --no-cpu-baseline > $O/k16p.json 2> $O/k16p.err || { echo "k16 prof failed"; tail -5 $O/k16p.err; exit 1; }
python3 tools/rocpd_stats.py $(db /tmp/r6l_k16 k) > $O/k16_kernel_stats.txt || exit 1
python3 tools/exclusive_time.py $(db /tmp/r6l_k16 k) --top 40 > $O/k16_exclusive.txt || exit 1
rm -rf /tmp/r6l_k16
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r6l_c4 -o c4 -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo "c4 failed"; tail -5 $O/c4.err; exit 1; }
python3 tools/rocpd_stats.py $(db /tmp/r6l_c4 c4) > $O/c4_kernel_stats.txt || exit 1
rm -rf /tmp/r6l_c4
ls -la $O
