#!/bin/bash
# round 6: timing ablations of ref_chain_s_kernel (abl/s1..s4: no x_j loads,
# no x_i loads, no arithmetic, x_i never waited for) at K=512 P=2M, 8 and 4 rows
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
for rows in 8 4; do for a in 0 1 2 3 4; do
  lib=multimodal-fl-security_amd/lib/libflr.so; [ $a != 0 ] && lib=abl/s$a/libflr.so
  FLR_LIB=$lib FLR_REF_SGPR=1 FLR_REF_SGPR_ROWS=$rows timeout -k 10 120 python -u tools/ref_bench.py --K 512 --P 2000003 --reps 3 --check 0 > $O/r${rows}_a$a.json 2> $O/r${rows}_a$a.err || { echo "r$rows a$a failed"; tail -5 $O/r${rows}_a$a.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r${rows}_a$a.json')); print('rows $rows abl $a', round(d['ms_median'],3))"
done; done
