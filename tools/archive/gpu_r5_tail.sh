#!/bin/bash
# kernel trace of C3 rounds on the final library (the end-of-backward tail)
set -o pipefail
D=gpurun_out/r5tail; mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d $D/prof -o p -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > $D/prof.log 2>&1 || { echo "prof failed"; tail -5 $D/prof.log; exit 1; }
python3 - <<'PY' > $D/tail.txt
import sqlite3, re
c=sqlite3.connect('gpurun_out/r5tail/prof/p_results.db')
rows=sorted(c.execute("select start,end,name,stream_id from kernels"))
sg=[r for r in rows if 'sgd_blocked' in r[2]]
for s0 in sg[6:9]:
    t=s0[0]
    for r in [r for r in rows if r[1] > t-2.5e6 and r[0] <= t]:
        print("%9.1f %9.1f %7.1f s%s %s" % ((r[0]-t)/1e3, (r[1]-t)/1e3, (r[1]-r[0])/1e3, r[3], re.sub(r"\(.*","",r[2]).replace("void ","")[:70]))
    print()
PY
rm -rf $D/prof
wc -l $D/tail.txt
