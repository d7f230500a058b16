import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
t = c.execute(f"select max(start) from kernels where {name} like '%orderstat%'").fetchone()[0]
rows = c.execute(f"select {name}, end-start from kernels where start > ? order by start", (t,)).fetchall()
print("kernels in round:", len(rows), "total us", sum(r[1] for r in rows)/1e3)
from collections import Counter
cnt = Counter(); tim = Counter()
for i, (n, d) in enumerate(rows):
    if n.startswith("void at::") or n.startswith("at::"):
        prev = rows[i-1][0][:50] if i else ""
        key = (n[:70], prev)
        cnt[key] += 1; tim[key] += d/1e3
for k, v in sorted(tim.items(), key=lambda x: -x[1])[:25]:
    print(f"{v:8.1f} us {cnt[k]:4d}x  {k[0]}  <- after {k[1]}")
