"""Summarise a rocprofv3 rocpd .db: per-kernel count / total / avg duration.
usage: rocpd_stats.py DB [--after-last SUBSTRING]  (only dispatches after the
last dispatch whose kernel name contains SUBSTRING)"""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
where = ""
if "--after-last" in sys.argv:
    marker = sys.argv[sys.argv.index("--after-last") + 1]
    t = c.execute(f"select max(start) from kernels where {name_col} like ?", (f"%{marker}%",)).fetchone()[0]
    where = f"where start > {t}"
    span = c.execute(f"select min(start), max(end) from kernels {where}").fetchone()
    print(f"window after last '{marker}': {(span[1]-span[0])/1e6:.3f} ms wall")
q = (f"select {name_col}, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
     f"from kernels {where} group by {name_col} order by sum(end-start) desc")
rows = list(c.execute(q))
tot = sum(r[2] for r in rows)
print(f"sum of kernel time: {tot/1e6:.3f} ms")
print(f"{'kernel':90s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
for name, n, s, avg, mn, mx in rows:
    print(f"{name[:90]:90s} {n:6d} {s/1e6:10.3f} {avg/1e3:10.2f} {mn/1e3:9.2f} {mx/1e3:9.2f} {100*s/tot:6.1f}")
