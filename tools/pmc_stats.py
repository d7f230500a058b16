"""Per-kernel mean of a PMC counter from a rocprofv3 rocpd .db (counters_collection)."""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
q = ("select kernel_name, counter_name, count(distinct dispatch_id), sum(value)/count(distinct dispatch_id), "
     "avg(duration) from counters_collection group by kernel_name, counter_name order by 4 desc")
print(f"{'kernel':70s} {'counter':12s} {'dispatches':>10s} {'value/dispatch':>16s} {'avg_dur_us':>10s}")
for k, cn, n, v, d in c.execute(q):
    print(f"{k[:70]:70s} {cn:12s} {n:10d} {v:16.1f} {d/1e3 if d else 0:10.2f}")
