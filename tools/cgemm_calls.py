"""List conv (cgemm) dispatches of the last profiled round: name, grid, us.
usage: cgemm_calls.py DB"""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
gx = [x for x in ("grid_size_x", "grid_x", "workgroup_count_x") if x in cols]
gy = [x for x in ("grid_size_y", "grid_y") if x in cols]
gz = [x for x in ("grid_size_z", "grid_z") if x in cols]
print("columns:", cols)
t = c.execute(f"select max(start) from kernels where {name} like '%orderstat%'").fetchone()[0]
sel = ", ".join([name] + (gx[:1] + gy[:1] + gz[:1]) + ["end-start"])
rows = c.execute(f"select {sel} from kernels where start > ? and ({name} like '%gemm_kernel%' or {name} like '%im2col%' or {name} like '%reduce_kernel<flr::convt%' or {name} like '%repad%') order by start",
                 (t,)).fetchall()
for r in rows[:140]:
    print(f"{r[0][:60]:60s} {r[1:-1]} {r[-1]/1e3:9.1f} us")
