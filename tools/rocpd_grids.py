"""Per-dispatch grid sizes and durations of the kernels whose name contains a
substring, from a rocprofv3 rocpd .db (which launch of a template is slow).
usage: rocpd_grids.py DB SUBSTRING [N]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "kernel_name" if "kernel_name" in cols else "name"
grid = [x for x in ("grid_size_x", "grid_x", "grid_size") if x in cols]
gy = [x for x in ("grid_size_y", "grid_y") if x in cols]
gz = [x for x in ("grid_size_z", "grid_z") if x in cols]
wg = [x for x in ("workgroup_size_x", "workgroup_x", "block_size_x") if x in cols]
sel = ", ".join([name_col] + grid[:1] + gy[:1] + gz[:1] + wg[:1] + ["end-start"])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
print("columns:", cols)
seen = {}
for row in c.execute(f"select {sel} from kernels where {name_col} like ? order by start", (f"%{sys.argv[2]}%",)):
    key = tuple(row[1:-1])
    d = seen.setdefault(key, [0, 0.0])
    d[0] += 1
    d[1] += row[-1]
for key, (cnt, tot) in sorted(seen.items(), key=lambda kv: -kv[1][1])[:n]:
    print(key, cnt, f"{tot / cnt / 1e3:.1f} us avg")
