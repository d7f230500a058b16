import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
t = c.execute("select max(start) from kernels where kernel_name like '%orderstat%'").fetchone()[0]
rows = c.execute("select kernel_name, grid_size_x, grid_size_y, grid_size_z, end-start from kernels "
                 "where start > ? and kernel_name like '%cgemm%' order by start", (t,)).fetchall()
for r in rows[:70]:
    print(f"{r[0][:45]:45s} grid=({r[1]},{r[2]},{r[3]}) {r[4]/1e3:9.1f} us")
