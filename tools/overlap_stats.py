"""Concurrency of one kernel family with everything else in a rocprofv3 rocpd
.db (kernel trace): for the kernels whose name contains PATTERN, their summed
duration, the part of it during which some other kernel ran at the same time,
and the trace's wall span vs its summed kernel time.
usage: overlap_stats.py DB PATTERN [--after-last SUBSTRING]"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = sys.argv[2]
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    where = ""
    if "--after-last" in sys.argv:
        marker = sys.argv[sys.argv.index("--after-last") + 1]
        t = c.execute(f"select max(start) from kernels where {name_col} like ?", (f"%{marker}%",)).fetchone()[0]
        where = f"where start > {t}"
    rows = sorted(c.execute(f"select start, end, {name_col} from kernels {where}"))
    if not rows:
        print("no kernels")
        return
    mine = [(s, e) for s, e, n in rows if pat in n]
    other = [(s, e) for s, e, n in rows if pat not in n]
    # union of the other kernels' intervals
    merged = []
    for s, e in other:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot = sum(e - s for s, e in mine)
    ov = 0
    j = 0
    for s, e in mine:
        while j < len(merged) and merged[j][1] <= s:
            j += 1
        k = j
        while k < len(merged) and merged[k][0] < e:
            ov += max(0, min(e, merged[k][1]) - max(s, merged[k][0]))
            k += 1
    wall = rows[-1][1] - rows[0][0]
    busy = sum(e - s for s, e, _ in rows)
    print(f"{pat}: {len(mine)} dispatches, {tot / 1e6:.3f} ms, concurrent with other kernels {ov / 1e6:.3f} ms "
          f"({100 * ov / max(tot, 1):.1f} %)")
    print(f"trace wall {wall / 1e6:.3f} ms, summed kernel time {busy / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
