"""Per kernel family: summed duration and the part of it during which NO other
kernel ran (exclusive time) in a rocprofv3 rocpd .db kernel trace — the
families with large exclusive time sit on the critical path; the wall span
minus the union of all kernels is idle time.
usage: exclusive_time.py DB [--top N] [--window START_NAME]"""
import re
import sqlite3
import sys
from collections import defaultdict


def family(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("void ", "")[:90]


def main():
    c = sqlite3.connect(sys.argv[1])
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = sorted(c.execute(f"select start, end, {name_col} from kernels"))
    ev = []
    for i, (s, e, n) in enumerate(rows):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    excl = defaultdict(float)
    tot = defaultdict(float)
    busy = 0.0
    last = ev[0][0]
    for t, kind, i in ev:
        if active:
            busy += t - last
            if len(active) == 1:
                (j,) = tuple(active)
                excl[family(rows[j][2])] += t - last
        last = t
        if kind == 1:
            active.add(i)
        else:
            active.discard(i)
    for s, e, n in rows:
        tot[family(n)] += e - s
    span = rows[-1][1] - rows[0][0]
    print(f"span {span/1e6:.1f} ms, busy (union) {busy/1e6:.1f} ms, summed kernel time {sum(tot.values())/1e6:.1f} ms")
    print(f"{'family':90s} {'total_ms':>9s} {'excl_ms':>9s}")
    for f in sorted(tot, key=lambda f: -excl[f])[:top]:
        print(f"{f:90s} {tot[f]/1e6:9.2f} {excl[f]/1e6:9.2f}")


if __name__ == "__main__":
    main()


def windows(db, marker):
    """Busy union and span of each window between consecutive starts of the
    kernel named by marker (one round each in a bench trace)."""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
    rows = sorted(c.execute(f"select start, end, {name_col} from kernels"))
    marks = [s for s, e, n in rows if marker in n]
    for a, b in zip(marks, marks[1:]):
        iv = sorted((max(s, a), min(e, b)) for s, e, n in rows if e > a and s < b)
        busy, cur = 0, None
        for s, e in iv:
            if cur is None or s > cur[1]:
                if cur:
                    busy += cur[1] - cur[0]
                cur = [s, e]
            else:
                cur[1] = max(cur[1], e)
        if cur:
            busy += cur[1] - cur[0]
        print(f"window {(b - a)/1e6:8.2f} ms  busy {busy/1e6:8.2f} ms  idle {(b - a - busy)/1e6:7.2f} ms")
