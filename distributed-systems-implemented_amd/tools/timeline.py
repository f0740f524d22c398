"""Print one step's GPU timeline (kernels and memory copies, in start order, with
the idle gap before each) from a rocprofv3 SQLite db.

usage: python tools/timeline.py <results.db> <anchor kernel substring> [which=-2]
The step runs from the `which`-th launch of the anchor kernel to the next one.
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
anchor = sys.argv[2]
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
ev = [(s, e, n.split("(")[0][:60]) for n, s, e in db.execute("select name, start, end from kernels")]
for view in ("memory_copies", "memory_copy"):
    try:
        ev += [(s, e, "COPY " + str(n)) for n, s, e in db.execute(f"select name, start, end from {view}")]
        break
    except sqlite3.Error:
        pass
ev.sort()
idx = [i for i, x in enumerate(ev) if anchor in x[2]]
a = idx[which]
b = idx[which + 1] if which + 1 < len(idx) and which != -1 else len(ev)
t0 = ev[a][0]
prev_end = ev[a - 1][1] if a > 0 else t0
busy = 0
for s, e, n in ev[a:b]:
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev_end) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f}  {n}")
    busy += e - s
    prev_end = max(prev_end, e)
print(f"span {(ev[b - 1][1] - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
