"""Exposed time per kernel group in a rocprofv3 (rocpd) kernel trace: the wall time during which
kernels of a group run while NO kernel of any other group does -- e.g. how much of the forest
predict is not hidden behind tree building.
    python scripts/exposed_time.py <run_results.db> [group=substr,substr ...]
Default groups: predict (k_predict, k_scores, k_apply, k_refine), build (everything else)."""
import sqlite3
import sys

db = sys.argv[1]
groups = {"predict": ("k_predict", "k_scores", "k_apply", "k_refine")}
for arg in sys.argv[2:]:
    name, subs = arg.split("=")
    groups[name] = tuple(subs.split(","))
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end from kernels order by start"))
if not rows:
    sys.exit("no kernels")


def group_of(name):
    for g, subs in groups.items():
        if any(s in name for s in subs):
            return g
    return "build"


events = []
for name, s, e in rows:
    g = group_of(name)
    events.append((s, 1, g))
    events.append((e, -1, g))
events.sort()
active = {}
exposed = {g: 0 for g in list(groups) + ["build"]}
busy = 0
last = events[0][0]
for t, d, g in events:
    live = [k for k, v in active.items() if v > 0]
    if live:
        busy += t - last
        if len(live) == 1:
            exposed[live[0]] += t - last
    active[g] = active.get(g, 0) + d
    last = t
wall = rows[-1][2] - rows[0][1]
total = {g: 0 for g in exposed}
for name, s, e in rows:
    total[group_of(name)] += e - s
print(f"wall {wall / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms ({100 * busy / wall:.1f} %)")
for g in exposed:
    print(f"  {g:10s} kernel time {total[g] / 1e6:9.1f} ms   exposed alone {exposed[g] / 1e6:8.1f} ms "
          f"({100 * exposed[g] / wall:.1f} % of wall)")
