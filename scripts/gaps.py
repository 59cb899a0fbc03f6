"""Idle gaps of a rocprofv3 kernel trace: every interval in which no kernel runs, attributed
to the (kernel before, kernel after) pair -- where a host sync or host-side work stalls the GPU.
usage: python scripts/gaps.py <trace dir> [min_gap_us=20] [skip_fraction=0.3]"""
import csv, glob, sys
from collections import defaultdict

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]) for r in rows)
min_gap = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 20e3
skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.3
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
iv = [x for x in iv if x[0] >= t0 + (t1 - t0) * skip]
gaps = defaultdict(lambda: [0, 0.0])
ce, cname = iv[0][1], iv[0][2]
total_idle, small = 0.0, 0.0
for s, e, n in iv[1:]:
    if s > ce:
        g = s - ce
        total_idle += g
        if g >= min_gap:
            k = (cname, n)
            gaps[k][0] += 1
            gaps[k][1] += g
        else:
            small += g
    if e > ce:
        ce, cname = e, n
wall = ce - iv[0][0]
print(f"window {wall/1e6:.1f} ms, idle {total_idle/1e6:.1f} ms ({100*total_idle/wall:.1f}%), of which gaps < {min_gap/1e3:.0f} us: {small/1e6:.1f} ms")
for (a, b), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"  {t/1e6:8.2f} ms  n={c:5d}  avg {t/c/1e3:8.1f} us   {a} -> {b}")
