"""Busy/idle analysis of a rocprofv3 kernel trace: union of kernel intervals vs wall span."""
import csv, glob, sys
from collections import defaultdict
rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
if not iv:
    sys.exit("no kernel trace")
arg = sys.argv[2] if len(sys.argv) > 2 else "0"
span0, span1 = iv[0][0], max(e for _, e, _ in iv)
try:   # skip the first fraction of the span (warmup) ...
    cut = span0 + (span1 - span0) * float(arg)
except ValueError:   # ... or start at the first kernel whose name contains the argument
    cut = min(s for s, _, n in iv if arg in n)
iv = [x for x in iv if x[0] >= cut]
busy, cs, ce = 0, None, None
for s, e, _ in iv:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
wall = max(e for _, e, _ in iv) - iv[0][0]
tot = defaultdict(int)
for s, e, n in iv:
    tot[n[:50]] += e - s
print(f"window {wall/1e6:.1f} ms, GPU busy (union of kernels) {busy/1e6:.1f} ms = {100*busy/wall:.1f}%, "
      f"sum of kernel time {sum(tot.values())/1e6:.1f} ms (overlap x{sum(tot.values())/max(1,busy):.2f})")
for n, v in sorted(tot.items(), key=lambda x: -x[1])[:12]:
    print(f"  {n:50s} {v/1e6:9.1f} ms")
