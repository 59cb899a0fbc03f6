"""GPU busy over a WHOLE command from a rocprofv3 kernel trace (the driver samples rocm-smi
every few seconds over the entire `python bench.py ...` process, setup included).
usage: python scripts/whole_run_busy.py <trace dir> <command wall seconds> [bin_s=5]
Prints the kernel-union busy fraction over the process wall time, over [first, last kernel],
and per bin of bin_s seconds (the rocm-smi-like view)."""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
wall_s = float(sys.argv[2])
bin_ns = float(sys.argv[3]) * 1e9 if len(sys.argv) > 3 else 5e9
merged = []
for s, e in iv:
    if merged and s <= merged[-1][1]:
        merged[-1][1] = max(merged[-1][1], e)
    else:
        merged.append([s, e])
busy = sum(e - s for s, e in merged)
t0, t1 = merged[0][0], merged[-1][1]
print(f"kernels {len(iv)}, first->last kernel {(t1 - t0) / 1e9:.2f} s, busy {busy / 1e9:.2f} s "
      f"({100 * busy / (t1 - t0):.1f}% of that span; {100 * busy / (wall_s * 1e9):.1f}% of the {wall_s:.1f} s command)")
print(f"process time before the first kernel (python/torch import, HIP init, library load): "
      f"<= {wall_s - (t1 - t0) / 1e9:.1f} s (includes exit)")
b = t0
while b < t1:
    e = b + bin_ns
    u = sum(max(0, min(e, y) - max(b, x)) for x, y in merged if y > b and x < e)
    print(f"  [{(b - t0) / 1e9:6.1f} s, {(e - t0) / 1e9:6.1f} s)  busy {100 * u / bin_ns:5.1f}%")
    b = e
