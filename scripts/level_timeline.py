"""Per-dispatch timeline of the last forest batch in a rocprofv3 (rocpd) database:
start offset, duration, grid (workgroups), VGPRs, LDS per dispatch; plus busy union."""
import sqlite3
import sys

db = sys.argv[1]
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 400
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end, grid_x, grid_y, workgroup_x, vgpr_count, accum_vgpr_count, lds_size, "
                      "stream_id from kernels order by start"))
fills = [i for i, r in enumerate(rows) if "k_fill_active" in r[0]]
seq = rows[fills[-1]:]
t0 = seq[0][1]
iv = sorted((r[1], r[2]) for r in seq)
busy, cs, ce = 0, None, None
for s, e in iv:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
wall = max(r[2] for r in seq) - t0
print(f"last batch: wall {wall / 1e6:.1f} ms, GPU busy (union) {busy / 1e6:.1f} ms, dispatches {len(seq)}")
for r in seq[:lim]:
    n = r[0].split("(")[0].replace("void dml::", "").replace("dml::", "")
    wg = (r[3] // max(1, r[5])) * r[4]
    print(f"{(r[1] - t0) / 1e6:9.2f} {(r[2] - r[1]) / 1e6:8.2f}  {n[:24]:24s} wg={wg:8d} vgpr={r[6]}+{r[7]} lds={r[8]} s={r[9]}")
