"""Per-level span of the last forest build in a rocprofv3 (rocpd) database: each level's
wall span and its tier kernels (duration / workgroups), plus kernel resource usage.
    python scripts/level_spans.py <run_results.db>"""
import sqlite3, sys
c=sqlite3.connect(sys.argv[1])
rows=list(c.execute("select name, start, end, grid_x*grid_y, workgroup_x, vgpr_count, accum_vgpr_count, lds_size, scratch_size from kernels order by start"))
fills=[i for i,r in enumerate(rows) if 'k_fill_active' in r[0]]
seq=rows[fills[-1]:]
t0=seq[0][1]
lev=[]; cur=[]
for r in seq:
    cur.append(r)
    if 'k_compact' in r[0]:
        lev.append(cur); cur=[]
lev.append(cur)
print("levels", len(lev), "build wall ms", (seq[-1][2]-t0)/1e6)
seen=set()
for r in seq:
    n=r[0].split('(')[0]
    if n not in seen:
        seen.add(n); print(f"  {n[:50]:50s} vgpr={r[5]}+{r[6]} lds={r[7]} scratch={r[8]}")
for i,L in enumerate(lev):
    s=min(r[1] for r in L); e=max(r[2] for r in L)
    parts=[]
    for r in L:
        n=r[0].split('(')[0].replace('void ','').replace('dml::','')
        if any(k in n for k in ('k_nodes','k_subtree','k_bigsub','k_hist_large','k_split_large','k_partition_large','k_predict')):
            parts.append(f"{n[:14]}:{(r[2]-r[1])/1e3:.0f}us/{r[3]//max(1,r[4])}")
    print(f"L{i:2d} start {(s-t0)/1e6:7.1f} span {(e-s)/1e3:8.0f}us  "+" ".join(parts))
