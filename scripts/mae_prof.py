import csv, sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if "k_mae_level" in r["Kernel_Name"]]
d=[(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e6 for r in rows]
keys=[k for k in rows[0] if "Grid" in k] if rows else []
print("grid keys", keys)
g=[int(r[keys[0]])//256 if keys else 0 for r in rows]
print(len(d), "level launches; first 14 (ms, wgs):", [(round(a,2), b) for a,b in zip(d[:14], g[:14])])
print("sum first 10 levels", round(sum(d[:10]),1), "rest", round(sum(d[10:]),1))
