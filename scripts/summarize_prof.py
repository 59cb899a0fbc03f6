"""Summarise rocprofv3 kernel-trace / PMC CSVs into a short text table (profiles/*.txt)."""
import csv
import glob
import sys
from collections import defaultdict


def kernel_stats(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows:
        return kernel_stats_db(d)
    tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1
    out = []
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        out.append(f"  {r['Name'][:60]:60s} calls={int(r['Calls']):6d} total_ms={float(r['TotalDurationNs'])/1e6:9.2f} "
                   f"{100*float(r['TotalDurationNs'])/tot:5.1f}%")
    return out


def kernel_stats_db(d):
    """rocprofv3 >= ROCm 7 writes a rocpd SQLite database by default (``*_results.db``)."""
    import sqlite3

    out = []
    for f in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(f)
        for name, calls, tot_ns, avg_ns, pct in c.execute(
                "select name, total_calls, total_duration, average, percentage from top_kernels"):
            if pct < 0.01:
                continue
            out.append(f"  {name[:60]:60s} calls={int(calls):6d} total_ms={tot_ns/1e3:9.2f} avg_us={avg_ns:9.1f} "
                       f"{pct:5.1f}%")
    return out


def pmc(d):
    agg = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    out = []
    for k, c in agg.items():
        out.append(f"  {k}")
        out.append("     " + "  ".join(f"{n}={v:.3g}" for n, v in sorted(c.items())))
        if "SQ_WAVES" in c and c["SQ_WAVES"]:
            w = c["SQ_WAVES"]
            extra = []
            if "SQ_INSTS_VALU" in c:
                extra.append(f"VALU/wave={c['SQ_INSTS_VALU']/w:.0f}")
            if "SQ_INSTS_LDS" in c:
                extra.append(f"LDS/wave={c['SQ_INSTS_LDS']/w:.0f}")
            if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
                extra.append(f"wait_frac={c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES']:.2f}")
            out.append("     " + "  ".join(extra))
    return out


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(f"== {d}")
        lines = kernel_stats(d)
        print("\n".join(lines) if lines else "\n".join(pmc(d)))
