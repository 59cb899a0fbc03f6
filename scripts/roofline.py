"""Merge several rocprofv3 ``--pmc`` passes (CSV) into one per-kernel memory-hierarchy table.

Usage: ``python scripts/roofline.py gpurun_out/pmc2_a gpurun_out/pmc2_b ...``

Per kernel (summed over dispatches): wall estimate from GRBM_GUI_ACTIVE (summed over the
8 XCDs, so cycles = GRBM / 8, at the clock given by --ghz), L2 requests and hit rate
(TCC_HIT/TCC_MISS), L1 (TCP) accesses, fabric-side bytes (FETCH_SIZE is reported in KB by
rocprofv3; MI355X_MICROARCH.md: it counts 64-B units of 128-B requests for wide reads, so it
is a lower bound for byte gathers), LDS bank-conflict cycles per LDS-array cycle.
"""
import argparse
import csv
import glob
from collections import defaultdict


def load(dirs):
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                agg[k][r["Counter_Name"] + "@" + d] += float(r["Counter_Value"])
                disp[k].add((d, r.get("Dispatch_Id", "")))
    return agg, disp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--ghz", type=float, default=2.1)
    ap.add_argument("--min-ms", type=float, default=1.0)
    args = ap.parse_args()
    agg, _ = load(args.dirs)
    rows = []
    for k, c in agg.items():
        def get(name):
            vals = [v for n, v in c.items() if n.split("@")[0] == name]
            return sum(vals) / len(vals) if vals else None   # same program in every pass: average
        grbm = get("GRBM_GUI_ACTIVE")
        ms = grbm / 8 / (args.ghz * 1e6) if grbm else 0.0
        if ms < args.min_ms:
            continue
        hit, miss = get("TCC_HIT_sum"), get("TCC_MISS_sum")
        fetch_kb = get("FETCH_SIZE")
        tcp = get("TCP_TOTAL_CACHE_ACCESSES_sum")
        tcp_tcc = get("TCP_TCC_READ_REQ_sum")
        lds_conf, lds_act = get("SQ_LDS_BANK_CONFLICT"), get("SQ_LDS_IDX_ACTIVE")
        vmem = get("SQ_INSTS_VMEM_RD")
        wait, wcyc = get("SQ_WAIT_ANY"), get("SQ_WAVE_CYCLES")
        ta = get("TA_TA_BUSY_sum")
        s = ms / 1e3
        line = f"{k[:48]:48s} ~{ms:8.1f} ms"
        if hit is not None and miss is not None:
            line += f" | L2 req {(hit + miss) / s / 1e9:6.1f} G/s hit {hit / max(hit + miss, 1):4.2f}"
        if tcp_tcc is not None:
            line += f" | L1->L2 rd {tcp_tcc / s / 1e9:6.1f} G/s"
        if tcp is not None:
            line += f" | L1 acc {tcp / s / 1e9:6.1f} G/s"
        if fetch_kb is not None:
            line += f" | fabric {fetch_kb * 1024 / s / 1e12:5.2f} TB/s (x2 for wide reads)"
        if vmem is not None:
            line += f" | vmem rd {vmem / s / 1e9:5.2f} Ginst/s"
        if ta is not None and grbm:
            line += f" | TA busy {ta / (grbm / 8 * 32):4.2f}"   # 32 TA per XCD (one per CU)
        if lds_conf is not None and lds_act:
            line += f" | LDS conflict/active {lds_conf / lds_act:4.2f}"
        if wait is not None and wcyc:
            line += f" | wait {wait / wcyc:4.2f}"
        rows.append((ms, line))
    for _, line in sorted(rows, reverse=True):
        print(line)


if __name__ == "__main__":
    main()
