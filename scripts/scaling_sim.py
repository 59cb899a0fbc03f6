"""Predict bench.py's multi-GPU weak-scaling efficiency on ONE GPU.

For a world size N, every rank's per-step candidate list is reconstructed exactly as
bench.py builds it (``--placement lpt``: the native LPT scheduler over the step pool;
``--placement group``: the earlier fixed one-candidate-per-cost-group rule) and each
rank's list is timed back to back on this GPU.  The step time of an N-GPU run is the
max over ranks, so efficiency ~= mean(rank time) / max(rank time) per step (ignoring
the one small score all-reduce).  Prints one JSON line per (N, placement).

    python scripts/scaling_sim.py --world 2,4,8 --steps 2 --placement lpt,group
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from bench import GRID
from cs230_distributed_machine_learning_amd.data import synthetic
from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, prepare_splits, run_candidates
from cs230_distributed_machine_learning_amd.engine.scheduler import lpt_assign
from cs230_distributed_machine_learning_amd.engine.service import candidate_costs
from cs230_distributed_machine_learning_amd.ops import binning
from cs230_distributed_machine_learning_amd.search.grid import expand_candidates


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", default="2,4,8")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--placement", default="lpt,group")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--cv", type=int, default=5)
    ap.add_argument("--cands-per-rank", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    X, y = synthetic.make_table(a.rows, a.features, informative=10, n_classes=2, noise=1.0, seed=0, device=dev)
    dd = DeviceData(X, y, classification=True, device=dev, name="sim")
    dd._edges = binning.quantile_edges(X)
    dd._Xb = binning.bin_matrix(X, dd._edges)
    cands = expand_candidates("GridSearchCV", {"param_grid": GRID})
    spec = JobSpec("RandomForestClassifier", cands, cv=a.cv, holdout=False, random_state=0, keep_models="none", seed=0)
    prepare_splits(dd, spec)
    plan = {"model_type": "RandomForestClassifier", "candidates": cands, "cv": a.cv, "holdout": False}
    costs = np.array(candidate_costs(plan, int(a.rows * (a.cv - 1) / a.cv), a.features, 2))
    groups = np.array_split(np.argsort(-costs, kind="stable"), a.cands_per_rank)
    golden = [np.argsort(np.argsort(np.mod(np.arange(len(g)) * 0.6180339887498949, 1.0), kind="stable"),
                         kind="stable") for g in groups]   # same pick order as bench.py

    def lists(N, step, how):
        if how == "group":
            return [[int(g[(step * N + r) % len(g)]) for g in groups] for r in range(N)]
        pool = [int(g[gp[(step * N + j) % len(g)]]) for g, gp in zip(groups, golden) for j in range(N)]
        owner = lpt_assign([float(costs[i]) for i in pool], N)
        return [[c for c, o in zip(pool, owner) if int(o) == r] for r in range(N)]

    def timed(cids):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = run_candidates(dd, spec, cids)
        torch.cuda.synchronize()
        assert all(x.ok for x in res)
        return time.perf_counter() - t0

    for _ in range(a.warmup):
        timed(lists(1, 0, "group")[0])
    for N in [int(v) for v in a.world.split(",")]:
        for how in a.placement.split(","):
            per_step = []
            for s in range(a.warmup, a.warmup + a.steps):
                t = [timed(cl) for cl in lists(N, s, how)]
                per_step.append(t)
            eff = float(np.mean([np.mean(t) / max(t) for t in per_step]))
            fits = N * a.cands_per_rank * a.cv * a.steps
            print(json.dumps({"world": N, "placement": how, "rank_seconds": [[round(v, 3) for v in t] for t in per_step],
                              "predicted_efficiency": round(eff, 4),
                              "predicted_fits_per_s": round(fits / sum(max(t) for t in per_step), 3)}), flush=True)


if __name__ == "__main__":
    main()
