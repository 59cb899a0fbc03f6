#!/usr/bin/env python3
"""SVC 50k x 20, 8 candidates x cv5 on one GPU (verdict item 9): wall time of the whole
search through the engine (run_candidates), SMO iterations per problem, kernel-column
cache statistics.  ``python scripts/svm_bench.py [--rows 50000] [--cache-mb N]``."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000)
    ap.add_argument("--features", type=int, default=20)
    ap.add_argument("--cv", type=int, default=5)
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    from sklearn.datasets import make_classification

    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
    from cs230_distributed_machine_learning_amd.models.base import family_of
    from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid

    X, y = make_classification(args.rows, args.features, n_informative=10, flip_y=0.05, random_state=0)
    dev = "cpu" if args.cpu else "cuda:0"
    dd = DeviceData(X.astype(np.float32), y, True, dev)
    grid = list(ParameterGrid({"C": [0.1, 1.0, 10.0, 100.0], "gamma": ["scale", "auto"]}))
    spec = JobSpec("SVC", grid, cv=args.cv, holdout=False, keep_models="none")
    t0 = time.perf_counter()
    res = run_candidates(dd, spec, range(len(grid)))
    if dev != "cpu":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fam = family_of("SVC")
    print(json.dumps({"rows": args.rows, "features": args.features, "candidates": len(grid), "cv": args.cv,
                      "fits": len(grid) * args.cv, "seconds": round(dt, 2),
                      "ok": sum(r.ok for r in res), "mean_cv": [round(r.result["mean_cv_score"], 4) for r in res],
                      "solver": getattr(fam, "last_solve_stats", None)}), flush=True)


if __name__ == "__main__":
    main()
