#!/usr/bin/env python3
"""Time one batched logistic objective evaluation (forward + gradient over every fit of a
batch): fp32 library GEMMs + link kernel vs the matrix-core path (csrc/kernels/lr_mfma.hip).

    python scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512
"""
from __future__ import annotations

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
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--features", type=int, default=1000)
    ap.add_argument("--fits", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    from cs230_distributed_machine_learning_amd.data import synthetic
    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.models import linear
    from cs230_distributed_machine_learning_amd.models.base import FitTask
    from cs230_distributed_machine_learning_amd.search.cv import make_split_roles

    dev = torch.device("cuda:0")
    X, y = synthetic.make_table(args.rows, args.features, informative=10, n_classes=2, noise=1.0, seed=1, device=dev,
                                block=args.rows // 8)
    dd = DeviceData(X, y, True, dev)
    roles, names = make_split_roles(y.cpu().numpy(), 5, True, holdout=False, test_size=0.2, random_state=0)
    dd.set_splits(roles, names)
    fam = linear.LogisticFamily()
    rng = np.random.RandomState(0)
    tasks = [FitTask(task_id=i, candidate=i, split=i % 5, model_type="LogisticRegression",
                     params=fam.resolve("LogisticRegression", {"C": float(10 ** rng.uniform(-3, 2))}, dd.n, dd.d, 2))
             for i in range(args.fits)]
    b = linear._Batch(dd, tasks)
    W = torch.randn((dd.d + 1, b.M), device=dev) * 0.01
    out = {"rows": args.rows, "features": args.features, "fits": args.fits}
    for name in ("fp32", "mfma"):
        if name == "mfma":
            t0 = time.perf_counter()
            b.mf = linear.MfmaPlan(dd, b)
            torch.cuda.synchronize()
            out["mfma_setup_s"] = round(time.perf_counter() - t0, 3)
        fam._objective(dd, b, W)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            f, G = fam._objective(dd, b, W)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        flops = 2 * 2 * args.rows * args.features * b.M
        out[f"{name}_ms"] = round(dt * 1e3, 2)
        out[f"{name}_tflops_fp32_equiv"] = round(flops / dt / 1e12, 1)
        out[f"{name}_loss0"] = float(f[0])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
