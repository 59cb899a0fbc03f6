"""Row-sharded forest builder vs the one-GPU builder on one device (world 1).

    python scripts/dp_forest_bench.py [rows] [features] [trees] [max_depth|0]

Prints one JSON line per builder: build seconds, levels, search rounds, histogram bytes
that an N-rank run would all-reduce, and whether the trees are identical.  At world 1
the all-reduce is a no-op, so the DP number is the builder's own compute cost; an N-rank
run adds (allreduce_bytes x 2(N-1)/N) / link bandwidth per build.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from cs230_distributed_machine_learning_amd.models.forest import native_seed  # noqa: E402
from cs230_distributed_machine_learning_amd.ops import binning, forest_dp, forest_ops  # noqa: E402
from cs230_distributed_machine_learning_amd.utils import native  # noqa: E402


def main():
    os.environ.setdefault("DML_DP_TIMING", "1")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    md = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn((n, d), device=dev, generator=g)
    w = torch.randn((d,), device=dev, generator=g)
    w[10:] = 0
    y = ((X @ w + 0.5 * torch.randn((n,), device=dev, generator=g)) > 0).to(torch.int32)
    Xb = binning.bin_matrix(X, binning.quantile_edges(X))
    del X
    roles = torch.ones((1, n), dtype=torch.uint8, device=dev)
    specs = forest_ops.make_specs(T)
    specs["seed"] = [native_seed(1, j) for j in range(T)]
    specs["max_depth"] = md if md > 0 else forest_ops.INT32_MAX
    specs["min_samples_split"], specs["min_samples_leaf"] = 2, 1
    specs["max_features"] = max(1, int(np.sqrt(d)))
    specs["bootstrap"], specs["criterion"] = 1, 0
    specs["pois_cdf"] = native.poisson_cdf_table(1.0)
    XbT = Xb.t().contiguous()
    out = {}
    for rep in range(2):   # first pass warms kernels / allocator
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ref = forest_ops.build_gpu(Xb, y, None, roles, specs, 2, False, XbT=XbT)
        torch.cuda.synchronize()
        t_ref = time.perf_counter() - t0
        t0 = time.perf_counter()
        dp = forest_dp.build_dp(Xb, y, None, roles, specs, 2, False, 0)
        torch.cuda.synchronize()
        t_dp = time.perf_counter() - t0
        out = {"rows": n, "features": d, "trees": T, "max_depth": md or None,
               "one_gpu_build_s": round(t_ref, 4), "dp_build_s": round(t_dp, 4),
               "dp_levels": dp.stats["levels"], "dp_rounds": dp.stats["rounds"],
               "dp_hist_s": round(dp.stats["hist_s"], 4),
               "dp_allreduce_gb": round(dp.stats["allreduce_bytes"] / 1e9, 3),
               "nodes_one_gpu": int(ref.stats["nodes"]), "nodes_dp": int(dp.stats["nodes"])}
    # identical forests: the same prediction for every row
    rows = torch.arange(n, dtype=torch.int32, device=dev)
    toff, roff = np.array([0, T]), np.array([0, n])
    same = bool(torch.equal(forest_ops.predict(ref, Xb, toff, roff, rows), forest_ops.predict(dp, Xb, toff, roff, rows)))
    out["same_predictions"] = same
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
