"""criterion="absolute_error": GPU MAE builder vs the C++ host builder (8 threads) on one batch.

    python scripts/bench_mae.py [rows] [features] [trees]
"""
import sys
import time

import numpy as np
import torch

from cs230_distributed_machine_learning_amd.ops import binning, forest_ops
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles
from cs230_distributed_machine_learning_amd.utils import native


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    rng = np.random.RandomState(0)
    X = rng.randn(n, d).astype(np.float32)
    y = (X[:, 0] - 0.5 * X[:, 1] ** 2 + rng.standard_t(2, n)).astype(np.float32)
    dev = torch.device("cuda:0")
    Xb = binning.bin_matrix(torch.from_numpy(X).to(dev), binning.quantile_edges(torch.from_numpy(X).to(dev)))
    roles, _ = make_split_roles(y, 5, False, holdout=False)
    specs = forest_ops.make_specs(T)
    for t in range(T):
        s = specs[t]
        s["seed"], s["split"], s["fit"] = 1000 + t, t % 5, t % 5
        s["max_depth"], s["min_samples_split"], s["min_samples_leaf"] = 2**31 - 1, 2, 1
        s["max_features"], s["bootstrap"], s["criterion"] = d, 1, forest_ops.MAE
        s["pois_cdf"] = native.poisson_cdf_table(1.0)
    yd, rd = torch.from_numpy(y).to(dev), torch.from_numpy(roles).to(dev)
    forest_ops.build_gpu_mae(Xb, yd, rd, specs[:1])          # warm-up (module load, allocations)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = forest_ops.build_gpu_mae(Xb, yd, rd, specs)
    torch.cuda.synchronize()
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    c = forest_ops.build_cpu(Xb.cpu().numpy(), None, y, roles, specs, 1, True)
    tc = time.perf_counter() - t0
    same = (g.nodes.shape[0] == c.nodes.shape[0])
    print(f"absolute_error {n}x{d}, {T} trees (all features, bootstrap): GPU {tg:.3f} s ({g.stats['levels']} levels, "
          f"{g.nodes.shape[0]} nodes), host {tc:.3f} s ({c.nodes.shape[0]} nodes), speedup {tc / tg:.1f}x, "
          f"node counts equal: {same}")


if __name__ == "__main__":
    main()
