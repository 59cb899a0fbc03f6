"""Sweep forest-builder tier parameters on a bench-like workload (1M x 100, 4 grid candidates x 5 folds)."""
import itertools, os, sys, time
import numpy as np, torch
sys.path.insert(0, '/root/repo')
from cs230_distributed_machine_learning_amd.ops import binning, forest_ops
from cs230_distributed_machine_learning_amd.utils import native
from cs230_distributed_machine_learning_amd.search.cv import make_split_roles
from cs230_distributed_machine_learning_amd.data import synthetic
dev = torch.device('cuda:0')
# SWEEP_TASK: bin (default, the bench) | mc (4 classes) | reg (squared_error on a continuous target)
task = os.environ.get("SWEEP_TASK", "bin")
X, y = synthetic.make_table(1_000_000, 100, informative=10, n_classes=4 if task == "mc" else 2, noise=1.0, seed=0,
                            device=dev)
y = y.to(torch.int32)
yreg = None
if task == "reg":
    yreg = (X[:, :10].sum(1) + 0.5 * X[:, 0] * X[:, 1]).float().contiguous()
edges = binning.quantile_edges(X); Xb = binning.bin_matrix(X, edges)
import os
XbT = None if os.environ.get("DML_NO_XBT") else Xb[:, :X.shape[1]].t().contiguous()
roles, _ = make_split_roles(y.cpu().numpy(), 5, True, holdout=False)
roles = torch.from_numpy(roles).to(dev)
# 4 candidates spanning the grid's cost range
cands = [(200, None, 2, 1), (150, 30, 5, 2), (100, 20, 10, 4), (50, 10, 20, 8)]
T = sum(c[0] for c in cands) * 5
specs = forest_ops.make_specs(T)
i = 0
for f, (ne, md, mss, msl) in enumerate(cands):
    for fold in range(5):
        for t in range(ne):
            s = specs[i]; s['seed'] = 7 + i; s['split'] = fold; s['fit'] = f * 5 + fold
            s['max_depth'] = md if md else 2**31 - 1; s['min_samples_split'] = mss; s['min_samples_leaf'] = msl
            s['max_features'] = 10; s['bootstrap'] = 1; s['criterion'] = 2 if task == "reg" else 0; s['pois_cdf'] = native.poisson_cdf_table(1.0)
            i += 1
base = forest_ops.ForestTiers()
grid = [dict()]
for kv in sys.argv[1:]:
    k, vals = kv.split('=')
    grid = [dict(g, **{k: int(v)}) for g in grid for v in vals.split(',')]
for g in grid:
    tiers = forest_ops.ForestTiers(**{**base.__dict__, **g})
    ts = []
    for rep in range(2):
        torch.cuda.synchronize(); t0 = time.time()
        fb = forest_ops.build_gpu(Xb, None if yreg is not None else y, yreg, roles, specs,
                                  4 if task == "mc" else (1 if yreg is not None else 2), yreg is not None, tiers, XbT=XbT)
        torch.cuda.synchronize(); ts.append(time.time() - t0)
        stats = fb.stats
        del fb
    print(g, f"build {min(ts):.3f}s  ({T} trees)", {k: stats[k] for k in ("levels", "pool_retries", "tier_nodes")}, flush=True)
