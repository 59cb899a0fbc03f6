"""Row-sharded forest: bytes exchanged per build vs forest_dp.SPARSE_ROWS (2 gloo ranks on CPU).

    PYTHONPATH=. python scripts/dp_exchange_sweep.py
"""
import os, sys, json
import numpy as np, torch, torch.multiprocessing as mp

def rank(r, world, port, sparse_rows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), OMP_NUM_THREADS="2")
    from cs230_distributed_machine_learning_amd.parallel import dist
    from cs230_distributed_machine_learning_amd.parallel.data_parallel import RowShard, shard_bounds
    from cs230_distributed_machine_learning_amd.ops import forest_dp, forest_ops
    from cs230_distributed_machine_learning_amd.models.forest import native_seed
    from cs230_distributed_machine_learning_amd.utils import native
    forest_dp.SPARSE_ROWS = sparse_rows
    inf = dist.init(want_gpu=False, timeout_s=120)
    rng = np.random.default_rng(0)
    n, d = 60000, 20
    X = rng.normal(size=(n, d)).astype(np.float32)
    y = (X[:, 0] + X[:, 1] + 0.8 * rng.normal(size=n) > 0).astype(np.int64)
    a, b = shard_bounds(n, world, r)
    sh = RowShard(X[a:b], y, a, True, inf.device)
    sh.set_splits(np.ones((1, n), np.uint8), ["full"])
    Xb = sh.binned()
    T = 8
    specs = forest_ops.make_specs(T)
    specs["seed"] = [native_seed(1, j) for j in range(T)]
    specs["max_depth"] = 2**31 - 1; specs["min_samples_split"] = 2; specs["min_samples_leaf"] = 1
    specs["max_features"] = 4; specs["bootstrap"] = 1; specs["criterion"] = 0
    specs["pois_cdf"] = native.poisson_cdf_table(1.0)
    fb = forest_dp.build_dp(Xb, sh.y_cls, None, sh.roles, specs, 2, False, sh.r0, reduce=sh.all_reduce, comm=sh)
    if r == 0:
        q.put({"sparse_rows": sparse_rows, "bytes_GB": fb.stats["allreduce_bytes"] / 1e9, "nodes": fb.stats["nodes"], "levels": fb.stats["levels"], "rounds": fb.stats["rounds"], "s": round(fb.stats["build_s"], 2)})
    dist.destroy()

if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    for i, sr in enumerate((0, 16, 48, 96)):
        q = ctx.Queue()
        ps = [ctx.Process(target=rank, args=(r, 2, 29650 + i, sr, q)) for r in range(2)]
        [p.start() for p in ps]
        print(json.dumps(q.get(timeout=600)), flush=True)
        [p.join() for p in ps]
