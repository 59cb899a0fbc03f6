#!/usr/bin/env python3
"""KNN neighbour search on one GPU: matrix-core squared-L2 path vs the scalar streaming
kernel (DML_KNN_MFMA=0), same results.  One JSON line per (rows, features, path)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.models import neighbors as nb
    from cs230_distributed_machine_learning_amd.search.cv import make_split_roles

    for n, d in ((100_000, 20), (100_000, 100), (200_000, 64)):
        rng = np.random.RandomState(0)
        X = rng.randn(n, d).astype(np.float32)
        y = rng.randint(0, 3, n)
        roles, names = make_split_roles(y, 5, True, holdout=False)
        res = {}
        for mode in ("0", "1"):
            os.environ["DML_KNN_MFMA"] = mode
            dd = DeviceData(X, y, True, "cuda:0")
            dd.set_splits(roles, names)
            nb.knn_search_hip(dd, list(range(5)), 15, nb.M_L2, 2.0)   # warm (operands, code objects)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = nb.knn_search_hip(dd, list(range(5)), 15, nb.M_L2, 2.0)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[mode] = out
            pairs = 5 * (n // 5) * (n - n // 5)
            print(json.dumps({"rows": n, "features": d, "K": 15, "splits": 5, "path": "mfma" if mode == "1" else "scalar",
                              "seconds": round(dt, 4), "distance_pairs_per_s": round(pairs / dt / 1e9, 2),
                              "unit": "G pairs/s"}), flush=True)
        same = all(torch.equal(res["0"][s][1], res["1"][s][1]) and torch.equal(res["0"][s][0], res["1"][s][0])
                   for s in range(5))
        print(json.dumps({"rows": n, "features": d, "identical_neighbours_and_distances": same}), flush=True)


if __name__ == "__main__":
    main()
