"""Root-table distribution: one pageable ``.to(device)`` + broadcast vs the chunked,
copy/broadcast-overlapped path (parallel/data.py ``_pipelined_broadcast``), on an RCCL group.

    python scripts/bcast_bench.py [GB]

Run at world 1 on the one-GPU box, where the broadcast itself is a no-op: what is timed is
the host -> HBM path of the root, which the pipeline overlaps with the broadcast of the
previous chunk at N > 1."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])

from cs230_distributed_machine_learning_amd.parallel import data as pdata  # noqa: E402
from cs230_distributed_machine_learning_amd.parallel import dist  # noqa: E402


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ["DML_FORCE_PG"] = "1"
    inf = dist.init(backend="nccl", want_gpu=True, timeout_s=300)
    d = 1000
    n = int(gb * 1e9 / (4 * d))
    X = np.empty((n, d), dtype=np.float32)
    X[:] = 1.25                                    # touch every page before timing
    dev = inf.device
    out = {"gb": round(n * d * 4 / 1e9, 2), "world": inf.world, "backend": inf.backend}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Xd = torch.from_numpy(X).to(dev)
        dist.broadcast(Xd, 0)
        torch.cuda.synchronize()
        out["to_device_then_broadcast_s"] = round(time.perf_counter() - t0, 3)
        del Xd
        Xd = torch.empty((n, d), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pdata._pipelined_broadcast(X, Xd)
        torch.cuda.synchronize()
        out["pipelined_s"] = round(time.perf_counter() - t0, 3)
        out["pipelined_ok"] = bool(Xd[-1, -1].item() == 1.25 and Xd[0, 0].item() == 1.25)
        del Xd
    out["pipelined_GBps"] = round(out["gb"] / out["pipelined_s"], 1)
    out["to_device_GBps"] = round(out["gb"] / out["to_device_then_broadcast_s"], 1)
    print(json.dumps(out), flush=True)
    dist.destroy()


if __name__ == "__main__":
    main()
