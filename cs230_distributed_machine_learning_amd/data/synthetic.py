"""Deterministic synthetic tabular data generated ON the device, block by block.

Rows are produced in fixed blocks whose RNG seed is the global block id, so the
table is identical whether one rank generates all of it or N ranks each generate a
contiguous block range and all-gather (parallel/data.py).  Used by ``bench.py``
(BASELINE configs 2-4: 1M x 100 classification, 10M x 1000 binary) — there is no
network for real datasets on the MI355X pool.
"""
from __future__ import annotations

from typing import Tuple

import torch

BLOCK = 15625  # 1M = 64 blocks; divisible by 1, 2, 4, 8 ranks


def _weights(d: int, informative: int, n_classes: int, seed: int, device) -> torch.Tensor:
    g = torch.Generator(device="cpu")
    g.manual_seed(seed * 7919 + 17)
    W = torch.randn(informative, 1 if n_classes == 2 else n_classes, generator=g)
    return W.to(device)


def make_block_range(b0: int, b1: int, d: int, informative: int = 10, n_classes: int = 2, noise: float = 1.0,
                     seed: int = 0, device="cpu", block: int = BLOCK, regression: bool = False
                     ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rows of blocks [b0, b1): X float32 [(b1-b0)*block, d], y int32 (or float32)."""
    device = torch.device(device)
    W = _weights(d, min(informative, d), 2 if regression else n_classes, seed, device)
    Xs, ys = [], []
    for b in range(b0, b1):
        g = torch.Generator(device=device)
        g.manual_seed(seed * 1_000_003 + b)
        X = torch.randn(block, d, device=device, generator=g)
        z = X[:, : W.shape[0]] @ W + noise * torch.randn(block, W.shape[1], device=device, generator=g)
        if regression:
            y = z[:, 0].float()
        elif n_classes == 2:
            y = (z[:, 0] > 0).to(torch.int32)
        else:
            y = z.argmax(1).to(torch.int32)
        Xs.append(X)
        ys.append(y)
    return torch.cat(Xs), torch.cat(ys)


def make_table(n: int, d: int, informative: int = 10, n_classes: int = 2, noise: float = 1.0, seed: int = 0,
               device="cpu", rank: int = 0, world: int = 1, block: int = BLOCK, regression: bool = False):
    """This rank's contiguous row shard of the n x d table (n must be a multiple of block*world)."""
    nb = n // block
    if nb * block != n or nb % world != 0:
        raise ValueError(f"n={n} must be a multiple of block({block}) x world({world})")
    per = nb // world
    return make_block_range(rank * per, (rank + 1) * per, d, informative, n_classes, noise, seed, device, block,
                            regression)
