"""Search-space expansion: grid, random sampling and serializable distributions.

Reference behaviour being reproduced (not copied):

* ``aws-prod/master/task_handler.py:186-207`` expands a ``GridSearchCV`` into one
  subtask per point of ``ParameterGrid(param_grid)``; candidate order is sklearn's
  (keys sorted, last key varying fastest).
* ``aws-prod/master/task_handler.py:210-236`` expands ``RandomizedSearchCV`` with
  ``ParameterSampler(param_distributions, n_iter, random_state=42)``.  The seed is
  hard-coded there (defect D7); here the user's ``random_state`` is honoured and 42
  is only the default.
* scipy distributions arrive as ``str(obj)`` on the wire (``distributed_ml/core.py:70``,
  defect D8) and crash the sampler.  This module defines a JSON distribution spec
  (``{"dist": "loguniform", "a": 1e-3, "b": 1e2}``) that is decoded server-side into a
  scipy frozen distribution so sampling is bit-identical to sklearn's sampler.

Nothing here imports scikit-learn: workers and the controller do not depend on it.
Tests check index-for-index equality against sklearn on the CPU box.
"""
from __future__ import annotations

import math
import warnings
from collections.abc import Mapping, Sequence
from itertools import product
from typing import Any, Dict, Iterator, List

import numpy as np

__all__ = [
    "ParameterGrid",
    "ParameterSampler",
    "sample_without_replacement",
    "decode_distribution",
    "encode_distribution",
    "DIST_KEY",
]

DIST_KEY = "dist"


def _check_random_state(seed):
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, (int, np.integer)):
        return np.random.RandomState(int(seed))
    if isinstance(seed, np.random.RandomState):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a numpy RandomState")


class ParameterGrid:
    """Cartesian product over a dict (or list of dicts) of value lists.

    Iteration order and ``__getitem__`` indexing match sklearn exactly: keys are
    sorted, the product runs with the last sorted key varying fastest, and
    ``grid[i]`` is the ``i``-th element of that iteration.
    """

    def __init__(self, param_grid):
        if isinstance(param_grid, Mapping):
            param_grid = [param_grid]
        if not isinstance(param_grid, Sequence):
            raise TypeError(f"Parameter grid should be a dict or a list, got {param_grid!r}")
        for grid in param_grid:
            if not isinstance(grid, Mapping):
                raise TypeError(f"Parameter grid is not a dict ({grid!r})")
            for key, value in grid.items():
                if isinstance(value, np.ndarray) and value.ndim > 1:
                    raise ValueError(f"Parameter array for {key!r} should be one-dimensional")
                if isinstance(value, str) or not isinstance(value, (np.ndarray, Sequence)):
                    raise TypeError(
                        f"Parameter grid for parameter {key!r} needs to be a list or a numpy "
                        f"array, but got {value!r} (of type {type(value).__name__}) instead."
                    )
                if len(value) == 0:
                    raise ValueError(f"Parameter grid for parameter {key!r} need to be a non-empty sequence")
        self.param_grid = [dict(g) for g in param_grid]

    def __iter__(self) -> Iterator[Dict[str, Any]]:
        for grid in self.param_grid:
            items = sorted(grid.items())
            if not items:
                yield {}
                continue
            keys, values = zip(*items)
            for combo in product(*values):
                yield dict(zip(keys, combo))

    def __len__(self) -> int:
        return sum(math.prod(len(v) for v in g.values()) if g else 1 for g in self.param_grid)

    def __getitem__(self, ind: int) -> Dict[str, Any]:
        for grid in self.param_grid:
            if not grid:
                if ind == 0:
                    return {}
                ind -= 1
                continue
            # mixed-radix decode, least significant digit = last sorted key
            items = sorted(grid.items())[::-1]
            total = math.prod(len(v) for _, v in items)
            if ind >= total:
                ind -= total
                continue
            out = {}
            for key, values in items:
                ind, off = divmod(ind, len(values))
                out[key] = values[off]
            return out
        raise IndexError("ParameterGrid index out of range")


def sample_without_replacement(n_population: int, n_samples: int, random_state=None) -> np.ndarray:
    """Same draws as ``sklearn.utils.random.sample_without_replacement(method="auto")``.

    sklearn picks a permutation prefix when 0.01 < ratio < 0.99, a tracking-selection
    loop of ``randint`` rejections when ratio < 0.2, and reservoir sampling otherwise;
    each branch consumes the RNG the same way here, so the sampled candidate indices
    are identical.
    """
    if n_population < 0 or n_samples < 0 or n_samples > n_population:
        raise ValueError("invalid sample_without_replacement arguments")
    rng = _check_random_state(random_state)
    ratio = n_samples / n_population if n_population != 0 else 1.0
    if 0.01 < ratio < 0.99:
        return rng.permutation(n_population)[:n_samples]
    out = np.empty(n_samples, dtype=np.int64)
    if ratio >= 0.2:
        out[:] = np.arange(n_samples)
        for i in range(n_samples, n_population):
            j = rng.randint(0, i + 1)
            if j < n_samples:
                out[j] = i
        return out
    selected = set()
    for i in range(n_samples):
        j = rng.randint(n_population)
        while j in selected:
            j = rng.randint(n_population)
        selected.add(j)
        out[i] = j
    return out


# --------------------------------------------------------------------------------------
# serializable distributions (fix for D8)
# --------------------------------------------------------------------------------------
_SCIPY_NAMES = {
    "uniform": ("uniform", ("loc", "scale")),
    "loguniform": ("loguniform", ("a", "b")),
    "reciprocal": ("loguniform", ("a", "b")),
    "randint": ("randint", ("low", "high")),
    "norm": ("norm", ("loc", "scale")),
    "normal": ("norm", ("loc", "scale")),
    "expon": ("expon", ("loc", "scale")),
    "lognorm": ("lognorm", ("s", "loc", "scale")),
    "beta": ("beta", ("a", "b", "loc", "scale")),
    "gamma": ("gamma", ("a", "loc", "scale")),
    "truncnorm": ("truncnorm", ("a", "b", "loc", "scale")),
}


def decode_distribution(spec: Any):
    """Turn a JSON distribution spec into an object with ``rvs(random_state=)``.

    Lists stay lists (sampled by index like sklearn).  A dict carrying the
    ``"dist"`` key is decoded into a scipy frozen distribution.
    """
    if isinstance(spec, Mapping) and DIST_KEY in spec:
        name = str(spec[DIST_KEY]).lower()
        if name not in _SCIPY_NAMES:
            raise ValueError(f"unknown distribution {name!r}; known: {sorted(_SCIPY_NAMES)}")
        import scipy.stats as st

        sp_name, arg_names = _SCIPY_NAMES[name]
        kwargs = {k: spec[k] for k in arg_names if k in spec}
        return getattr(st, sp_name)(**kwargs)
    return spec


def encode_distribution(obj: Any) -> Any:
    """Client-side: scipy frozen distribution -> JSON spec (lists pass through)."""
    dist = getattr(obj, "dist", None)
    if dist is None or not hasattr(obj, "rvs"):
        return obj
    name = getattr(dist, "name", None)
    args, kwds = tuple(getattr(obj, "args", ())), dict(getattr(obj, "kwds", {}))
    for key, (sp_name, arg_names) in _SCIPY_NAMES.items():
        if sp_name == name and key == sp_name:
            spec = {DIST_KEY: key}
            for i, a in enumerate(args):
                spec[arg_names[i]] = float(a) if not isinstance(a, (int, np.integer)) else int(a)
            for k, v in kwds.items():
                spec[k] = float(v) if not isinstance(v, (int, np.integer)) else int(v)
            return spec
    raise ValueError(f"distribution {name!r} has no wire encoding")


class ParameterSampler:
    """Random candidates; draws identical to ``sklearn.model_selection.ParameterSampler``."""

    def __init__(self, param_distributions, n_iter: int, random_state=None):
        if isinstance(param_distributions, Mapping):
            param_distributions = [param_distributions]
        decoded = []
        for dist in param_distributions:
            if not isinstance(dist, Mapping):
                raise TypeError(f"Parameter distribution is not a dict ({dist!r})")
            d = {}
            for key, value in dist.items():
                value = decode_distribution(value)
                if not isinstance(value, (list, tuple, np.ndarray)) and not hasattr(value, "rvs"):
                    raise TypeError(
                        f"Parameter grid for parameter {key!r} is not iterable or a distribution (value={value!r})"
                    )
                d[key] = value
            decoded.append(d)
        self.param_distributions = decoded
        self.n_iter = int(n_iter)
        self.random_state = random_state

    def _is_all_lists(self) -> bool:
        return all(all(not hasattr(v, "rvs") for v in d.values()) for d in self.param_distributions)

    def __iter__(self):
        rng = _check_random_state(self.random_state)
        if self._is_all_lists():
            grid = ParameterGrid(self.param_distributions)
            size = len(grid)
            n_iter = self.n_iter
            if size < n_iter:
                warnings.warn(
                    f"The total space of parameters {size} is smaller than n_iter={self.n_iter}. "
                    f"Running {size} iterations. For exhaustive searches, use GridSearchCV.",
                    UserWarning,
                )
                n_iter = size
            for i in sample_without_replacement(size, n_iter, random_state=rng):
                yield grid[int(i)]
        else:
            for _ in range(self.n_iter):
                dist = rng.choice(self.param_distributions)
                params = {}
                for k, v in sorted(dist.items()):
                    if hasattr(v, "rvs"):
                        params[k] = v.rvs(random_state=rng)
                    else:
                        params[k] = v[rng.randint(len(v))]
                yield params

    def __len__(self) -> int:
        if self._is_all_lists():
            return min(self.n_iter, len(ParameterGrid(self.param_distributions)))
        return self.n_iter


def to_jsonable(v: Any) -> Any:
    """numpy scalar -> python scalar (candidate params go on the wire as JSON)."""
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, np.ndarray):
        return v.tolist()
    return v


def expand_candidates(search_type: str | None, search_params: Dict[str, Any], random_state=None) -> List[Dict[str, Any]]:
    """Candidate list for a job (``[{}]`` for a plain estimator)."""
    if not search_type:
        return [{}]
    if search_type == "GridSearchCV":
        grid = search_params.get("param_grid", {})
        return [{k: to_jsonable(v) for k, v in p.items()} for p in ParameterGrid(grid)]
    if search_type == "RandomizedSearchCV":
        dists = search_params.get("param_distributions", {})
        n_iter = int(search_params.get("n_iter", 10))
        rs = 42 if random_state is None else random_state
        return [{k: to_jsonable(v) for k, v in p.items()} for p in ParameterSampler(dists, n_iter, random_state=rs)]
    raise ValueError(f"unsupported search_type {search_type!r}")
