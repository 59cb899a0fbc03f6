"""Cross-validation / holdout splits as per-row *role* vectors.

The reference worker does one holdout fit (``train_test_split``) plus
``cross_val_score(model, X, y, cv=5)`` per candidate
(``aws-prod/worker/worker.py:302-303,326,341``).  ``cross_val_score`` with an int
``cv`` uses ``StratifiedKFold(cv)`` for classifiers and ``KFold(cv)`` otherwise,
both unshuffled.  The holdout call is broken positionally (D1); here it is
implemented as intended: ``ShuffleSplit``-style permutation seeded by
``random_state`` with ``n_test = ceil(test_size * n)``.

Instead of materialising index copies per fold (the reference re-reads the full CSV
per task, ``worker.py:406-425``) every split is a ``uint8`` role vector of length
``n`` (0 = unused, 1 = train, 2 = test).  Kernels read the role of a row directly,
so one resident dataset copy serves every candidate x fold.
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np

ROLE_UNUSED, ROLE_TRAIN, ROLE_TEST = 0, 1, 2

__all__ = [
    "ROLE_UNUSED",
    "ROLE_TRAIN",
    "ROLE_TEST",
    "kfold_test_folds",
    "stratified_test_folds",
    "holdout_indices",
    "make_split_roles",
]


def kfold_test_folds(n: int, n_splits: int) -> np.ndarray:
    """Fold id per row for unshuffled ``KFold``."""
    if n_splits < 2 or n_splits > n:
        raise ValueError(f"Cannot have number of splits n_splits={n_splits} greater than the number of samples n_samples={n}.")
    sizes = np.full(n_splits, n // n_splits, dtype=np.int64)
    sizes[: n % n_splits] += 1
    return np.repeat(np.arange(n_splits, dtype=np.int32), sizes)


def stratified_test_folds(y: np.ndarray, n_splits: int) -> np.ndarray:
    """Fold id per row for unshuffled ``StratifiedKFold`` (same allocation as sklearn)."""
    y = np.asarray(y).ravel()
    _, y_idx, y_inv = np.unique(y, return_index=True, return_inverse=True)
    _, class_perm = np.unique(y_idx, return_inverse=True)
    y_enc = class_perm[y_inv]
    n_classes = len(y_idx)
    counts = np.bincount(y_enc)
    if np.all(n_splits > counts):
        raise ValueError(f"n_splits={n_splits} cannot be greater than the number of members in each class.")
    y_order = np.sort(y_enc)
    alloc = np.asarray([np.bincount(y_order[i::n_splits], minlength=n_classes) for i in range(n_splits)])
    folds = np.empty(len(y), dtype=np.int32)
    for k in range(n_classes):
        folds[y_enc == k] = np.arange(n_splits).repeat(alloc[:, k])
    return folds


def holdout_indices(n: int, test_size=0.2, random_state=None):
    """(train_idx, test_idx) exactly as ``train_test_split(..., shuffle=True)``."""
    if np.asarray(test_size).dtype.kind == "f":
        test_size = float(test_size)
        if not 0 < test_size < 1:
            raise ValueError(f"test_size={test_size} should be in the (0, 1) range")
        n_test = math.ceil(test_size * n)
    else:
        n_test = int(test_size)
        if not 0 < n_test < n:
            raise ValueError(f"test_size={n_test} should be smaller than the number of samples {n}")
    n_train = n - n_test
    if n_train <= 0:
        raise ValueError("resulting train set is empty")
    if random_state is None:
        rng = np.random.mtrand._rand
    elif isinstance(random_state, np.random.RandomState):
        rng = random_state
    else:
        rng = np.random.RandomState(int(random_state))
    perm = rng.permutation(n)
    return perm[n_test : n_test + n_train], perm[:n_test]


def _approximate_mode(class_counts: np.ndarray, n_draws: int, rng) -> np.ndarray:
    """sklearn.utils.extmath._approximate_mode: per-class draws closest to the class
    proportions, ties among equal remainders broken by ``rng``."""
    continuous = class_counts / class_counts.sum() * n_draws
    floored = np.floor(continuous)
    need = int(n_draws - floored.sum())
    if need > 0:
        remainder = continuous - floored
        for value in np.sort(np.unique(remainder))[::-1]:
            (inds,) = np.where(remainder == value)
            add_now = min(len(inds), need)
            inds = rng.choice(inds, size=add_now, replace=False)
            floored[inds] += 1
            need -= add_now
            if need == 0:
                break
    return floored.astype(int)


def stratified_holdout_indices(y: np.ndarray, test_size=0.1, random_state=None):
    """(train_idx, test_idx) exactly as ``train_test_split(..., stratify=y)``
    (StratifiedShuffleSplit's first split; GradientBoosting's early-stopping split)."""
    y = np.asarray(y)
    n = len(y)
    n_test = math.ceil(float(test_size) * n) if np.asarray(test_size).dtype.kind == "f" else int(test_size)
    n_train = n - n_test
    classes, y_idx = np.unique(y, return_inverse=True)
    counts = np.bincount(y_idx)
    if counts.min() < 2:
        raise ValueError("The least populated class in y has only 1 member, which is too few.")
    if n_train < len(classes) or n_test < len(classes):
        raise ValueError("train/test size should be greater or equal to the number of classes")
    class_indices = np.split(np.argsort(y_idx, kind="mergesort"), np.cumsum(counts)[:-1])
    if random_state is None:
        rng = np.random.mtrand._rand
    elif isinstance(random_state, np.random.RandomState):
        rng = random_state
    else:
        rng = np.random.RandomState(int(random_state))
    n_i = _approximate_mode(counts, n_train, rng)
    t_i = _approximate_mode(counts - n_i, n_test, rng)
    train, test = [], []
    for i in range(len(classes)):
        perm = class_indices[i].take(rng.permutation(counts[i]), mode="clip")
        train.extend(perm[:n_i[i]])
        test.extend(perm[n_i[i]:n_i[i] + t_i[i]])
    return rng.permutation(train), rng.permutation(test)


def make_split_roles(
    y: np.ndarray,
    cv: int,
    is_classifier: bool,
    holdout: bool = True,
    test_size=0.2,
    random_state=42,
) -> tuple[np.ndarray, List[str]]:
    """Stack of role vectors ``[n_splits_total, n]`` and their names.

    Row 0..cv-1 are the CV folds (names ``cv0..``); the optional last row is the
    holdout split (``holdout``).
    """
    n = len(y)
    roles: List[np.ndarray] = []
    names: List[str] = []
    if cv and cv >= 2:
        if is_classifier and _is_discrete(y):
            folds = stratified_test_folds(y, cv)
        else:
            folds = kfold_test_folds(n, cv)
        for f in range(cv):
            r = np.full(n, ROLE_TRAIN, dtype=np.uint8)
            r[folds == f] = ROLE_TEST
            roles.append(r)
            names.append(f"cv{f}")
    if holdout:
        tr, te = holdout_indices(n, test_size, random_state)
        r = np.zeros(n, dtype=np.uint8)
        r[tr] = ROLE_TRAIN
        r[te] = ROLE_TEST
        roles.append(r)
        names.append("holdout")
    if not roles:
        roles.append(np.full(n, ROLE_TRAIN, dtype=np.uint8))
        names.append("full")
    return np.stack(roles), names


def full_fit_roles(n: int) -> np.ndarray:
    return np.full((1, n), ROLE_TRAIN, dtype=np.uint8)


def _is_discrete(y: np.ndarray) -> bool:
    y = np.asarray(y)
    if y.dtype.kind in "OUSb":
        return True
    if y.dtype.kind in "iu":
        return True
    if y.dtype.kind == "f":
        return bool(np.all(np.mod(y, 1) == 0))
    return False
