"""Regression fixed point on heavy-tailed targets (forest_common.h reg_exponents_counts).

Both forest builders sum w, w*yq and w*y2q as 64-bit integers on one grid per build.
The y^2 grid used to be n * max|y|^2 * 2^-61: one outlier made every small target's
y^2 quantise to 0, so nodes of small targets looked pure and stopped splitting where
sklearn (float64 sums) keeps going.  The grid now follows the targets' total energy
(sum y^2, from an exact exponent histogram), and these tests pin the trees of such a
target against sklearn's: fully grown trees on integer features end in one leaf per
distinct feature cell, whatever the split order, so leaf counts and leaf means must
agree exactly.
"""
import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.service import refit_model
from cs230_distributed_machine_learning_amd.ops.forest_ops import (EXP_BINS, reg_exponent_counts, reg_exponents,
                                                                   reg_exponents_of_counts)
from cs230_distributed_machine_learning_amd.utils import native

sklearn = pytest.importorskip("sklearn")


def _heavy_tailed(n=2000, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 6, size=(n, 3)).astype(np.float32)
    y = (rng.random(n) * 1e-3 + 1e-4 * X[:, 0]).astype(np.float32)   # small targets ...
    y[rng.integers(0, n)] = 1e4                                      # ... and one outlier
    return X, y


def _old_rule(max_abs_y, n):
    import math
    kw, k = math.frexp(15.0 * n)[1], math.frexp(max_abs_y)[1]
    return 61 - kw - k, 61 - kw - 2 * k


def test_y2_grid_resolves_small_targets_beside_an_outlier():
    X, y = _heavy_tailed()
    e1, e2 = reg_exponents(y, len(y))
    # the old grid zeroed y^2 of most small targets; the new one resolves them
    y2 = y.astype(np.float64) ** 2
    assert np.mean(np.rint(y2 * 2.0 ** _old_rule(1e4, len(y))[1]) == 0) > 0.5
    assert np.mean(np.rint(y2 * 2.0 ** e2) == 0) < 0.01
    assert np.median(np.rint(y2 * 2.0 ** e2)) >= 100
    # the bound still holds: 15 * sum over all rows < 2^61 on both channels
    yd = y.astype(np.float64)
    assert 15 * np.abs(np.rint(yd * 2.0 ** e1)).sum() < 2.0 ** 62
    assert 15 * np.rint(yd * yd * 2.0 ** e2).sum() < 2.0 ** 62


def test_exponent_rule_python_equals_c_and_torch():
    rng = np.random.default_rng(1)
    lib = native.cpu_lib()
    for trial in range(20):
        T, n = int(rng.integers(1, 4)), int(rng.integers(1, 500))
        scale = 10.0 ** rng.uniform(-30, 30, size=(T, 1))
        Y = (rng.standard_t(1.5, size=(T, n + 7)) * scale).astype(np.float32)
        Y[rng.random(Y.shape) < 0.2] = 0.0
        c_np = reg_exponent_counts(Y, n, n + 7, T)
        c_t = reg_exponent_counts(torch.from_numpy(Y), n, n + 7, T)
        assert np.array_equal(c_np, c_t.numpy())
        assert c_np.shape == (T, EXP_BINS) and c_np.sum() == T * n
        out = np.zeros(2, np.int32)
        lib.dml_reg_exponents(native.ptr(np.ascontiguousarray(c_np)), T, native.ptr(out))
        assert tuple(out) == reg_exponents_of_counts(c_np), trial


def _leaves_match_sklearn(device):
    from sklearn.ensemble import RandomForestRegressor

    X, y = _heavy_tailed()
    params = {"n_estimators": 1, "bootstrap": False, "max_features": None, "random_state": 0}
    m = refit_model({"model_type": "RandomForestRegressor", "scoring": None}, params,
                    DeviceData(X, y, False, device))
    sk = RandomForestRegressor(**params).fit(X, y).estimators_[0].tree_
    nodes, vals = np.asarray(m["nodes"]), np.asarray(m["vals"])
    lv = nodes[:, 0] < 0
    ref = np.sort(sk.value[sk.children_left == -1][:, 0, 0])
    assert len(ref) == len(np.unique(X, axis=0))    # sklearn: one leaf per feature cell
    assert lv.sum() == len(ref)
    np.testing.assert_allclose(np.sort(vals[lv, 1] / vals[lv, 0]), ref, rtol=1e-6, atol=1e-9)


def test_heavy_tailed_target_tree_matches_sklearn_host():
    _leaves_match_sklearn("cpu")


@pytest.mark.gpu
def test_heavy_tailed_target_tree_matches_sklearn_gpu():
    _leaves_match_sklearn("cuda")


@pytest.mark.gpu
def test_exponent_histogram_kernel_matches_numpy():
    """gbrt.hip k_exp_hist (boosting recounts every stage's targets on the device) against the
    numpy histogram, multi-target with a row stride, zeros and a wide dynamic range."""
    rng = np.random.default_rng(4)
    for T, n, stride in ((1, 100_003, 100_003), (5, 70_000, 70_016)):
        Y = (rng.standard_t(1.3, size=(T, stride)) * 10.0 ** rng.uniform(-20, 20, size=(T, 1))).astype(np.float32)
        Y[rng.random(Y.shape) < 0.1] = 0.0
        want = reg_exponent_counts(Y, n, stride if T > 1 else 0, T)
        got = reg_exponent_counts(torch.from_numpy(Y).to("cuda").reshape(-1)[: (T - 1) * stride + n] if T > 1
                                  else torch.from_numpy(Y[0, :n]).to("cuda"), n, stride if T > 1 else 0, T)
        assert np.array_equal(got.cpu().numpy(), want)
    bad = torch.tensor([1.0, float("nan"), 2.0], device="cuda")
    with pytest.raises(ValueError):
        reg_exponent_counts(bad, 3)


def test_packed_word_bound_from_exponents():
    """The large tier packs a row's count above its biased fixed-point target only when every
    |yq| < 2^39 (forest.hip kPackShift): ops/forest_ops.py reads max |y| < 2^kmax from the exponent
    histogram and requires kmax + e1 <= 38.  Check kmax and that the rule holds for the grid."""
    from cs230_distributed_machine_learning_amd.ops.forest_ops import _max_exponent, reg_exponents_of_counts

    rng = np.random.RandomState(0)
    for scale, n in ((1.0, 800_000), (1e-3, 50_000), (37.0, 3_000), (0.0, 10)):
        y = (rng.uniform(-1, 1, n) * scale).astype(np.float32)
        cnt = reg_exponent_counts(y, n)
        kmax = _max_exponent(cnt)
        if scale == 0.0:
            assert kmax is None
            continue
        assert np.all(np.abs(y) < 2.0 ** kmax) and np.any(np.abs(y) >= 2.0 ** (kmax - 1))
        e1, _ = reg_exponents_of_counts(cnt)
        yq = np.rint(y.astype(np.float64) * 2.0 ** e1)
        if kmax + e1 <= 38:   # packed: the biased sum over 3,840 rows never reaches the count bits
            assert np.abs(yq).max() < 2.0 ** 39
            assert 3840 * (np.abs(yq).max() + 2.0 ** 39) < 2.0 ** 52
