"""Search-space expansion, CV splits and scorers vs scikit-learn (the reference's
semantics: task_handler.py:186-236 expansion, worker.py:302-341 splits/scores)."""
import numpy as np
import pytest
import scipy.stats as st
import torch

from cs230_distributed_machine_learning_amd.search import cv as dcv
from cs230_distributed_machine_learning_amd.search import grid as dgrid
from cs230_distributed_machine_learning_amd.search import scoring as dsc

sk_ms = pytest.importorskip("sklearn.model_selection")


GRIDS = [
    {"C": [0.1, 1.0, 10.0, 100], "solver": ["liblinear", "lbfgs"]},
    {"n_estimators": [100, 200, 500], "max_depth": [10, 20, 50, None], "min_samples_split": [2, 5, 10],
     "min_samples_leaf": [1, 2, 4], "bootstrap": [True, False]},
    [{"a": [1, 2]}, {"b": ["x", "y", "z"], "c": [0]}],
    {},
]


@pytest.mark.parametrize("g", GRIDS)
def test_parameter_grid_order_and_indexing(g):
    ours = dgrid.ParameterGrid(g)
    ref = sk_ms.ParameterGrid(g)
    assert len(ours) == len(ref)
    assert list(ours) == list(ref)
    for i in range(len(ref)):
        assert ours[i] == ref[i]


def test_reference_grid_sizes():
    # results1.py:34-40 grid has 216 points; README grid 8 with subtask-1 = {C:0.1, liblinear}
    assert len(dgrid.ParameterGrid(GRIDS[1])) == 216
    assert dgrid.expand_candidates("GridSearchCV", {"param_grid": GRIDS[0]})[0] == {"C": 0.1, "solver": "liblinear"}
    assert dgrid.expand_candidates("GridSearchCV", {"param_grid": GRIDS[0]})[1] == {"C": 0.1, "solver": "lbfgs"}


@pytest.mark.parametrize("n_pop,n", [(10, 3), (216, 50), (8, 8), (1000, 5), (1000, 995), (5000, 10)])
@pytest.mark.parametrize("seed", [0, 42, 7])
def test_sample_without_replacement_matches_sklearn(n_pop, n, seed):
    from sklearn.utils.random import sample_without_replacement

    ref = sample_without_replacement(n_pop, n, random_state=seed)
    ours = dgrid.sample_without_replacement(n_pop, n, random_state=seed)
    assert np.array_equal(np.asarray(ref), ours)


@pytest.mark.parametrize("seed", [0, 42, 123])
def test_parameter_sampler_lists_matches_sklearn(seed):
    d = GRIDS[1]
    ref = list(sk_ms.ParameterSampler(d, 50, random_state=seed))
    ours = list(dgrid.ParameterSampler(d, 50, random_state=seed))
    assert ours == ref


def test_parameter_sampler_caps_n_iter():
    with pytest.warns(UserWarning):
        out = list(dgrid.ParameterSampler(GRIDS[0], 10, random_state=0))
    assert len(out) == 8


def test_parameter_sampler_distributions_match_sklearn():
    ref_d = {"C": st.loguniform(1e-3, 1e2), "alpha": st.uniform(0, 2), "k": [1, 3, 5], "n": st.randint(2, 9)}
    wire = {"C": {"dist": "loguniform", "a": 1e-3, "b": 1e2}, "alpha": {"dist": "uniform", "loc": 0, "scale": 2},
            "k": [1, 3, 5], "n": {"dist": "randint", "low": 2, "high": 9}}
    ref = list(sk_ms.ParameterSampler(ref_d, 20, random_state=3))
    ours = list(dgrid.ParameterSampler(wire, 20, random_state=3))
    assert len(ref) == len(ours)
    for a, b in zip(ref, ours):
        assert set(a) == set(b)
        for k in a:
            assert a[k] == pytest.approx(b[k])


def test_encode_distribution_roundtrip():
    for dist in (st.loguniform(0.01, 10), st.uniform(1, 3), st.randint(0, 5), st.norm(2, 0.5), st.expon(0, 2)):
        spec = dgrid.encode_distribution(dist)
        back = dgrid.decode_distribution(spec)
        a = dist.rvs(size=5, random_state=1)
        b = back.rvs(size=5, random_state=1)
        assert np.allclose(a, b)


@pytest.mark.parametrize("n,k", [(150, 5), (151, 5), (20, 3), (1000, 10)])
def test_kfold_folds_match_sklearn(n, k):
    folds = dcv.kfold_test_folds(n, k)
    for f, (_tr, te) in enumerate(sk_ms.KFold(k).split(np.zeros(n))):
        assert np.array_equal(np.flatnonzero(folds == f), te)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_stratified_folds_match_sklearn(seed):
    rng = np.random.RandomState(seed)
    y = rng.choice(["a", "b", "c"], size=173, p=[0.5, 0.3, 0.2])
    folds = dcv.stratified_test_folds(y, 5)
    for f, (_tr, te) in enumerate(sk_ms.StratifiedKFold(5).split(np.zeros(len(y)), y)):
        assert np.array_equal(np.flatnonzero(folds == f), te)


@pytest.mark.parametrize("ts,rs", [(0.25, 42), (0.2, 0), (30, 7), (0.33, None)])
def test_holdout_matches_train_test_split(ts, rs):
    n = 150
    idx = np.arange(n)
    if rs is None:
        return
    tr, te = sk_ms.train_test_split(idx, test_size=ts, random_state=rs)
    otr, ote = dcv.holdout_indices(n, ts, rs)
    assert np.array_equal(tr, otr) and np.array_equal(te, ote)


def test_split_roles_layout():
    y = np.array([0, 1] * 50)
    roles, names = dcv.make_split_roles(y, 5, True, holdout=True, test_size=0.2, random_state=0)
    assert names == ["cv0", "cv1", "cv2", "cv3", "cv4", "holdout"]
    assert roles.shape == (6, 100)
    assert ((roles[:5] == dcv.ROLE_TEST).sum(0) == 1).all()       # every row tested exactly once across folds
    assert (roles[5] == dcv.ROLE_TEST).sum() == 20


@pytest.mark.parametrize("name", ["accuracy", "balanced_accuracy", "f1_macro", "f1_micro", "f1_weighted",
                                  "precision_macro", "recall_macro", "recall_weighted", "jaccard_macro"])
def test_classification_scorers_match_sklearn(name):
    from sklearn import metrics as skm

    rng = np.random.RandomState(0)
    y = rng.randint(0, 3, 300)
    p = np.where(rng.rand(300) < 0.7, y, rng.randint(0, 3, 300))
    fn = {"accuracy": skm.accuracy_score, "balanced_accuracy": skm.balanced_accuracy_score}.get(name)
    if fn is None:
        base, avg = name.split("_")
        fn = {"f1": skm.f1_score, "precision": skm.precision_score, "recall": skm.recall_score,
              "jaccard": skm.jaccard_score}[base]
        ref = fn(y, p, average=avg)
    else:
        ref = fn(y, p)
    assert dsc.score(name, torch.from_numpy(y), torch.from_numpy(p), 3) == pytest.approx(ref)


def test_binary_scorers_match_sklearn():
    from sklearn import metrics as skm

    rng = np.random.RandomState(1)
    y = rng.randint(0, 2, 400)
    prob = np.clip(y * 0.6 + rng.rand(400) * 0.5, 0, 1)
    p = (prob > 0.5).astype(int)
    yt, pt = torch.from_numpy(y), torch.from_numpy(p)
    proba = torch.from_numpy(np.stack([1 - prob, prob], 1))
    assert dsc.score("f1", yt, pt, 2) == pytest.approx(skm.f1_score(y, p))
    assert dsc.score("precision", yt, pt, 2) == pytest.approx(skm.precision_score(y, p))
    assert dsc.score("recall", yt, pt, 2) == pytest.approx(skm.recall_score(y, p))
    assert dsc.score("roc_auc", yt, pt, 2, proba) == pytest.approx(skm.roc_auc_score(y, prob))
    assert dsc.score("neg_log_loss", yt, pt, 2, proba) == pytest.approx(-skm.log_loss(y, np.stack([1 - prob, prob], 1)))


@pytest.mark.parametrize("name", ["r2", "neg_mean_squared_error", "neg_mean_absolute_error",
                                  "neg_root_mean_squared_error", "explained_variance", "max_error",
                                  "neg_median_absolute_error"])
def test_regression_scorers_match_sklearn(name):
    from sklearn.metrics import get_scorer

    rng = np.random.RandomState(2)
    y = rng.randn(200) * 3 + 1
    p = y + rng.randn(200)

    class _Fixed:
        def predict(self, X):
            return p

    ref = get_scorer(name)(_Fixed(), np.zeros((200, 1)), y)
    assert dsc.score(name, torch.from_numpy(y), torch.from_numpy(p)) == pytest.approx(ref, rel=1e-9, abs=1e-12)


def test_validate_scoring():
    assert dsc.validate_scoring(None, True) == "accuracy"
    assert dsc.validate_scoring(None, False) == "r2"
    with pytest.raises(ValueError):
        dsc.validate_scoring("r2", True)


def test_stratified_holdout_matches_sklearn():
    """GradientBoosting's early-stopping split: train_test_split(..., stratify=y)."""
    from sklearn.model_selection import train_test_split

    from cs230_distributed_machine_learning_amd.search.cv import stratified_holdout_indices

    for seed in range(6):
        rng = np.random.default_rng(seed)
        y = rng.integers(0, 3 + seed % 3, size=97 + seed * 13)
        idx = np.arange(len(y))
        a, b = train_test_split(idx, test_size=0.1 + 0.05 * seed, random_state=seed, stratify=y)
        c, d = stratified_holdout_indices(y, 0.1 + 0.05 * seed, seed)
        assert np.array_equal(a, c) and np.array_equal(b, d)


@pytest.mark.parametrize("C", [2, 4])
@pytest.mark.parametrize("name", ["matthews_corrcoef", "jaccard_micro", "jaccard_weighted", "neg_brier_score",
                                  "average_precision", "roc_auc_ovr", "roc_auc_ovr_weighted", "roc_auc_ovo",
                                  "roc_auc_ovo_weighted", "top_k_accuracy"])
def test_more_classification_scorers_match_sklearn(name, C):
    """Scorer strings a GridSearchCV user passes, through sklearn's own scorer objects."""
    from sklearn.metrics import get_scorer

    if C == 2 and name.startswith("roc_auc_ov"):
        pytest.skip("multiclass-only scorer")
    if C > 2 and name in ("average_precision",):
        pytest.skip("binary-only scorer")
    rng = np.random.RandomState(5 + C)
    y = rng.randint(0, C, 500)
    logits = rng.randn(500, C) + 1.5 * np.eye(C)[y]
    logits = np.round(logits, 1)                    # some tied scores
    proba = np.exp(logits) / np.exp(logits).sum(1, keepdims=True)
    pred = proba.argmax(1)

    from sklearn.base import BaseEstimator, ClassifierMixin

    class _Fixed(ClassifierMixin, BaseEstimator):
        classes_ = np.arange(C)

        def predict(self, X):
            return pred

        def predict_proba(self, X):
            return proba

    ref = get_scorer(name)(_Fixed(), np.zeros((500, 1)), y)
    got = dsc.score(name, torch.from_numpy(y), torch.from_numpy(pred), C, torch.from_numpy(proba))
    assert got == pytest.approx(ref, rel=1e-9, abs=1e-12), (name, got, ref)


@pytest.mark.parametrize("name", ["neg_max_error", "neg_mean_squared_log_error", "neg_root_mean_squared_log_error",
                                  "neg_mean_poisson_deviance", "neg_mean_gamma_deviance", "d2_absolute_error_score",
                                  "neg_mean_absolute_percentage_error"])
def test_more_regression_scorers_match_sklearn(name):
    from sklearn.metrics import get_scorer

    rng = np.random.RandomState(3)
    y = np.abs(rng.randn(200) * 3) + 0.5
    p = np.abs(y + rng.randn(200) * 0.5) + 0.05

    class _Fixed:
        def predict(self, X):
            return p

    ref = get_scorer(name)(_Fixed(), np.zeros((200, 1)), y)
    got = dsc.score(name, torch.from_numpy(y), torch.from_numpy(p))
    assert got == pytest.approx(ref, rel=1e-9, abs=1e-12), (name, got, ref)


@pytest.mark.parametrize("name", ["positive_likelihood_ratio", "neg_negative_likelihood_ratio", "rand_score",
                                  "adjusted_rand_score", "fowlkes_mallows_score", "mutual_info_score",
                                  "normalized_mutual_info_score", "homogeneity_score", "completeness_score",
                                  "v_measure_score", "adjusted_mutual_info_score"])
@pytest.mark.parametrize("C", [2, 3])
def test_label_agreement_scorers_match_sklearn(name, C):
    from sklearn.metrics import get_scorer

    if C > 2 and "likelihood" in name:
        pytest.skip("binary-only scorer")
    rng = np.random.RandomState(11 + C)
    y = rng.randint(0, C, 300)
    pred = np.where(rng.rand(300) < 0.7, y, rng.randint(0, C, 300))

    class _Fixed:
        def predict(self, X):
            return pred

    ref = get_scorer(name)(_Fixed(), np.zeros((300, 1)), y)
    got = dsc.score(name, torch.from_numpy(y), torch.from_numpy(pred), C)
    assert got == pytest.approx(ref, rel=1e-9, abs=1e-12), (name, got, ref)
