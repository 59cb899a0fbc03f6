"""Tables too large for HBM as float32: tree models train on streamed, binned-only data.

DeviceData(binned_only=True) streams the host rows (numpy / np.memmap) in chunks through
pinned buffers and keeps only the uint8 bins on the device; the edges come from the same
row sample the resident path uses, so bins, trees and CV scores are identical."""
import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.data.device import DeviceData
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.search.grid import ParameterGrid


def _table(n, d, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, d).astype(np.float32)
    y = (X[:, 0] + 0.5 * X[:, 1] ** 2 + 0.3 * rng.randn(n) > 0.4).astype(int)
    return X, y


def _scores(dd, model, grid):
    res = run_candidates(dd, JobSpec(model, list(ParameterGrid(grid)), cv=3), range(len(list(ParameterGrid(grid)))))
    assert all(r.ok for r in res), [r.error for r in res]
    return [r.result["cv_scores"] for r in res]


def _check(dev, n, d, chunk, tmp_path):
    X, y = _table(n, d)
    mm = np.lib.format.open_memmap(str(tmp_path / "X.npy"), mode="w+", dtype=np.float32, shape=X.shape)
    mm[:] = X
    mm.flush()
    Xmm = np.load(str(tmp_path / "X.npy"), mmap_mode="r")       # rows read from disk chunk by chunk
    res_dd = DeviceData(X, y, True, dev)
    bin_dd = DeviceData(Xmm, y, True, dev, binned_only=True, chunk_rows=chunk)
    assert bin_dd.X is None
    assert torch.equal(res_dd.edges.cpu(), bin_dd.edges.cpu())
    assert torch.equal(res_dd.binned().cpu(), bin_dd.binned().cpu())
    for model, grid in (("RandomForestClassifier", {"n_estimators": [8], "max_depth": [4, None]}),
                        ("GradientBoostingClassifier", {"n_estimators": [5], "max_depth": [2]})):
        assert _scores(res_dd, model, grid) == _scores(bin_dd, model, grid)
    with pytest.raises(ValueError, match="binned form"):
        run_candidates(bin_dd, JobSpec("LogisticRegression", [{"C": 1.0}], cv=3), [0])


def test_binned_only_cpu_matches_resident(tmp_path):
    _check("cpu", 5000, 9, 1234, tmp_path)


@pytest.mark.gpu
def test_binned_only_gpu_streaming_matches_resident(tmp_path):
    # > 200k rows: the edge sample path; small chunks: the pinned double-buffer pipeline
    _check("cuda:0", 260_000, 17, 50_000, tmp_path)
