"""Sharded dataset loads (parallel/data.py ``stage_host`` + ``sharded_load``).

Rank 0 stages the parsed table once in a memory-mappable host file; every rank copies only
its own 1/N row block to its device and one all-gather assembles the table -- N host links
in parallel instead of rank 0's single one (the reference re-reads the whole CSV per task,
aws-prod/worker/worker.py:406-425).  Runs over gloo with 3 ranks on CPU."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _table(n=1003, d=7):
    rng = np.random.RandomState(4)
    X = rng.randn(n, d).astype(np.float32)
    y = np.array(["b", "a", "c"], dtype=object)[rng.randint(0, 3, n)]
    return X, y


def _rank(rank, world, port, path, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1")
    from cs230_distributed_machine_learning_amd.parallel import data as pdata
    from cs230_distributed_machine_learning_amd.parallel import dist

    inf = dist.init(want_gpu=False, timeout_s=60)
    X, y, h2d = pdata.sharded_load(path, inf.device)
    outq.put((rank, X.numpy().tobytes(), list(y), h2d, tuple(X.shape)))
    dist.destroy()


def test_sharded_load_identical_tables_on_every_rank(tmp_path):
    from cs230_distributed_machine_learning_amd.parallel import data as pdata

    X, y = _table()
    path = pdata.stage_host(X, y, str(tmp_path / "t.npy"), threads=3)
    Xl, yl = pdata.load_staged(path, "cpu")          # the host-staged (joiner) path reads it too
    assert np.array_equal(Xl.numpy(), X) and list(yl) == list(y)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 3, port, path, q)) for r in range(3)]
    for p in procs:
        p.start()
    outs = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, xb, ys, h2d, shape in outs:
        assert shape == X.shape
        assert xb == X.tobytes(), rank          # byte-identical on every rank
        assert ys == list(y)
        assert h2d >= 0.0


def _grid_job(job_id, dataset, model, grid, cv=3):
    return {"job_id": job_id, "dataset_id": dataset, "model_details": {
        "model_type": model, "search_type": "GridSearchCV", "hyperparameters": {
            "base_estimator_params": {"n_estimators": 6, "random_state": 3}, "search_params": {"param_grid": grid},
            "cv_params": {"cv": cv}}}, "train_params": {"target_column": "target"}}


def _drive(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "classification?n=4000&d=9&seed=8", "dataset_name": "s",
                            "dataset_type": "synthetic"})
    st, a = ctl.train(sid, _grid_job("job-s", "s", "RandomForestClassifier", {"max_depth": [3, 5, None]}))
    ctl.table.wait_finished(a["job_id"], timeout=180)
    s = ctl.check_status(sid, a["job_id"])[1]
    return {"status": s["job_status"], "h2d": list(runner.core.load_h2d_s),
            "scores": {str(r["parameters"]["max_depth"]): r["cv_scores"] for r in s["job_result"]["results"]}}


def test_cluster_job_on_sharded_table_matches_local():
    """A job whose table loads sharded (DML_SHARD_LOAD_MIN_MB=0) returns the local runner's CV
    scores on 3 gloo ranks."""
    from tests.test_cluster import _launch
    from cs230_distributed_machine_learning_amd.config import Config
    from cs230_distributed_machine_learning_amd.engine.service import Controller

    r = _launch(3, _drive, env={"DML_SHARD_LOAD_MIN_MB": "0"})
    assert r["status"] == "completed" and r["h2d"], r      # rank 0 loaded through sharded_load
    root = tempfile.mkdtemp()
    ctl = Controller(Config.from_env(data_root=root, device="cpu", chunk_target_s=0.0))
    try:
        sid = ctl.create_session()[1]["session_id"]
        ctl.download_data(sid, {"dataset_url": "classification?n=4000&d=9&seed=8", "dataset_name": "s",
                                "dataset_type": "synthetic"})
        st, a = ctl.train(sid, _grid_job("job-s", "s", "RandomForestClassifier", {"max_depth": [3, 5, None]}))
        ctl.table.wait_finished(a["job_id"], timeout=180)
        s = ctl.check_status(sid, a["job_id"])[1]
        local = {str(x["parameters"]["max_depth"]): x["cv_scores"] for x in s["job_result"]["results"]}
    finally:
        ctl.shutdown()
    assert set(local) == set(r["scores"])
    for k in local:
        assert np.allclose(r["scores"][k], local[k], rtol=0, atol=1e-12), (k, r["scores"][k], local[k])
