"""Controller / gateway / client end-to-end on CPU (reference: master.py routes,
DistributedLibrary core.py client, J1-J8 contracts in SURVEY §3)."""
import json
import os
import socket
import time

import numpy as np
import pytest

from cs230_distributed_machine_learning_amd.config import Config
from cs230_distributed_machine_learning_amd.engine import jobs as jobsmod
from cs230_distributed_machine_learning_amd.engine.service import Controller
from cs230_distributed_machine_learning_amd.engine.model_store import load_model, predict

sklearn = pytest.importorskip("sklearn")
from sklearn.ensemble import RandomForestClassifier, RandomForestRegressor  # noqa: E402
from sklearn.linear_model import LinearRegression, LogisticRegression  # noqa: E402
from sklearn.model_selection import GridSearchCV, RandomizedSearchCV  # noqa: E402


@pytest.fixture
def ctl(tmp_path):
    cfg = Config(data_root=str(tmp_path / "data"), journal=str(tmp_path / "journal.jsonl"), device="cpu",
                 sse_interval_s=0.05)
    c = Controller(cfg)
    yield c
    c.shutdown()


def _wait(c, sid, jid, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        st, body = c.check_status(sid, jid)
        assert st == 200
        if body["job_status"] in ("completed", "failed"):
            return body
        time.sleep(0.05)
    raise AssertionError("job did not finish")


def _j1(job_id, model_type, params, search="GridSearchCV", search_params=None, cv=3, dataset="iris", target="target",
        scoring=None):
    """A J1 request in the client's layout (core.py _extract_model_details)."""
    sp = search_params or {"param_grid": params}
    return {"job_id": job_id, "dataset_id": dataset, "model_details": {
        "model_type": model_type, "search_type": search, "hyperparameters": {
            "base_estimator_params": {}, "search_params": sp, "cv_params": {"cv": cv, "scoring": scoring}}},
        "train_params": {"target_column": target}, "timestamp": "2026-01-01T00:00:00"}


def test_routes_and_sessions(ctl):
    st, home = ctl.home()
    assert st == 200 and "RandomForestClassifier" in home["models"]
    assert ctl.health()[0] == 200
    st, body = ctl.create_session()
    assert st == 201
    sid = body["session_id"]
    assert ctl.check_data("bogus", "iris")[0] == 404
    assert ctl.check_data(sid, "iris")[0] == 404
    assert ctl.download_data(sid, {"dataset_name": "iris"})[0] == 400
    st, _ = ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
    assert st == 200
    assert ctl.check_data(sid, "iris")[0] == 200
    assert ctl.check_data(sid, "../etc")[0] in (400, 404)
    # unknown dataset / bad params
    assert ctl.train(sid, _j1("j0", "LogisticRegression", {"C": [1.0]}, dataset="nope"))[0] == 404
    assert ctl.train(sid, _j1("j0", "NotAModel", {"C": [1.0]}))[0] == 400


def test_grid_job_contract(ctl):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
    grid = {"C": [0.1, 1.0, 10.0, 100], "solver": ["liblinear", "lbfgs"]}
    st, ack = ctl.train(sid, _j1("job-a", "LogisticRegression", grid, cv=5))
    assert st == 200 and ack["job_id"] == "job-a" and ack["total_subtasks"] == 8
    assert ctl.train(sid, _j1("job-a", "LogisticRegression", grid))[0] == 409     # duplicate id
    status = _wait(ctl, sid, "job-a")
    assert status["job_status"] == "completed" and status["tasks_pending"] == 0
    res = status["job_result"]["results"]
    assert len(res) == 8
    for r in res:
        assert len(r["cv_scores"]) == 5 and r["scoring"] == "accuracy"
        assert 0 <= r["mean_cv_score"] <= 1
    best = status["best_result"]
    assert best["mean_cv_score"] == max(r["mean_cv_score"] for r in res)
    assert best.get("model_path"), best     # refit of the job's best, whichever slice it ran in
    # north-star counters: 8 candidates x (5 CV + 1 holdout) fits, per job and per node
    assert status["fits_done"] == 48 and status["fits_per_s"] > 0
    health = ctl.health()[1]
    assert health["fits_done"] >= 48 and health["fits_per_s_since_start"] > 0
    # J8 records: one per subtask with J2 ids
    st, recs = ctl.metrics(sid, "job-a")
    assert st == 200 and len(recs) == 8
    for r in recs:   # GPU fields (None on this CPU controller) and slice throughput
        assert "gpu_id" in r and "hbm_peak_bytes" in r and r["slice_fits"] >= r["n_fits"] > 0
    ids = sorted(r["subtask_id"] for r in recs)
    assert ids == sorted(f"job-a-subtask-{i}" for i in range(1, 9))
    assert all(r["status"] == "DONE" for r in recs)          # J3 (worker.py:233-244)
    # best model stored, loadable without pickle, predicts
    st, f = ctl.download_model(sid, "job-a", {})
    assert st == 200 and f["__file__"].endswith(".npz")
    m = load_model(f["__file__"])
    from sklearn.datasets import load_iris

    iris = load_iris()
    names = np.asarray(iris.target_names)[iris.target]      # the registry stores class names
    acc = (np.asarray(predict(m, iris.data)).astype(str) == names).mean()
    assert acc > 0.9


def test_grid_scores_close_to_sklearn(ctl):
    """LR lbfgs CV scores agree with sklearn GridSearchCV on iris (converged problems)."""
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
    grid = {"C": [0.01, 0.1, 1.0]}
    ctl.train(sid, _j1("job-lr", "LogisticRegression", grid, cv=5))
    status = _wait(ctl, sid, "job-lr")
    from sklearn.datasets import load_iris

    X, y = load_iris(return_X_y=True)
    ref = GridSearchCV(LogisticRegression(max_iter=1000), grid, cv=5).fit(X, y)
    ours = {r["parameters"]["C"]: r["mean_cv_score"] for r in status["job_result"]["results"]}
    for C, m in zip(ref.cv_results_["param_C"], ref.cv_results_["mean_test_score"]):
        assert abs(ours[C] - m) <= 0.0134 + 1e-9, (C, ours[C], m)   # <= 1 sample per fold on 30-row folds


def test_randomized_and_regression(ctl):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "diabetes", "dataset_name": "diab", "dataset_type": "sklearn"})
    sp = {"param_distributions": {"n_estimators": [5, 10, 20], "max_depth": [2, 4, None],
                                  "min_samples_leaf": {"dist": "randint", "low": 1, "high": 6}},
          "n_iter": 4, "random_state": 7}
    st, ack = ctl.train(sid, _j1("job-r", "RandomForestRegressor", None, search="RandomizedSearchCV",
                                 search_params=sp, dataset="diab"))
    assert st == 200 and ack["total_subtasks"] == 4
    status = _wait(ctl, sid, "job-r")
    assert status["job_status"] == "completed"
    res = status["job_result"]["results"]
    assert all(r["scoring"] == "r2" for r in res)
    assert max(r["mean_cv_score"] for r in res) > 0.3
    # same candidates as sklearn's ParameterSampler
    from sklearn.model_selection import ParameterSampler
    import scipy.stats as st_

    ref = list(ParameterSampler({"n_estimators": [5, 10, 20], "max_depth": [2, 4, None],
                                 "min_samples_leaf": st_.randint(1, 6)}, 4, random_state=7))
    got = [{k: r["parameters"][k] for k in ("n_estimators", "max_depth", "min_samples_leaf")} for r in res]
    assert got == ref
    # linear regression single-candidate job
    ctl.train(sid, _j1("job-lin", "LinearRegression", {"fit_intercept": [True, False]}, dataset="diab"))
    s2 = _wait(ctl, sid, "job-lin")
    from sklearn.datasets import load_diabetes

    X, y = load_diabetes(return_X_y=True)
    ref = GridSearchCV(LinearRegression(), {"fit_intercept": [True, False]}, cv=3).fit(X, y)
    ours = {r["parameters"]["fit_intercept"]: r["mean_cv_score"] for r in s2["job_result"]["results"]}
    for fi, m in zip(ref.cv_results_["param_fit_intercept"], ref.cv_results_["mean_test_score"]):
        assert ours[fi] == pytest.approx(m, abs=1e-4)


def test_sse_stream(ctl):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
    st, stream = ctl.train_status(sid, _j1("job-s", "RandomForestClassifier", {"n_estimators": [5, 10]}))
    assert st == 200
    events = [json.loads(e[len("data: "):]) for e in stream]
    assert events[-1]["job_status"] == "completed"
    assert all("progress" in e or "completed_subtasks" in e or "job_status" in e for e in events)


def test_journal_resume(tmp_path):
    """A job journaled as submitted but never finished is re-run after a restart (D10)."""
    cfg = Config(data_root=str(tmp_path / "d"), journal=str(tmp_path / "j.jsonl"), device="cpu")
    t = jobsmod.JobTable(cfg.journal)
    sid = t.create_session()
    req = {**_j1("jr", "LogisticRegression", {"C": [1.0, 2.0]}), "session_id": sid}
    subs = jobsmod.make_subtasks(req, [{"C": 1.0}, {"C": 2.0}], 3)
    job = t.create_job(req, subs)
    t.finish_subtask("jr", job.subtasks[0].subtask_id, "completed",
                     result={"mean_cv_score": 0.5, "parameters": {"C": 1.0}})
    # restart: a fresh table replays the journal
    t2 = jobsmod.JobTable(cfg.journal)
    pending = t2.replay()
    assert [j.job_id for j in pending] == ["jr"]
    j2 = t2.get(sid, "jr")
    assert j2.subtasks[0].status == "completed" and j2.subtasks[1].status != "completed"
    # exactly-once: repeating a finish is ignored
    t2.finish_subtask("jr", j2.subtasks[0].subtask_id, "completed", result={"mean_cv_score": 0.1})
    assert j2.subtasks[0].result["mean_cv_score"] == 0.5
    # a Controller on that journal runs the remaining subtask to completion
    from sklearn.datasets import load_iris
    import pandas as pd

    os.makedirs(os.path.join(cfg.data_root, "datasets", "iris"), exist_ok=True)
    X, y = load_iris(return_X_y=True)
    df = pd.DataFrame(X, columns=[f"f{i}" for i in range(4)])
    df["target"] = y
    df.to_csv(os.path.join(cfg.data_root, "datasets", "iris", "iris.csv"), index=False)
    c = Controller(cfg)
    try:
        assert c._resumed == 1
        st = _wait(c, sid, "jr")
        assert st["job_status"] == "completed"
        assert st["job_result"]["results"][0]["mean_cv_score"] == 0.5   # not recomputed
    finally:
        c.shutdown()


def test_preprocess_titanic_list_form(ctl, tmp_path):
    import pandas as pd

    rng = np.random.RandomState(0)
    n = 200
    df = pd.DataFrame({
        "PassengerId": np.arange(n), "Survived": rng.randint(0, 2, n), "Pclass": rng.randint(1, 4, n),
        "Name": [f"n{i}" for i in range(n)], "Sex": rng.choice(["male", "female"], n),
        "Age": np.where(rng.rand(n) < 0.2, np.nan, rng.rand(n) * 70), "SibSp": rng.randint(0, 4, n),
        "Parch": rng.randint(0, 3, n), "Ticket": ["t"] * n, "Fare": rng.rand(n) * 100,
        "Cabin": [None] * n, "Embarked": rng.choice(["S", "C", "Q", None], n)})
    src = tmp_path / "titanic.csv"
    df.to_csv(src, index=False)
    sid = ctl.create_session()[1]["session_id"]
    assert ctl.download_data(sid, {"dataset_url": str(src), "dataset_name": "titanic", "dataset_type": "local"})[0] == 200
    yaml_text = open(os.path.join(os.path.dirname(__file__), "fixtures", "titanic_preprocess.yaml")).read()
    st, body = ctl.preprocess(sid, {"dataset_id": "titanic", "yaml": yaml_text})
    assert st == 200, body
    path = ctl.registry.find_file("titanic")
    out = pd.read_csv(path)
    assert list(out.columns)[-1] == "Survived"
    assert "Sex_male" in out.columns and "Embarked_S" in out.columns and "Pclass_1" in out.columns
    for c in ("Cabin", "Ticket", "Name", "PassengerId", "Sex"):
        assert c not in out.columns
    assert out["Age"].isna().sum() == 0
    assert abs(out["Fare"].mean()) < 1e-6 and abs(out["Fare"].std() - 1) < 1e-6
    # training on the preprocessed table works
    st, ack = ctl.train(sid, _j1("job-t", "RandomForestClassifier", {"max_depth": [3, 5]}, dataset="titanic",
                                 target="Survived"))
    assert st == 200
    assert _wait(ctl, sid, "job-t")["job_status"] == "completed"


def test_scheduler_routes(ctl):
    st, body = ctl.subscribe({"host": "h1", "mem_capacity_mb": 1024, "device": "cpu"})
    wid = body["worker_id"]
    assert ctl.heartbeat({"worker_id": wid})[0] == 200
    assert ctl.heartbeat({"worker_id": "nope"})[0] == 404
    st, ws = ctl.workers()
    assert any(w["worker_id"] == wid for w in ws)
    assert ctl.queues()[0] == 200
    assert ctl.unsubscribe({"worker_id": wid})[0] == 200


def test_local_client_e2e(ctl, tmp_path):
    from distributed_ml import MLTaskManager

    m = MLTaskManager(controller=ctl)
    assert m.download_data("iris", "iris", "sklearn")["message"].startswith("Dataset downloaded")
    g = GridSearchCV(RandomForestClassifier(n_estimators=10), {"max_depth": [2, None], "min_samples_leaf": [1, 3]},
                     cv=3)
    out = m.train(g, "iris", {"target_column": "target"}, wait_for_completion=True, polling_interval=0.05)
    assert out["job_status"] == "completed"
    st = m.check_job_status()
    assert st["total_subtasks"] == 4 and st["best_result"]["mean_cv_score"] > 0.85
    p = m.download_best_model(dest=str(tmp_path / "best.npz"))
    assert os.path.exists(p)
    # RandomizedSearchCV with a scipy distribution is serialised (D7/D8)
    import scipy.stats as sst

    r = RandomizedSearchCV(LogisticRegression(max_iter=300), {"C": sst.loguniform(1e-2, 1e1)}, n_iter=3,
                           random_state=0, cv=3)
    out = m.train(r, "iris", {"target_column": "target"}, wait_for_completion=True, polling_interval=0.05)
    assert out["job_status"] == "completed" and out["total_subtasks"] == 3
    ref = [p["C"] for p in __import__("sklearn.model_selection", fromlist=["x"]).ParameterSampler(
        {"C": sst.loguniform(1e-2, 1e1)}, 3, random_state=0)]
    got = sorted(r_["parameters"]["C"] for r_ in out["job_result"]["results"])
    assert np.allclose(sorted(ref), got)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_http_gateway_roundtrip(ctl):
    from cs230_distributed_machine_learning_amd.gateway.app import serve
    from distributed_ml import MLTaskManager

    port = _free_port()
    server = serve(ctl, "127.0.0.1", port, block=False)
    try:
        for _ in range(200):
            if server.started:
                break
            time.sleep(0.05)
        m = MLTaskManager(f"http://127.0.0.1:{port}")
        assert "message" in m.download_data("iris", "iris", "sklearn")
        assert "status" in m.check_data("iris")
        g = GridSearchCV(LogisticRegression(max_iter=200), {"C": [0.5, 5.0]}, cv=3)
        out = m.train(g, "iris", {"target_column": "target"}, wait_for_completion=True, polling_interval=0.05)
        assert out["job_status"] == "completed"
        # streamed (SSE) variant
        last = m.train(g, "iris", {"target_column": "target"}, stream=True)   # final J7 event
        assert last["job_status"] == "completed" and len(last["job_result"]["results"]) == 2
        recs = m.metrics()
        assert len(recs) == 2
        dest = m.download_best_model(dest=os.path.join(ctl.config.data_root, "dl.npz"))
        assert os.path.getsize(dest) > 0
        import requests

        r = requests.get(f"http://127.0.0.1:{port}/check_status/{m.session_id}/missing")
        assert r.status_code == 404
    finally:
        server.should_exit = True
        time.sleep(0.3)


def test_session_fair_share(tmp_path):
    """A one-candidate job of session B overtakes a 20-candidate search of session A."""
    cfg = Config(data_root=str(tmp_path / "d"), device="cpu", chunk_target_s=0.0)
    c = Controller(cfg)
    try:
        sa = c.create_session()[1]["session_id"]
        sb = c.create_session()[1]["session_id"]
        c.download_data(sa, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
        big = _j1("big", "RandomForestClassifier", {"n_estimators": [20, 30, 40, 50, 60], "max_depth": [2, 3, 4, None]})
        assert c.train(sa, big)[0] == 200
        assert c.train(sb, _j1("small", "LogisticRegression", {"C": [1.0]}))[0] == 200
        assert c.table.wait_finished("small", timeout=120)
        st_big = c.check_status(sa, "big")[1]
        assert st_big["job_status"] != "completed" and st_big["tasks_pending"] > 0
        assert c.table.wait_finished("big", timeout=300)
        assert c.check_status(sa, "big")[1]["job_status"] == "completed"
    finally:
        c.shutdown()


def test_keep_models_all_returns_every_candidate_model(tmp_path):
    """``keep_models="all"``: every candidate's holdout model is stored and its J4 result
    carries ``model_path``/``model_id`` (reference worker.py:351-361); the client downloads a
    NON-best candidate's model by that path (core.py:201-206)."""
    cfg = Config(data_root=str(tmp_path / "data"), device="cpu", keep_models="all")
    c = Controller(cfg)
    try:
        sid = c.create_session()[1]["session_id"]
        c.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
        st, ack = c.train(sid, _j1("job-k", "RandomForestClassifier", {"max_depth": [1, 3, None]}, cv=3))
        assert st in (200, 202), ack
        status = _wait(c, sid, "job-k")
        assert status["job_status"] == "completed"
        res = status["job_result"]["results"]
        assert len(res) == 3 and all(r.get("model_path") and r.get("model_id") for r in res)
        best = status["best_result"]
        other = [r for r in res if r["model_path"] != best["model_path"]][0]
        st, f = c.download_model(sid, "job-k", {"model_path": other["model_path"], "model_id": other["model_id"]})
        assert st == 200 and f["__file__"].endswith(".npz")
        m = load_model(f["__file__"])
        assert m["kind"] == "forest" and m["params"]["max_depth"] == (other["parameters"]["max_depth"] or 2**31 - 1)
        from sklearn.datasets import load_iris

        iris = load_iris()
        names = np.asarray(iris.target_names)[iris.target]
        assert (np.asarray(predict(m, iris.data)).astype(str) == names).mean() > 0.6
    finally:
        c.shutdown()


def test_refit_attaches_model_when_best_ran_in_an_early_slice(tmp_path):
    """One candidate per slice: the winner's result is published long before the job ends,
    and the refit model path must still land on it (J5 best_result.model_path)."""
    c = Controller(Config(data_root=str(tmp_path / "data"), device="cpu", chunk_target_s=0.0))
    try:
        sid = c.create_session()[1]["session_id"]
        c.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
        # the most expensive (first-run, LPT) candidates are the best ones here
        grid = {"n_estimators": [1, 2, 3, 40], "max_depth": [1, None]}
        c.train(sid, _j1("job-r", "RandomForestClassifier", grid, cv=3))
        status = _wait(c, sid, "job-r")
        best = status["best_result"]
        assert status["job_status"] == "completed" and best.get("model_path"), best
        assert os.path.exists(best["model_path"])
    finally:
        c.shutdown()
