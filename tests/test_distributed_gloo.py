"""Multi-process (gloo, world_size 2) runs of the distributed runtime on CPU.

Exercises the same code the MI355X ranks run over RCCL: store-based job announcement,
dataset broadcast, dynamic slice claiming, score all-reduce, result publication."""
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


def _rank_main(rank, world, port, root, outq):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    import threading

    from cs230_distributed_machine_learning_amd.config import Config
    from cs230_distributed_machine_learning_amd.parallel import dist
    from cs230_distributed_machine_learning_amd.parallel.runner import DistributedRunner, WorkerCore, worker_loop

    inf = dist.init(want_gpu=False, timeout_s=120)
    core = WorkerCore(inf.device)
    if rank == 0:
        from cs230_distributed_machine_learning_amd.engine.service import Controller

        cfg = Config.from_env(data_root=root, device="cpu", chunk_target_s=0.0)
        runner = DistributedRunner(core)
        ctl = Controller(cfg, runner=runner)

        def drive():
            try:
                sid = ctl.create_session()[1]["session_id"]
                ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
                body = {"dataset_id": "iris", "train_params": {"test_size": 0.25, "random_state": 42,
                                                               "target_column": "species"},
                        "model_details": {"model_type": "LogisticRegression", "search_type": "GridSearchCV",
                                          "hyperparameters": {"base_estimator_params": {},
                                                              "search_params": {"param_grid": {
                                                                  "C": [0.1, 1.0, 10.0, 100],
                                                                  "solver": ["liblinear", "lbfgs"]}},
                                                              "cv_params": {"cv": 5}}}}
                st, resp = ctl.train(sid, body)
                jid = resp["job_id"]
                ctl.table.wait_finished(jid, timeout=300)
                st, status = ctl.check_status(sid, jid)
                body2 = dict(body, model_details={"model_type": "RandomForestClassifier",
                                                  "search_type": "GridSearchCV",
                                                  "hyperparameters": {"base_estimator_params": {"n_estimators": 10, "random_state": 7},
                                                                      "search_params": {"param_grid": {
                                                                          "max_depth": [2, 4, None]}},
                                                                      "cv_params": {"cv": 3}}})
                st, resp2 = ctl.train(sid, body2)
                ctl.table.wait_finished(resp2["job_id"], timeout=300)
                st, status2 = ctl.check_status(sid, resp2["job_id"])
                metrics = ctl.metrics(sid, jid)[1]
                extra = []
                for model, grid in [("SVC", {"C": [0.5, 5.0], "kernel": ["rbf", "linear"]}),
                                    ("KNeighborsClassifier", {"n_neighbors": [3, 9], "weights": ["uniform", "distance"]}),
                                    ("GradientBoostingClassifier", {"n_estimators": [10, 30]}),
                                    ("PCA", {"n_components": [1, 2, 3]})]:
                    b = dict(body, model_details={"model_type": model, "search_type": "GridSearchCV",
                                                  "hyperparameters": {"base_estimator_params": {},
                                                                      "search_params": {"param_grid": grid},
                                                                      "cv_params": {"cv": 5}}})
                    st, r = ctl.train(sid, b)
                    ctl.table.wait_finished(r["job_id"], timeout=300)
                    extra.append((model, ctl.check_status(sid, r["job_id"])[1]))
                # the same LR grid row-sharded over both ranks (parallel/data_parallel.py)
                b3 = dict(body, train_params=dict(body["train_params"], parallelism="data"))
                st, r3 = ctl.train(sid, b3)
                ctl.table.wait_finished(r3["job_id"], timeout=300)
                status3 = ctl.check_status(sid, r3["job_id"])[1]
                b3 = status3.get("best_result") or {}
                status3["_resolved_model"] = ctl.models.resolve(b3.get("model_path"), b3.get("model_id"))
                # the RF grid row-sharded too (per-level histogram all-reduce, ops/forest_dp.py)
                b4 = dict(body2, train_params=dict(body2["train_params"], parallelism="data"))
                st, r4 = ctl.train(sid, b4)
                ctl.table.wait_finished(r4["job_id"], timeout=300)
                status4 = ctl.check_status(sid, r4["job_id"])[1]
                b4 = status4.get("best_result") or {}
                status4["_resolved_model"] = ctl.models.resolve(b4.get("model_path"), b4.get("model_id"))
                outq.put(("ok", status, status2, metrics, extra, status3, status4))
            except Exception as e:  # pragma: no cover
                import traceback

                outq.put(("err", traceback.format_exc()))
            finally:
                runner.shutdown()

        t = threading.Thread(target=drive, daemon=True)
        t.start()
        runner.serve_forever()
        t.join()
    else:
        worker_loop(core)
    dist.destroy()


def test_two_rank_gridsearch_gloo():
    root = tempfile.mkdtemp()
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, root, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = q.get(timeout=600)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert out[0] == "ok", out[1]
    status, status2, metrics = out[1], out[2], out[3]
    assert status["job_status"] == "completed" and status["total_subtasks"] == 8
    res = status["job_result"]["results"]
    assert len(res) == 8
    # the final records' scores came from the job's scores epoch (all_gather over the
    # group: gloo here, RCCL on the MI355X ranks), not from the per-slice store copies
    assert all(r.get("scores_via") == "gloo" for r in res), [r.get("scores_via") for r in res]
    assert all(r.get("scores_via") == "gloo" for r in status2["job_result"]["results"])
    best = status["best_result"]
    assert best["mean_cv_score"] >= 0.95
    assert len(best["cv_scores"]) == 5
    workers = {m["worker_id"] for m in metrics}
    assert workers <= {"rank0", "rank1"} and len(metrics) == 8
    assert status2["job_status"] == "completed" and len(status2["job_result"]["results"]) == 3
    assert status2["best_result"]["mean_cv_score"] > 0.9
    status3 = out[5]
    assert status3["job_status"] == "completed" and len(status3["job_result"]["results"]) == 8
    task_par = {(r["parameters"]["C"], r["parameters"]["solver"]): r for r in res}
    for r in status3["job_result"]["results"]:
        ref = task_par[(r["parameters"]["C"], r["parameters"]["solver"])]
        assert len(r["cv_scores"]) == 5
        if r["parameters"]["solver"] == "liblinear":   # same device solver, rows summed over 2 shards
            assert np.allclose(r["cv_scores"], ref["cv_scores"], atol=0.034), (r, ref)
    assert status3["best_result"]["mean_cv_score"] >= 0.95
    assert status3["_resolved_model"] and os.path.exists(status3["_resolved_model"])
    # row-sharded forests grow the task-parallel job's trees: identical CV and holdout scores
    status4 = out[6]
    assert status4["job_status"] == "completed", status4
    rf_task = {str(r["parameters"]["max_depth"]): r for r in status2["job_result"]["results"]}
    for r in status4["job_result"]["results"]:
        ref = rf_task[str(r["parameters"]["max_depth"])]
        assert r["cv_scores"] == ref["cv_scores"] and r.get("accuracy") == ref.get("accuracy"), (r, ref)
    assert status4["_resolved_model"] and os.path.exists(status4["_resolved_model"])
    for model, st in out[4]:
        assert st["job_status"] == "completed", (model, st)
        assert all("cv_scores" in r for r in st["job_result"]["results"]), model
        if model != "PCA":
            assert st["best_result"]["mean_cv_score"] > 0.9, (model, st["best_result"])
