"""The RCCL path on one MI355X: a real ``nccl`` (= RCCL) process group at world size 1.

The multi-GPU bench and the cluster runner call RCCL at N=8 on the driver's node; this
test makes every one of those calls execute on the one GPU we have (``DML_FORCE_PG=1``
builds the group even for one rank): ``all_gather_into_tensor``, ``broadcast``,
``all_reduce`` SUM/MAX, ``barrier(device_ids=...)``, the dataset broadcast + shared
bin edges, the row scatter of a data-parallel job, and then the DistributedRunner +
worker loop end to end (RF and LR grid searches, one row-sharded LR job) on that group.
Reference channels replaced: aws-prod/scheduler/scheduler_service.py:268-273 (Kafka
`train` routing), aws-prod/worker/worker.py:253 (Kafka `result`).
"""
import os
import socket
import threading

import numpy as np
import pytest
import torch

from cs230_distributed_machine_learning_amd.config import Config


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(model, grid, cv=3, par=None):
    tp = {"target_column": "species", "test_size": 0.25, "random_state": 0}
    if par:
        tp["parallelism"] = par
    return {"dataset_id": "iris", "train_params": tp,
            "model_details": {"model_type": model, "search_type": "GridSearchCV",
                              "hyperparameters": {"base_estimator_params": {}, "search_params": {"param_grid": grid},
                                                  "cv_params": {"cv": cv}}}}


@pytest.mark.gpu
def test_rccl_world1_collectives_and_cluster_runner(tmp_path, monkeypatch):
    for k, v in dict(DML_FORCE_PG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                     WORLD_SIZE="1", LOCAL_RANK="0").items():
        monkeypatch.setenv(k, v)
    from cs230_distributed_machine_learning_amd.engine.service import Controller
    from cs230_distributed_machine_learning_amd.parallel import data as pdata
    from cs230_distributed_machine_learning_amd.parallel import dist
    from cs230_distributed_machine_learning_amd.parallel.runner import DistributedRunner, WorkerCore

    dist.destroy()
    inf = dist.init(want_gpu=True, timeout_s=300)
    try:
        assert inf.backend == "nccl" and inf.is_dist and inf.device.type == "cuda"
        dev = inf.device
        x = torch.arange(24, dtype=torch.float32, device=dev).reshape(6, 4)
        assert torch.equal(dist.all_gather_rows(x), x)                 # all_gather_into_tensor
        b = x.clone()
        dist.broadcast(b, 0)
        assert torch.equal(b, x)
        s = x.clone()
        dist.all_reduce_sum(s)
        assert torch.equal(s, x)
        m = x.clone()
        dist.all_reduce_max(m)
        assert torch.equal(m, x)
        dist.barrier()                                                 # barrier(device_ids=[0])
        Xd, yh = pdata.broadcast_table(np.arange(40, dtype=np.float32).reshape(10, 4), np.arange(10), dev)
        assert Xd.device == dev and float(Xd.sum()) == float(np.arange(40).sum()) and len(yh) == 10
        torch.cuda.synchronize()

        core = WorkerCore(dev)
        runner = DistributedRunner(core)
        ctl = Controller(Config(data_root=str(tmp_path), device="cuda:0", chunk_target_s=0.0), runner=runner)
        t = threading.Thread(target=runner.serve_forever, daemon=True)
        t.start()
        try:
            sid = ctl.create_session()[1]["session_id"]
            assert ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris",
                                           "dataset_type": "sklearn"})[0] == 200
            out = {}
            for name, body in (("rf", _job("RandomForestClassifier", {"n_estimators": [10], "max_depth": [3, None]})),
                               ("lr", _job("LogisticRegression", {"C": [0.1, 1.0, 10.0]})),
                               ("lr_dp", _job("LogisticRegression", {"C": [1.0, 10.0]}, par="data"))):
                st, ack = ctl.train(sid, body)
                assert st in (200, 202), ack
                assert ctl.table.wait_finished(ack["job_id"], timeout=300)
                out[name] = (ctl.check_status(sid, ack["job_id"])[1], ctl.metrics(sid, ack["job_id"])[1])
        finally:
            runner.shutdown()
            t.join(timeout=120)
        for name, (status, metrics) in out.items():
            assert status["job_status"] == "completed", (name, status)
            assert status["best_result"]["mean_cv_score"] > 0.85, (name, status["best_result"])
        # task-parallel jobs: the final records' scores came from the job's scores epoch,
        # an all_gather_into_tensor on the RCCL group (parallel/runner.py), not the store copies
        for name in ("rf", "lr"):
            res = out[name][0]["job_result"]["results"]
            assert res and all(r.get("scores_via") == "rccl" for r in res), (name, [r.get("scores_via") for r in res])
        assert {m["worker_id"] for m in out["rf"][1]} == {"rank0"}
        assert {m["worker_id"] for m in out["lr_dp"][1]} == {"data-parallel"}
        assert all(js.transport == "rccl" for js in runner.jobs) and not runner.dead
    finally:
        dist.destroy()


@pytest.mark.gpu
def test_rccl_group_reforms_after_break(tmp_path, monkeypatch):
    """A side collective fails on the RCCL group (injected): the group is broken, rank 0
    re-forms it as communicator generation 1 (destroy + a fresh ``nccl`` init on the same
    store, parallel/dist.py regroup), and the next jobs travel by RCCL again -- a task-parallel
    job's scores all-gathered on the new group and a row-sharded job on its data-parallel
    communicator."""
    import time

    for k, v in dict(DML_FORCE_PG="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
                     WORLD_SIZE="1", LOCAL_RANK="0", DML_SIDE_TIMEOUT_S="20", DML_REGROUP_DELAY_S="0.2").items():
        monkeypatch.setenv(k, v)
    from cs230_distributed_machine_learning_amd.engine.service import Controller
    from cs230_distributed_machine_learning_amd.parallel import dist
    from cs230_distributed_machine_learning_amd.parallel.runner import DistributedRunner, WorkerCore

    dist.destroy()
    inf = dist.init(want_gpu=True, timeout_s=300)
    try:
        core = WorkerCore(inf.device)
        runner = DistributedRunner(core)
        ctl = Controller(Config(data_root=str(tmp_path), device="cuda:0", chunk_target_s=0.0), runner=runner)
        t = threading.Thread(target=runner.serve_forever, daemon=True)
        t.start()

        def run(name, body):
            st, ack = ctl.train(sid, dict(body, job_id=name))
            assert st in (200, 202), ack
            assert ctl.table.wait_finished(name, timeout=300)
            return ctl.check_status(sid, name)[1]

        try:
            sid = ctl.create_session()[1]["session_id"]
            assert ctl.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris",
                                           "dataset_type": "sklearn"})[0] == 200
            monkeypatch.setenv("DML_FAIL_RANK_IN", "0:scores")    # the next scores gather raises
            broken = run("rf-break", _job("RandomForestClassifier", {"n_estimators": [8], "max_depth": [3, None]}))
            t0 = time.time()
            while not runner.group_broken and time.time() - t0 < 60:
                time.sleep(0.05)
            monkeypatch.delenv("DML_FAIL_RANK_IN")
            t0 = time.time()
            while (runner.group_broken or runner.stats["regroups"] < 1) and time.time() - t0 < 120:
                time.sleep(0.05)
            assert runner.stats["regroups"] >= 1 and not runner.group_broken, runner.stats
            lr = run("lr-gen1", _job("LogisticRegression", {"C": [0.1, 1.0, 10.0]}))
            dp = run("lr-dp-gen1", _job("LogisticRegression", {"C": [1.0, 10.0]}, par="data"))
        finally:
            runner.shutdown()
            t.join(timeout=120)
        assert broken["job_status"] == "completed"
        for st in (lr, dp):
            assert st["job_status"] == "completed" and st["best_result"]["mean_cv_score"] > 0.85, st
        log = runner.job_log
        assert log["lr-gen1"]["transport"] == "rccl" and log["lr-gen1"]["generation"] >= 1, log
        assert all(r.get("scores_via") == "rccl" for r in lr["job_result"]["results"]), lr["job_result"]["results"]
        assert log["lr-dp-gen1"]["mode"] == "data" and log["lr-dp-gen1"]["generation"] >= 1, log
        assert dist.generation() >= 1 and dist.info().backend == "nccl"
    finally:
        dist.destroy()
