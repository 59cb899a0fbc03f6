"""Cluster runner behaviour over real multi-process groups (gloo on CPU).

* concurrent jobs: the dispatcher interleaves the slices of every active job across every
  rank with slice-level session fair share, so a one-candidate job of session B finishes
  while session A's 20-candidate search is still running (reference scheduler: every
  job's tasks interleaved over every worker, aws-prod/scheduler/scheduler_service.py:173-191,
  249-293; the local-runner version of this is tests/test_service.py);
* elastic membership: a process outside the launch world joins the running service,
  receives slices (host-staged dataset) and leaves on /unsubscribe (reference
  aws-prod/scheduler/scheduler.py:105-139).
"""
import os
import socket
import tempfile
import time

import pytest
import torch.multiprocessing as mp

from cs230_distributed_machine_learning_amd.config import Config
from cs230_distributed_machine_learning_amd.engine.service import Controller


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _grid_job(job_id, dataset, model, grid, cv=3, base=None, target="target"):
    return {"job_id": job_id, "dataset_id": dataset, "model_details": {
        "model_type": model, "search_type": "GridSearchCV", "hyperparameters": {
            "base_estimator_params": base or {}, "search_params": {"param_grid": grid}, "cv_params": {"cv": cv}}},
        "train_params": {"target_column": target}}


def _serve(rank, world, port, root, outq, drive_fn, env=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), OMP_NUM_THREADS="1", **(env or {}))
    import threading

    from cs230_distributed_machine_learning_amd.parallel import dist
    from cs230_distributed_machine_learning_amd.parallel.runner import DistributedRunner, WorkerCore, worker_loop

    inf = dist.init(want_gpu=False, timeout_s=120)
    core = WorkerCore(inf.device)
    if rank == 0:
        cfg = Config.from_env(data_root=root, device="cpu", chunk_target_s=0.0)
        runner = DistributedRunner(core)
        ctl = Controller(cfg, runner=runner)

        def drive():
            try:
                outq.put(("ok", drive_fn(ctl, runner)))
            except Exception:  # pragma: no cover
                import traceback

                outq.put(("err", traceback.format_exc()))
            finally:
                runner.shutdown()

        t = threading.Thread(target=drive, daemon=True)
        t.start()
        runner.serve_forever()
        t.join()
        time.sleep(0.5)
    else:
        worker_loop(core)
    os._exit(0)


def _launch(world, drive_fn, extra=None, timeout=300, env=None):
    root = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve, args=(r, world, port, root, q, drive_fn, env)) for r in range(world)]
    for p in procs:
        p.start()
    others = [ctx.Process(target=fn, args=(port,)) for fn in (extra or [])]
    for p in others:
        p.start()
    try:
        out = q.get(timeout=timeout)
    finally:
        deadline = time.time() + 60
        for p in procs + others:
            p.join(timeout=max(1, deadline - time.time()))
            if p.is_alive():
                p.kill()
    assert out[0] == "ok", out[1]
    return out[1]


def _drive_fair_share(ctl, runner):
    sa = ctl.create_session()[1]["session_id"]
    sb = ctl.create_session()[1]["session_id"]
    ctl.download_data(sa, {"dataset_url": "classification?n=30000&d=20&seed=3", "dataset_name": "big",
                           "dataset_type": "synthetic"})
    ctl.download_data(sb, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
    grid = {"min_samples_leaf": list(range(1, 21))}
    st, a = ctl.train(sa, _grid_job("job-a", "big", "RandomForestClassifier", grid, base={"n_estimators": 30}))
    assert st in (200, 202), a
    time.sleep(0.5)   # A is running on every rank
    st, b = ctl.train(sb, _grid_job("job-b", "iris", "LogisticRegression", {"C": [1.0]}, target="species"))
    assert st in (200, 202), b
    ctl.table.wait_finished(b["job_id"], timeout=240)
    a_when_b_done = ctl.check_status(sa, a["job_id"])[1]
    b_status = ctl.check_status(sb, b["job_id"])[1]
    ctl.table.wait_finished(a["job_id"], timeout=240)
    a_final = ctl.check_status(sa, a["job_id"])[1]
    a_metrics = ctl.metrics(sa, a["job_id"])[1]
    return a_when_b_done, b_status, a_final, a_metrics


def test_concurrent_jobs_small_job_overtakes_search():
    a_mid, b, a_final, a_metrics = _launch(2, _drive_fair_share)
    assert b["job_status"] == "completed" and len(b["job_result"]["results"]) == 1
    assert a_mid["job_status"] != "completed", a_mid      # B finished while A was still running
    assert a_final["job_status"] == "completed" and len(a_final["job_result"]["results"]) == 20
    assert {m["worker_id"] for m in a_metrics} == {"rank0", "rank1"}   # A ran on both ranks


def _joiner(port):
    os.environ.update(OMP_NUM_THREADS="1")
    import torch

    from cs230_distributed_machine_learning_amd.parallel.runner import join_cluster

    time.sleep(1.0)
    join_cluster("127.0.0.1", port, torch.device("cpu"))
    os._exit(0)


def _drive_join(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "classification?n=6000&d=10&seed=5", "dataset_name": "mid",
                            "dataset_type": "synthetic"})
    t0 = time.time()
    while not any(not w.in_group and w.alive for w in runner.workers.values()):
        if time.time() - t0 > 60:
            raise RuntimeError("joiner never arrived")
        time.sleep(0.1)
    grid = {"min_samples_leaf": list(range(1, 25))}
    st, a = ctl.train(sid, _grid_job("job-j", "mid", "RandomForestClassifier", grid, base={"n_estimators": 20}))
    ctl.table.wait_finished(a["job_id"], timeout=240)
    status = ctl.check_status(sid, a["job_id"])[1]
    metrics = ctl.metrics(sid, a["job_id"])[1]
    joined = [w for w in runner.workers.values() if not w.in_group]
    sched_id = runner.worker_ids[joined[0].wid]
    sub = ctl.subscribe({"host": "newbox", "device": "cpu"})[1]   # the REST answer points at the store
    assert sub["status"] == "join" and sub["join"]["port"] > 0 and "--join" in sub["command"], sub
    left = ctl.unsubscribe({"worker_id": sched_id})[1]
    return status, metrics, joined[0].wid, left


def test_worker_joins_running_service_and_leaves():
    status, metrics, wid, left = _launch(2, _drive_join, extra=[_joiner])
    assert status["job_status"] == "completed" and len(status["job_result"]["results"]) == 24
    workers = {m["worker_id"] for m in metrics}
    assert f"rank{wid}" in workers, workers        # the joiner really ran slices
    assert left["left"] is True
