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

import numpy as np
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
    while not any(w.joined and w.alive for w in runner.workers.values()):
        if time.time() - t0 > 60:
            raise RuntimeError("joiner never arrived")
        time.sleep(0.1)
    grid = {"min_samples_leaf": list(range(1, 25))}
    st, a = ctl.train(sid, _grid_job("job-j", "mid", "RandomForestClassifier", grid, base={"n_estimators": 20}))
    ctl.table.wait_finished(a["job_id"], timeout=240)
    status = ctl.check_status(sid, a["job_id"])[1]
    metrics = ctl.metrics(sid, a["job_id"])[1]
    joined = [w for w in runner.workers.values() if w.joined]
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


# ---- RCCL failure safety and collective ordering (run here on gloo) ---------------
def _serve_rc(rank, world, port, root, outq, drive_fn, env):
    """_serve, but rank 0 reports its own exit status through the queue."""
    _serve(rank, world, port, root, outq, drive_fn, env)


def _launch_faulty(world, drive_fn, env, timeout=240):
    """Like _launch, for runs where a rank hangs (SIGSTOP): the caller gets rank 0's result
    and exit code; every other process is killed afterwards."""
    root = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve, args=(r, world, port, root, q, drive_fn, env)) for r in range(world)]
    for p in procs:
        p.start()
    t0 = time.time()
    try:
        out = q.get(timeout=timeout)
        procs[0].join(timeout=60)
        rc0, wall = procs[0].exitcode, time.time() - t0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert out[0] == "ok", out[1]
    return out[1], rc0, wall


def _drive_two_jobs(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "classification?n=3000&d=8&seed=11", "dataset_name": "t",
                            "dataset_type": "synthetic"})
    grid = {"min_samples_leaf": [1, 2, 4, 8]}
    t0 = time.time()
    st, a = ctl.train(sid, _grid_job("job-1", "t", "RandomForestClassifier", grid, base={"n_estimators": 8}))
    assert st in (200, 202), a
    ctl.table.wait_finished(a["job_id"], timeout=180)
    t1 = time.time() - t0
    s1 = ctl.check_status(sid, a["job_id"])[1]
    st, b = ctl.train(sid, _grid_job("job-2", "t", "RandomForestClassifier", {"max_depth": [2, 4]},
                                     base={"n_estimators": 8}))
    ctl.table.wait_finished(b["job_id"], timeout=180)
    s2 = ctl.check_status(sid, b["job_id"])[1]
    vias = [r.get("scores_via") for r in s1["job_result"]["results"]]
    return {"s1": s1, "s2": s2, "t1": t1, "broken": runner.group_broken, "vias": vias,
            "dead": sorted(runner.dead), "pending": len(runner.coll_pending)}


def test_hung_rank_in_scores_gather_rank0_survives():
    """A rank hangs (SIGSTOP, sockets stay open) inside a job's scores all-gather: rank 0's
    side collective times out (DML_SIDE_TIMEOUT_S) and RAISES instead of tearing the process
    down; the dispatcher marks the group broken, the job completes from the store copies, the
    next job runs host-staged, and rank 0 exits 0."""
    env = {"DML_STOP_RANK_IN": "2:scores", "DML_SIDE_TIMEOUT_S": "6", "DML_DEAD_AFTER_S": "600", "DML_REGROUP": "0"}
    r, rc0, wall = _launch_faulty(3, _drive_two_jobs, env)
    assert r["s1"]["job_status"] == "completed" and len(r["s1"]["job_result"]["results"]) == 4
    assert r["s2"]["job_status"] == "completed" and len(r["s2"]["job_result"]["results"]) == 2
    assert r["broken"] and r["dead"] == [] and r["pending"] == 0, r   # hung, not declared dead
    assert all(v in (None, "store-fallback") for v in r["vias"]), r["vias"]
    assert r["t1"] < 6 + 30 + 60, r["t1"]     # within the side timeout (+ deadline grace + fit time)
    assert rc0 == 0, rc0


def test_failed_collective_breaks_group_next_job_completes():
    """One rank's collective task raises before the gather (an OOM while its peers are already
    inside): the group is marked broken at once, pending scores fall back to the store copies,
    and the next job still completes (host-staged)."""
    env = {"DML_FAIL_RANK_IN": "1:scores", "DML_SIDE_TIMEOUT_S": "6", "DML_REGROUP": "0"}
    r, rc0, _ = _launch_faulty(3, _drive_two_jobs, env)
    assert r["s1"]["job_status"] == "completed" and r["s2"]["job_status"] == "completed"
    assert r["broken"] and r["pending"] == 0, r
    assert rc0 == 0, rc0


def _drive_dp_during_broadcast(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "classification?n=4000&d=8&seed=12", "dataset_name": "a",
                            "dataset_type": "synthetic"})
    ctl.download_data(sid, {"dataset_url": "classification?n=4000&d=8&seed=13", "dataset_name": "b",
                            "dataset_type": "synthetic"})
    # job A needs a broadcast of table "a" (slow: DML_COLL_DELAY_S); the data-parallel job B is
    # submitted while it is in flight
    st, a = ctl.train(sid, _grid_job("job-a", "a", "RandomForestClassifier", {"max_depth": [2, 3]},
                                     base={"n_estimators": 4}))
    t0 = time.time()
    while not runner.coll_pending and time.time() - t0 < 30:
        time.sleep(0.02)
    in_flight = bool(runner.coll_pending)
    body = _grid_job("job-b", "b", "LogisticRegression", {"C": [0.5, 1.0]})
    body["train_params"]["parallelism"] = "data"
    st, b = ctl.train(sid, body)
    assert st in (200, 202), b
    ctl.table.wait_finished(a["job_id"], timeout=180)
    ctl.table.wait_finished(b["job_id"], timeout=180)
    return {"in_flight": in_flight, "a": ctl.check_status(sid, a["job_id"])[1]["job_status"],
            "b": ctl.check_status(sid, b["job_id"])[1]["job_status"], "iv": list(runner.core.intervals)}


def test_dp_epoch_never_overlaps_side_collectives():
    """A data-parallel job (default-group collectives, worker thread) submitted while a
    side-group broadcast is in flight starts only after it, and no side task is posted while
    the epoch holds the group: on every rank the two communicators never have operations in
    flight together (RCCL may deadlock on unordered use of two communicators)."""
    r = _launch(2, _drive_dp_during_broadcast, env={"DML_COLL_DELAY_S": "1.5"})
    assert r["in_flight"] and r["a"] == "completed" and r["b"] == "completed", r
    iv = r["iv"]
    dp = [(s, e) for k, s, e in iv if k == "dp"]
    side = [(s, e) for k, s, e in iv if k.startswith("side:")]
    assert dp and side, iv
    for s0, e0 in dp:
        for s1, e1 in side:
            assert e1 <= s0 or e0 <= s1, (iv,)


def test_score_rows_carry_every_fold():
    """cv > 60 folds: the scores epoch's rows are sized from the job's cv, so J5 keeps every
    fold score (a fixed 64-column row cut them to 60)."""
    from cs230_distributed_machine_learning_amd.parallel.runner import SCORE_HEAD, score_row, score_width

    w = score_width({"cv": 80})
    assert w == SCORE_HEAD + 80
    row = score_row(True, {"cv_scores": [i / 100 for i in range(80)], "mean_cv_score": 0.4,
                           "std_cv_score": 0.1}, w)
    assert int(row[3]) == 80 and row[SCORE_HEAD + 79] == 0.79


def _drive_cv80(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "classification?n=800&d=5&seed=14", "dataset_name": "s",
                            "dataset_type": "synthetic"})
    st, a = ctl.train(sid, _grid_job("job-cv", "s", "LogisticRegression", {"C": [0.5, 2.0]}, cv=80))
    ctl.table.wait_finished(a["job_id"], timeout=180)
    s = ctl.check_status(sid, a["job_id"])[1]
    return [(len(r["cv_scores"]), r.get("scores_via")) for r in s["job_result"]["results"]]


def test_cv80_job_through_scores_epoch():
    out = _launch(2, _drive_cv80)
    assert out == [(80, "gloo"), (80, "gloo")], out


def _mae_mono_job(parallelism):
    body = _grid_job("job-mae", "r", "RandomForestRegressor",
                     {"criterion": ["absolute_error", "squared_error"], "max_depth": [3]},
                     base={"n_estimators": 4, "random_state": 0, "monotonic_cst": [1, 0, 0, 0, 0, -1]})
    body["train_params"]["parallelism"] = parallelism
    return body


def _drive_mae_dp(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "regression?n=1500&d=6&seed=21", "dataset_name": "r",
                            "dataset_type": "synthetic"})
    st, a = ctl.train(sid, _mae_mono_job("data"))
    assert st in (200, 202), a
    ctl.table.wait_finished(a["job_id"], timeout=180)
    s = ctl.check_status(sid, a["job_id"])[1]
    return {r["parameters"]["criterion"]: r["cv_scores"] for r in s["job_result"]["results"]}


def test_row_shard_request_keeps_absolute_error_and_monotonic_cst():
    """parallelism='data' on a job whose candidates need every row on one rank (absolute_error
    medians, monotonic_cst node bounds): the cluster runs it task-parallel and returns the
    local runner's CV scores -- never a silently different estimator."""
    dist_scores = _launch(3, _drive_mae_dp)
    root = tempfile.mkdtemp()
    ctl = Controller(Config.from_env(data_root=root, device="cpu", chunk_target_s=0.0))
    try:
        sid = ctl.create_session()[1]["session_id"]
        ctl.download_data(sid, {"dataset_url": "regression?n=1500&d=6&seed=21", "dataset_name": "r",
                                "dataset_type": "synthetic"})
        st, a = ctl.train(sid, _mae_mono_job("task"))
        ctl.table.wait_finished(a["job_id"], timeout=180)
        s = ctl.check_status(sid, a["job_id"])[1]
        local = {r["parameters"]["criterion"]: r["cv_scores"] for r in s["job_result"]["results"]}
    finally:
        ctl.shutdown()
    assert set(dist_scores) == {"absolute_error", "squared_error"}
    for k in local:
        assert np.allclose(dist_scores[k], local[k], rtol=0, atol=1e-12), (k, dist_scores[k], local[k])


# ---- a rank dies or hangs inside a row-sharded (data-parallel) epoch -------------------------
def _dp_lr_job(parallelism):
    body = _grid_job("job-dp", "dpt", "LogisticRegression", {"C": [0.1, 1.0, 10.0]})
    body["train_params"]["parallelism"] = parallelism
    return body


def _drive_dp_hang(ctl, runner):
    sid = ctl.create_session()[1]["session_id"]
    ctl.download_data(sid, {"dataset_url": "classification?n=3000&d=8&seed=31", "dataset_name": "dpt",
                            "dataset_type": "synthetic"})
    t0 = time.time()
    st, a = ctl.train(sid, _dp_lr_job("data"))
    assert st in (200, 202), a
    ctl.table.wait_finished(a["job_id"], timeout=200)
    t1 = time.time() - t0
    s = ctl.check_status(sid, a["job_id"])[1]
    # the service keeps serving: a second job on the same table completes too
    st, b = ctl.train(sid, _grid_job("job-next", "dpt", "LogisticRegression", {"C": [2.0]}))
    ctl.table.wait_finished(b["job_id"], timeout=120)
    s2 = ctl.check_status(sid, b["job_id"])[1]
    return {"status": s["job_status"], "t1": t1, "requeued": runner.stats.get("dp_requeued", 0),
            "broken": runner.group_broken, "next": s2["job_status"],
            "scores": {r["parameters"]["C"]: r["cv_scores"] for r in s["job_result"]["results"]}}


def _local_dp_lr_scores():
    root = tempfile.mkdtemp()
    ctl = Controller(Config.from_env(data_root=root, device="cpu", chunk_target_s=0.0))
    try:
        sid = ctl.create_session()[1]["session_id"]
        ctl.download_data(sid, {"dataset_url": "classification?n=3000&d=8&seed=31", "dataset_name": "dpt",
                                "dataset_type": "synthetic"})
        st, a = ctl.train(sid, _dp_lr_job("task"))
        ctl.table.wait_finished(a["job_id"], timeout=180)
        s = ctl.check_status(sid, a["job_id"])[1]
        return {r["parameters"]["C"]: r["cv_scores"] for r in s["job_result"]["results"]}
    finally:
        ctl.shutdown()


@pytest.mark.parametrize("fault", ["stop", "fail"])
def test_rank_lost_inside_data_parallel_epoch_job_reruns_task_parallel(fault):
    """A rank hangs (SIGSTOP) or raises inside a row-sharded LogisticRegression epoch: the
    survivors' data-parallel collectives time out after DML_DP_TIMEOUT_S (their own
    communicator, not the default group's 30 min), rank 0 abandons the epoch, breaks the group
    and re-runs the job TASK-parallel on the survivors (reference re-places a dead worker's
    tasks, aws-prod/scheduler/scheduler_service.py:205-247).  The job completes with the local
    runner's CV scores, the next job completes, and rank 0 exits 0."""
    var = "DML_STOP_RANK_IN" if fault == "stop" else "DML_FAIL_RANK_IN"
    env = {var: "2:dp", "DML_DP_TIMEOUT_S": "8", "DML_SIDE_TIMEOUT_S": "8", "DML_DEAD_AFTER_S": "600",
           "DML_REGROUP": "0"}
    r, rc0, wall = _launch_faulty(3, _drive_dp_hang, env)
    assert r["status"] == "completed" and r["next"] == "completed", r
    assert r["requeued"] == 1 and r["broken"], r
    assert r["t1"] < 8 + 60, r["t1"]          # the epoch timeout plus re-run time, not 30 minutes
    local = _local_dp_lr_scores()
    assert set(r["scores"]) == set(local)
    for k in local:
        assert np.allclose(r["scores"][k], local[k], rtol=0, atol=1e-12), (k, r["scores"][k], local[k])
    assert rc0 == 0, rc0
