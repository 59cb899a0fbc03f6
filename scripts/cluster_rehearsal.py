"""Rehearse the cluster runner at the target world size on CPU (gloo): N ranks, two
sessions, three datasets, concurrent RandomForest / LogisticRegression / GradientBoosting
searches, optionally one rank killed mid-run -- the reference's 4-worker compose topology
(aws-prod/docker-compose.yml:133-199, ingress routed by
aws-prod/scheduler/scheduler_service.py:249-293) at the 8 GPUs of one MI355X node.

    python scripts/cluster_rehearsal.py --world 8 [--kill 5] [--json out.json]

Prints one JSON line: per-job status, wall time, the dispatcher's control-plane load
(store operations per second issued by rank 0, dispatcher loop turns) and the answer ->
next-slice dispatch latency percentiles.  ``tests/test_cluster_8rank.py`` runs it."""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(dataset, target, model, grid, cv=3, base=None):
    return {"dataset_id": dataset, "train_params": {"test_size": 0.25, "random_state": 0, "target_column": target},
            "model_details": {"model_type": model, "search_type": "GridSearchCV",
                              "hyperparameters": {"base_estimator_params": base or {},
                                                  "search_params": {"param_grid": grid}, "cv_params": {"cv": cv}}}}


DATASETS = [("iris", "species"), ("wine", "target"), ("breast_cancer", "target")]
# the heavy rehearsal's extra table: a 4.8 MB float32 broadcast to every rank, slices of seconds
HEAVY = ("synth", "target", "classification?n=62500&d=20&informative=8&noise=1.0&seed=4&gen=blocks")


def _datasets(heavy: bool):
    return DATASETS + ([HEAVY[:2]] if heavy else [])


def _register(ctl, sid, heavy: bool):
    for name, _t in DATASETS:
        st, _ = ctl.download_data(sid, {"dataset_url": name, "dataset_name": name, "dataset_type": "sklearn"})
        assert st == 200, name
    if heavy:
        st, _ = ctl.download_data(sid, {"dataset_url": HEAVY[2], "dataset_name": HEAVY[0], "dataset_type": "synthetic"})
        assert st == 200, HEAVY


def _jobs(heavy: bool = False):
    """(session, dataset, body) of the rehearsal: 2 sessions x 3 datasets, mixed families
    (+ the heavy table's RandomForest and LogisticRegression searches)."""
    rf = {"max_depth": [2, 4, None], "min_samples_leaf": [1, 3]}
    lr = {"C": [0.1, 1.0, 10.0], "solver": ["lbfgs", "liblinear"]}
    gb = {"n_estimators": [10, 20], "max_depth": [2, 3]}
    out = []
    for s in (0, 1):
        for d, (name, tgt) in enumerate(DATASETS):
            model, grid, base = [("RandomForestClassifier", rf, {"n_estimators": 12, "random_state": 3}),
                                 ("LogisticRegression", lr, {"max_iter": 300}),
                                 ("GradientBoostingClassifier", gb, {"random_state": 5})][(s + d) % 3]
            out.append((s, name, _job(name, tgt, model, grid, base=base)))
    if heavy:
        out.append((0, HEAVY[0], _job(HEAVY[0], HEAVY[1], "RandomForestClassifier",
                                      {"max_depth": [8, None], "min_samples_leaf": [1, 4]},
                                      base={"n_estimators": 16, "random_state": 1})))
        out.append((1, HEAVY[0], _job(HEAVY[0], HEAVY[1], "LogisticRegression", {"C": [0.1, 1.0]},
                                      base={"max_iter": 200})))
    return out


# BASELINE config 5's queue shape (scripts/bench_configs.py config5: 4 sessions x (RF grid of 4
# candidates + LR RandomizedSearchCV of 16) at cv=5, submitted together) on a CPU-sized table
C5_TABLE = ("mixed", "target", "classification?n=20000&d=20&informative=5&noise=1.0&seed=0")


def _config5_jobs():
    out = []
    for s in range(4):
        out.append((s, C5_TABLE[0], {"dataset_id": C5_TABLE[0], "train_params": {"target_column": "target"},
                                     "model_details": {"model_type": "RandomForestClassifier",
                                                       "search_type": "GridSearchCV", "hyperparameters": {
                                                           "base_estimator_params": {}, "cv_params": {"cv": 5},
                                                           "search_params": {"param_grid": {
                                                               "n_estimators": [10, 20], "max_depth": [6, None]}}}}}))
        out.append((s, C5_TABLE[0], {"dataset_id": C5_TABLE[0], "train_params": {"target_column": "target"},
                                     "model_details": {"model_type": "LogisticRegression",
                                                       "search_type": "RandomizedSearchCV", "hyperparameters": {
                                                           "base_estimator_params": {}, "cv_params": {"cv": 5},
                                                           "search_params": {"param_distributions": {
                                                               "C": {"dist": "loguniform", "a": 1e-3, "b": 1e2}},
                                                               "n_iter": 16, "random_state": s}}}}))
    return out


def _poll_gateway(port, targets, stop, lat):
    """Poll GET /check_status of the running jobs through the HTTP gateway (what a client's
    progress bar does) until ``stop``; record each request's latency."""
    import requests

    sess = requests.Session()
    i = 0
    while not stop.is_set() and targets:
        sid, jid = targets[i % len(targets)]
        i += 1
        t0 = time.perf_counter()
        try:
            sess.get(f"http://127.0.0.1:{port}/check_status/{sid}/{jid}", timeout=30)
            lat.append(time.perf_counter() - t0)
        except Exception:
            pass
        time.sleep(0.005)


def _rank_main(rank, world, port, root, kill, outq, heavy=False, env_extra=None, queue="mixed"):
    env = dict(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_RANK=str(rank), OMP_NUM_THREADS="1", DML_DEAD_AFTER_S="3")
    if kill is not None:
        env["DML_KILL_RANK_AFTER"] = f"{kill}:1"     # rank `kill` dies holding its 2nd slice
    env.update(env_extra or {})
    os.environ.update(env)
    import threading

    from cs230_distributed_machine_learning_amd.config import Config
    from cs230_distributed_machine_learning_amd.parallel import dist
    from cs230_distributed_machine_learning_amd.parallel.runner import DistributedRunner, WorkerCore, worker_loop

    inf = dist.init(want_gpu=False, timeout_s=120)
    core = WorkerCore(inf.device)
    if rank != 0:
        worker_loop(core)
        os._exit(0)
    from cs230_distributed_machine_learning_amd.engine.service import Controller

    cfg = Config.from_env(data_root=root, device="cpu", chunk_target_s=0.0)
    runner = DistributedRunner(core)
    ctl = Controller(cfg, runner=runner)

    gw_lat: list = []
    gw_targets: list = []
    gw_stop = threading.Event()

    def drive():
        try:
            if queue == "config5":
                sids = [ctl.create_session()[1]["session_id"] for _ in range(4)]
                st, _ = ctl.download_data(sids[0], {"dataset_url": C5_TABLE[2], "dataset_name": C5_TABLE[0],
                                                    "dataset_type": "synthetic"})
                assert st == 200
                jobs_in = _config5_jobs()
                from cs230_distributed_machine_learning_amd.gateway.app import serve

                gw_port = _free_port()
                serve(ctl, port=gw_port, block=False)
                time.sleep(1.0)
            else:
                sids = [ctl.create_session()[1]["session_id"] for _ in range(2)]
                _register(ctl, sids[0], heavy)
                jobs_in = _jobs(heavy)
            t0 = time.time()
            ops0 = runner.store_ops()
            acks = []
            for s, name, body in jobs_in:   # every job submitted at once: concurrent searches
                st, ack = ctl.train(sids[s], body)
                assert st in (200, 202), ack
                acks.append((s, name, body["model_details"]["model_type"], ack["job_id"]))
            poller = None
            if queue == "config5":
                gw_targets.extend((sids[s], jid) for s, _n, _m, jid in acks)
                poller = threading.Thread(target=_poll_gateway, args=(gw_port, gw_targets, gw_stop, gw_lat),
                                          daemon=True)
                poller.start()
            jobs = []
            for s, name, model, jid in acks:
                ctl.table.wait_finished(jid, timeout=600)
                status = ctl.check_status(sids[s], jid)[1]
                res = (status.get("job_result") or {}).get("results") or []
                jobs.append({"session": s, "dataset": name, "model": model, "status": status["job_status"],
                             "n_results": len(res), "total": status.get("total_subtasks"),
                             "scores_via": sorted({str(r.get("scores_via")) for r in res}),
                             "best": (status.get("best_result") or {}).get("mean_cv_score"),
                             "scores": sorted((json.dumps(r.get("parameters"), sort_keys=True), r.get("cv_scores"))
                                              for r in res)})
            wall = time.time() - t0
            gw_stop.set()
            if poller is not None:
                poller.join(timeout=10)
            lat = sorted(runner.stats["dispatch_latency_s"])
            pct = lambda q: round(lat[min(len(lat) - 1, int(q * len(lat)))] * 1e3, 2) if lat else None
            al = sorted(runner.stats.get("answer_lag_s", []))
            apct = lambda q: round(al[min(len(al) - 1, int(q * len(al)))] * 1e3, 2) if al else None
            gl = sorted(gw_lat)
            gpct = lambda q: round(gl[min(len(gl) - 1, int(q * len(gl)))] * 1e3, 2) if gl else None
            ops = runner.store_ops() - ops0
            outq.put(("ok", {"world": world, "killed": kill, "dead": sorted(runner.dead), "wall_s": round(wall, 2),
                             "jobs": jobs, "dispatcher_loops": runner.stats["loops"],
                             "answers": runner.stats["answers"], "rank0_store_ops": ops,
                             "max_drain_wait_s": round(runner.stats["max_drain_wait_s"], 3),
                             "rank0_store_ops_per_s": round(ops / max(wall, 1e-9), 1),
                             "dispatch_latency_ms": {"p50": pct(0.5), "p90": pct(0.9), "p99": pct(0.99),
                                                     "max": pct(1.0), "n": len(lat)},
                             "answer_lag_ms": {"p50": apct(0.5), "p90": apct(0.9), "p99": apct(0.99),
                                               "max": apct(1.0), "n": len(al)},
                             "queue": queue,
                             "gateway_check_status_ms": {"p50": gpct(0.5), "p90": gpct(0.9), "p99": gpct(0.99),
                                                         "max": gpct(1.0), "n": len(gl)} if gl else None}))
        except Exception:  # pragma: no cover
            import traceback

            outq.put(("err", traceback.format_exc()))
        finally:
            runner.shutdown()

    t = threading.Thread(target=drive, daemon=True)
    t.start()
    runner.serve_forever()
    t.join()
    time.sleep(1.0)   # let the workers read their stop keys before the store host exits
    os._exit(0)       # a peer may be dead: skip the collective teardown


def local_scores(body_jobs=None, heavy: bool = False) -> list:
    """The same jobs through the one-process LocalRunner (per-candidate CV scores)."""
    from cs230_distributed_machine_learning_amd.config import Config
    from cs230_distributed_machine_learning_amd.engine.service import Controller

    ctl = Controller(Config(data_root=tempfile.mkdtemp(prefix="dml_local_"), device="cpu", chunk_target_s=0.0))
    sid = ctl.create_session()[1]["session_id"]
    _register(ctl, sid, heavy)
    out = []
    for s, name, body in (body_jobs or _jobs(heavy)):
        st, ack = ctl.train(sid, body)
        ctl.table.wait_finished(ack["job_id"], timeout=600)
        res = (ctl.check_status(sid, ack["job_id"])[1].get("job_result") or {}).get("results") or []
        out.append(sorted((json.dumps(r.get("parameters"), sort_keys=True), r.get("cv_scores")) for r in res))
    ctl.shutdown() if hasattr(ctl, "shutdown") else None
    return out


def run(world: int = 8, kill=None, timeout_s: float = 900.0, heavy: bool = False, env_extra=None,
        queue: str = "mixed") -> dict:
    import torch.multiprocessing as mp

    root = tempfile.mkdtemp(prefix="dml_rehearsal_")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, root, kill, q, heavy, env_extra, queue))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = q.get(timeout=timeout_s)
    finally:
        deadline = time.time() + 60
        for p in procs:
            p.join(timeout=max(1, deadline - time.time()))
            if p.is_alive():
                p.kill()
    if out[0] != "ok":
        raise RuntimeError(out[1])
    res = out[1]
    res["exitcodes"] = [p.exitcode for p in procs]
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--kill", type=int, default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--heavy", action="store_true", help="add the 62.5k x 20 table's RF / LR searches")
    ap.add_argument("--queue", choices=("mixed", "config5"), default="mixed",
                    help="config5: BASELINE config 5's queue shape, /check_status polled through the gateway")
    args = ap.parse_args()
    r = run(args.world, args.kill, heavy=args.heavy, queue=args.queue)
    line = json.dumps(r)
    print(line)
    if args.json:
        with open(args.json, "w") as f:
            f.write(line + "\n")
