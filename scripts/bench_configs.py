#!/usr/bin/env python3
"""The five BASELINE.json configurations, one JSON line each (single process / 1 device).

  1  LogisticRegression GridSearchCV cv=5 on iris through the client API (plumbing, CPU)
  2  RandomForestClassifier 64-point grid, 1M x 100 synthetic, 1 GPU
  3  the headline 256-point RF GridSearchCV is ``bench.py`` (1/2/4/8 GPUs)
  4  RandomizedSearchCV LogisticRegression n_iter=512 cv=5 on --lr-rows x 1000 dense
  5  mixed queue: concurrent RF + LR jobs from several sessions through the controller
  6  GradientBoostingClassifier GridSearchCV n_estimators {100, 200} x max_depth {3, 5},
     cv=5, 1M x 100 synthetic, 1 GPU (every fit of the grid boosted in one stage loop), timed
     after an untimed warmup fit (DML_C6_WARMUP=0: the cold first job); --gb-loss / --gb-depths /
     --gb-estimators / --random-state give its variants

  configs 2 and 6 take --random-state N (a fixed random_state in the grid: exact n_estimators /
  max_depth prefix sharing, models/base.py prefix_groups); config 2 --whole runs its grid as one call

    python scripts/bench_configs.py --configs 1,2,4,5 [--lr-rows 10000000]

Metric everywhere: CV fits per second of wall time (a candidate x fold fit counts 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _emit(cfg, fits, seconds, **extra):
    print(json.dumps({"config": cfg, "cv_fits": fits, "seconds": round(seconds, 3),
                      "cv_fits_per_s": round(fits / seconds, 4), **extra}), flush=True)


def config1():
    from sklearn.linear_model import LogisticRegression
    from sklearn.model_selection import GridSearchCV

    from cs230_distributed_machine_learning_amd.config import Config
    from cs230_distributed_machine_learning_amd.engine.service import Controller
    from distributed_ml import MLTaskManager

    ctl = Controller(Config(data_root=tempfile.mkdtemp(), device="cpu"))
    tm = MLTaskManager(controller=ctl)
    tm.download_data("iris", "iris", "sklearn")
    grid = {"C": [0.1, 1.0, 10.0, 100], "solver": ["liblinear", "lbfgs"]}
    t0 = time.time()
    out = tm.train(GridSearchCV(LogisticRegression(), grid, cv=5), "iris", {"target_column": "target"},
                   wait_for_completion=True, polling_interval=0.02)
    dt = time.time() - t0
    best = out["best_result"]
    _emit(1, 8 * 6, dt, best={k: best["parameters"][k] for k in ("C", "solver")},
          best_mean_cv=round(best["mean_cv_score"], 4), note="48 fits = 8 candidates x (5 CV + 1 holdout)")
    ctl.shutdown()


def _synthetic(rows, d, dev, seed=0):
    from cs230_distributed_machine_learning_amd.data import synthetic
    from cs230_distributed_machine_learning_amd.data.device import DeviceData

    X, y = synthetic.make_table(rows, d, informative=10, n_classes=2, noise=1.0, seed=seed, device=dev)
    return DeviceData(X, y, classification=True, device=dev, name=f"synthetic-{rows}x{d}")


def config2(dev, random_state=None, whole=False):
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
    from cs230_distributed_machine_learning_amd.search.grid import expand_candidates

    dd = _synthetic(1_000_000, 100, dev)
    grid = {"n_estimators": [50, 100, 150, 200], "max_depth": [10, 20, 30, None], "min_samples_leaf": [1, 2, 4, 8]}
    if random_state is not None:   # fixed seeds: exact n_estimators prefix sharing (models/base.py)
        grid["random_state"] = [random_state]
    cands = expand_candidates("GridSearchCV", {"param_grid": grid})
    spec = JobSpec("RandomForestClassifier", cands, cv=5, holdout=False, keep_models="none")
    dd.binned()
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    t0 = time.time()
    done = 0
    step = len(cands) if whole else 4   # 4 candidates (20 fits) per device batch, or the whole grid
    for i in range(0, len(cands), step):
        res = run_candidates(dd, spec, list(range(i, min(i + step, len(cands)))))
        assert all(r.ok for r in res)
        done += 5 * len(res)
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    _emit(2, done, time.time() - t0, grid_points=len(cands), random_state=random_state, whole_grid_call=whole,
          prefix_share=os.environ.get("DML_PREFIX_SHARE", "1") != "0")


def config4(dev, rows):
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
    from cs230_distributed_machine_learning_amd.search.grid import expand_candidates

    dd = _synthetic(rows, 1000, dev, seed=1)
    dist = {"C": {"dist": "loguniform", "a": 1e-3, "b": 1e2}, "solver": ["lbfgs", "liblinear"],
            "max_iter": [100]}
    cands = expand_candidates("RandomizedSearchCV", {"param_distributions": dist, "n_iter": 512, "random_state": 0})
    spec = JobSpec("LogisticRegression", cands, cv=5, holdout=False, keep_models="none")
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    t0 = time.time()
    res = run_candidates(dd, spec, list(range(len(cands))))
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    ok = [r for r in res if r.ok]
    _emit(4, 5 * len(ok), time.time() - t0, rows=rows, features=1000, candidates=len(cands),
          best_mean_cv=round(max(r.result["mean_cv_score"] for r in ok), 4))


def _config5_data(root):
    import pandas as pd

    rng = np.random.RandomState(0)
    n, d = 200_000, 20
    X = rng.randn(n, d).astype(np.float32)
    y = (X[:, :5].sum(1) + rng.randn(n) > 0).astype(int)
    df = pd.DataFrame(X, columns=[f"f{i}" for i in range(d)])
    df["label"] = y
    os.makedirs(os.path.join(root, "datasets", "mixed"), exist_ok=True)
    df.to_csv(os.path.join(root, "datasets", "mixed", "mixed.csv"), index=False)


def _config5_drive(ctl, runner_name):
    # untimed warm-up job: the dataset's first load (parse, placement; on the cluster runner
    # also the side communicator's first collective) is a once-per-service cost, reported
    # separately as load_s, so both runners are timed on the same steady-state queue
    t_w = time.time()
    sid0 = ctl.create_session()[1]["session_id"]
    st, _ = ctl.train(sid0, {"job_id": "warm", "dataset_id": "mixed", "train_params": {"target_column": "label"},
                             "model_details": {"model_type": "RandomForestClassifier", "search_type": "GridSearchCV",
                                               "hyperparameters": {"base_estimator_params": {}, "cv_params": {"cv": 2},
                                                                   "search_params": {"param_grid": {"n_estimators": [2]}}}}})
    assert st == 200
    ctl.table.wait_finished("warm", timeout=3600)
    load_s = time.time() - t_w
    jobs = []
    t0 = time.time()
    for s in range(4):
        sid = ctl.create_session()[1]["session_id"]
        for kind in ("rf", "lr"):
            if kind == "rf":
                md = {"model_type": "RandomForestClassifier", "search_type": "GridSearchCV", "hyperparameters": {
                    "base_estimator_params": {}, "cv_params": {"cv": 5},
                    "search_params": {"param_grid": {"n_estimators": [50, 100], "max_depth": [10, None]}}}}
            else:
                md = {"model_type": "LogisticRegression", "search_type": "RandomizedSearchCV", "hyperparameters": {
                    "base_estimator_params": {}, "cv_params": {"cv": 5}, "search_params": {
                        "param_distributions": {"C": {"dist": "loguniform", "a": 1e-3, "b": 1e2}},
                        "n_iter": 16, "random_state": s}}}
            jid = f"{kind}-{s}"
            st, _ = ctl.train(sid, {"job_id": jid, "dataset_id": "mixed", "model_details": md,
                                    "train_params": {"target_column": "label"}})
            assert st == 200
            jobs.append((sid, jid))
    fits = 0
    workers = set()
    for sid, jid in jobs:
        ctl.table.wait_finished(jid, timeout=3600)
        st = ctl.check_status(sid, jid)[1]
        assert st["job_status"] == "completed", st
        fits += st["total_subtasks"] * 6
        workers |= {m.get("worker_id") for m in ctl.metrics(sid, jid)[1]}
    _emit(5, fits, time.time() - t0, jobs=len(jobs), sessions=4, runner=runner_name, workers=sorted(workers),
          load_s=round(load_s, 3))


def config5(dev):
    """Mixed queue through the controller: the local runner on one process, or -- under
    torchrun / DML_FORCE_PG=1 -- the cluster DistributedRunner (rank 0 dispatches, every
    rank works), the path BASELINE config 5 names for 8 GPUs."""
    from cs230_distributed_machine_learning_amd.config import Config
    from cs230_distributed_machine_learning_amd.engine.service import Controller

    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("DML_FORCE_PG") == "1":
        import threading

        from cs230_distributed_machine_learning_amd.parallel import dist
        from cs230_distributed_machine_learning_amd.parallel.runner import DistributedRunner, WorkerCore, worker_loop

        inf = dist.init(want_gpu=dev.type == "cuda")
        core = WorkerCore(inf.device)
        if inf.rank == 0:
            root = tempfile.mkdtemp()
            _config5_data(root)
            runner = DistributedRunner(core)
            ctl = Controller(Config(data_root=root, device=str(inf.device)), runner=runner)

            def drive():
                try:
                    _config5_drive(ctl, f"distributed x{inf.world}")
                finally:
                    runner.shutdown()

            t = threading.Thread(target=drive, daemon=True)
            t.start()
            runner.serve_forever()
            t.join()
        else:
            worker_loop(core)
        dist.destroy()
        return
    root = tempfile.mkdtemp()
    _config5_data(root)
    ctl = Controller(Config(data_root=root, device=str(dev)))
    _config5_drive(ctl, "local")
    ctl.shutdown()


def config6(dev, loss=None, depths=None, estimators=None, random_state=None):
    """Config 6: GradientBoostingClassifier GridSearchCV (4 points x cv5) on 1M x 100; with
    ``loss`` (e.g. huber): the same grid as a GradientBoostingRegressor of that loss on a
    continuous target of the same table (the percentile-loss stage kernels)."""
    from cs230_distributed_machine_learning_amd.data.device import DeviceData
    from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
    from cs230_distributed_machine_learning_amd.search.grid import expand_candidates
    from cs230_distributed_machine_learning_amd.utils import trace

    dd = _synthetic(1_000_000, 100, dev)
    grid = {"n_estimators": estimators or [100, 200], "max_depth": depths or [3, 5]}
    if random_state is not None:
        grid["random_state"] = [random_state]
    model = "GradientBoostingClassifier"
    if loss:
        g = torch.Generator(device=dev).manual_seed(5)
        yr = dd.X[:, :10].sum(1) + 0.5 * torch.randn(dd.n, device=dev, generator=g)
        dd = DeviceData(dd.X, yr.float(), classification=False, device=dev, name="synthetic-reg-1Mx100")
        grid["loss"] = [loss]
        model = "GradientBoostingRegressor"
    cands = expand_candidates("GridSearchCV", {"param_grid": grid})
    spec = JobSpec(model, cands, cv=5, holdout=False, keep_models="none")
    dd.binned()
    if os.environ.get("DML_C6_WARMUP", "1") != "0":
        # untimed warmup fit (as bench.py's warmup steps): first kernel launches load their code
        # objects, the device arenas and caching allocator reach their sizes
        warm = [dict(c, n_estimators=3) for c in cands if c["n_estimators"] == min(x["n_estimators"] for x in cands)]
        run_candidates(dd, JobSpec(model, warm, cv=5, holdout=False, keep_models="none"), list(range(len(warm))))
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    for rep in range(int(os.environ.get("DML_C6_REPEAT", "1")) - 1):   # study: back-to-back jobs
        t0 = time.time()
        run_candidates(dd, spec, list(range(len(cands))))
        torch.cuda.synchronize(dev) if dev.type == "cuda" else None
        print(f"repeat {rep}: {time.time() - t0:.3f} s", file=sys.stderr, flush=True)
    trace.summary(reset=True)
    t0 = time.time()
    res = run_candidates(dd, spec, list(range(len(cands))))
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    dt = time.time() - t0
    assert all(r.ok for r in res), [r.error for r in res if not r.ok]
    _emit(6, 5 * len(res), dt, grid_points=len(cands), stages_total=5 * sum(int(c["n_estimators"]) for c in cands),
          best_mean_cv=round(max(r.result["mean_cv_score"] for r in res), 4), random_state=random_state,
          prefix_share=os.environ.get("DML_PREFIX_SHARE", "1") != "0", phases=trace.summary())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,4,5")
    ap.add_argument("--lr-rows", type=int, default=2_000_000)
    ap.add_argument("--gpus", type=int, default=1, help="config 5 on N ranks (relaunches under torchrun)")
    ap.add_argument("--gb-loss", default=None, help="config 6 as a GradientBoostingRegressor of this loss")
    ap.add_argument("--gb-depths", default=None, help="config 6 variant: comma-separated max_depth values")
    ap.add_argument("--gb-estimators", default=None, help="config 6 variant: comma-separated n_estimators values")
    ap.add_argument("--whole", action="store_true", help="config 2: the whole grid in one run_candidates call")
    ap.add_argument("--random-state", type=int, default=None,
                    help="configs 2 / 6: a fixed random_state in the grid (exact n_estimators prefix sharing)")
    args = ap.parse_args()
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", "29571", os.path.abspath(__file__),
               "--configs", "5"]
        return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    want = {int(c) for c in args.configs.split(",")}
    if 1 in want:
        config1()
    if 2 in want:
        config2(dev, args.random_state, args.whole)
    if 4 in want:
        config4(dev, args.lr_rows)
    if 5 in want:
        config5(dev)
    if 6 in want:
        ints = lambda v: [int(x) for x in v.split(",")] if v else None
        config6(dev, args.gb_loss, ints(args.gb_depths), ints(args.gb_estimators), args.random_state)


if __name__ == "__main__":
    sys.exit(main())
