"""The real launcher (``python -m ...serve --gpus 2``) keeps serving after a worker rank dies.

serve.py's parent process starts one child per rank and supervises them itself (no
torchrun elastic agent, which would tear rank 0 -- controller + gateway -- down with the
failed worker).  Rank 1 hard-exits mid-job (DML_KILL_RANK_AFTER); the job still completes
on rank 0 (dead-rank detection + re-queue, parallel/runner.py), the gateway keeps
answering, and a job on a NEW dataset completes on the survivor.  gloo on CPU."""
import os
import socket
import subprocess
import sys
import time

import pytest

httpx = pytest.importorskip("httpx")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job(dataset, target, grid):
    return {"dataset_id": dataset, "train_params": {"target_column": target, "test_size": 0.25, "random_state": 0},
            "model_details": {"model_type": "RandomForestClassifier", "search_type": "GridSearchCV",
                              "hyperparameters": {"base_estimator_params": {"n_estimators": 8},
                                                  "search_params": {"param_grid": grid}, "cv_params": {"cv": 3}}}}


def _wait_done(c, sid, jid, timeout):
    t0 = time.time()
    while time.time() - t0 < timeout:
        st = c.get(f"/check_status/{sid}/{jid}").json()
        if st.get("job_status") in ("completed", "failed"):
            return st
        time.sleep(0.5)
    raise AssertionError(f"job {jid} not finished after {timeout}s: {st}")


@pytest.mark.timeout(400)
def test_worker_rank_death_under_real_launcher(tmp_path):
    port, mport = _free_port(), _free_port()
    env = dict(os.environ, DML_KILL_RANK_AFTER="1:0", OMP_NUM_THREADS="2", PYTHONUNBUFFERED="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    log = open(tmp_path / "serve.log", "w")
    proc = subprocess.Popen([sys.executable, "-m", "cs230_distributed_machine_learning_amd.serve", "--gpus", "2",
                             "--device", "cpu", "--port", str(port), "--master-port", str(mport),
                             "--data-root", str(tmp_path / "data"), "--chunk-target-s", "0"],
                            env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        c = httpx.Client(base_url=f"http://127.0.0.1:{port}", timeout=30)
        t0 = time.time()
        while True:
            try:
                if c.get("/health").status_code == 200:
                    break
            except httpx.HTTPError:
                pass
            assert proc.poll() is None, (tmp_path / "serve.log").read_text()
            assert time.time() - t0 < 180, "service did not come up"
            time.sleep(0.5)
        sid = c.post("/create_session").json()["session_id"]
        r = c.post(f"/download_data/{sid}", json={"dataset_url": "iris", "dataset_name": "iris",
                                                  "dataset_type": "sklearn"})
        assert r.status_code == 200, r.text
        jid = c.post(f"/train/{sid}", json=_job("iris", "species", {"max_depth": [2, 3, 4, 5, 6, None],
                                                                     "min_samples_leaf": [1, 2, 3, 4]})).json()["job_id"]
        st = _wait_done(c, sid, jid, 200)
        assert st["job_status"] == "completed" and len(st["job_result"]["results"]) == 24, st
        text = (tmp_path / "serve.log").read_text()
        assert "worker on GPU 1 exited" in text, text[-3000:]   # the worker really died ...
        assert proc.poll() is None                            # ... and the service did not
        # a new dataset after the death: served by the survivor
        r = c.post(f"/download_data/{sid}", json={"dataset_url": "classification?n=3000&d=8&seed=2",
                                                  "dataset_name": "synth2", "dataset_type": "synthetic"})
        assert r.status_code == 200, r.text
        t1 = time.time()
        jid2 = c.post(f"/train/{sid}", json=_job("synth2", "target", {"max_depth": [3, None]})).json()["job_id"]
        st2 = _wait_done(c, sid, jid2, 60)
        assert st2["job_status"] == "completed" and time.time() - t1 < 60, st2
        assert c.get("/health").status_code == 200
    finally:
        try:
            os.killpg(proc.pid, 15)
        except ProcessLookupError:
            pass
        try:
            proc.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)
        log.close()
