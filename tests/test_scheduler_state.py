"""The scheduler's learned calibration survives a restart (reference: the runtime
predictor is saved after each refit and reloaded at start,
aws-prod/scheduler/scheduler_service.py:44-46,82)."""
import json
import os

import pytest

from cs230_distributed_machine_learning_amd.config import Config
from cs230_distributed_machine_learning_amd.engine.scheduler import Scheduler, Unit
from cs230_distributed_machine_learning_amd.engine.service import Controller, job_plan, plan_slices, \
    scheduler_state_path

pytest.importorskip("sklearn")

from test_service import _j1, _wait  # noqa: E402


def test_state_roundtrip(tmp_path):
    p = str(tmp_path / "s.json")
    s = Scheduler(state_path=p)
    wid = s.register(host="h", device="cuda:3")
    s.place([Unit("u1", cost=10.0, algo="RandomForestClassifier")])
    s.observe(wid, Unit("u1", cost=10.0, algo="RandomForestClassifier"), 2.0)
    s.place([Unit("u2", cost=5.0, algo="randomforestclassifier")])
    s.observe(wid, Unit("u2", cost=5.0, algo="randomforestclassifier"), 0.5)
    assert os.path.exists(p)
    s2 = Scheduler(state_path=p)
    assert s2.calib == pytest.approx(s.calib)
    assert s2._calib_sums == pytest.approx(s._calib_sums)
    # a re-registered worker on the same device starts at its learned speed
    w2 = s2.register(host="h", device="cuda:3")
    assert s2.workers[w2].speed_factor == pytest.approx(s.workers[wid].speed_factor)
    assert s2.workers[w2].speed_factor != 1.0
    # another device starts neutral
    assert s2.workers[s2.register(host="h", device="cuda:4")].speed_factor == 1.0
    assert s2.estimate("RandomForestClassifier", 7.0) == pytest.approx(s.estimate("RandomForestClassifier", 7.0))


def test_corrupt_state_is_ignored(tmp_path):
    p = tmp_path / "s.json"
    p.write_text("{not json")
    assert Scheduler(state_path=str(p)).calib == {}
    p.write_text(json.dumps({"version": 1, "calib": {"a": "x"}}))
    assert Scheduler(state_path=str(p)).calib == {}


def test_restart_plans_like_warm_process(tmp_path):
    """A Controller restarted on the same journal slices its first job exactly like the
    warm process would (same calibration, same slice plan, same estimates)."""
    cfg = Config(data_root=str(tmp_path / "data"), journal=str(tmp_path / "journal.jsonl"), device="cpu",
                 chunk_target_s=0.05)
    grid = {"n_estimators": [3, 5, 8], "max_depth": [2, 4, None]}
    nxt = _j1("job-next", "RandomForestClassifier", {"n_estimators": [4, 6, 9, 12], "max_depth": [3, 5, 7]})
    c = Controller(cfg)
    try:
        sid = c.create_session()[1]["session_id"]
        c.download_data(sid, {"dataset_url": "iris", "dataset_name": "iris", "dataset_type": "sklearn"})
        c.train(sid, _j1("job-warm", "RandomForestClassifier", grid))
        assert _wait(c, sid, "job-warm")["job_status"] == "completed"
        assert c.scheduler.calib, "the warm job calibrated nothing"
        plan = job_plan(nxt)
        todo = list(range(len(plan["candidates"])))
        warm_calib = dict(c.scheduler.calib)
        warm_slices = plan_slices(c, plan, todo, 120, 4, 3)
        warm_est = [c.scheduler.estimate(plan["model_type"], u) for u in (1.0, 123.0)]
    finally:
        c.shutdown()
    assert os.path.exists(scheduler_state_path(cfg))
    c2 = Controller(cfg)
    try:
        assert c2.scheduler.calib == pytest.approx(warm_calib)
        assert plan_slices(c2, plan, todo, 120, 4, 3) == warm_slices
        assert [c2.scheduler.estimate(plan["model_type"], u) for u in (1.0, 123.0)] == pytest.approx(warm_est)
    finally:
        c2.shutdown()
    # without the state file the restart falls back to the prior (1.0 s per cost unit)
    os.remove(scheduler_state_path(cfg))
    c3 = Controller(cfg)
    try:
        assert c3.scheduler.calib == {}
    finally:
        c3.shutdown()
