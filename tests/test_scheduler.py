"""Scheduler core (reference scheduler_service.py:111-351 semantics, D10-D14 fixed)."""
import numpy as np

from cs230_distributed_machine_learning_amd.engine.scheduler import Scheduler, Unit, chunk_units, lpt_assign


def test_lpt_assign_balances_makespan():
    rng = np.random.RandomState(0)
    costs = rng.lognormal(0, 1.2, 200)
    out = lpt_assign(costs, 8)
    loads = np.bincount(out, weights=costs, minlength=8)
    # LPT bound: makespan <= 4/3 OPT; OPT >= max(mean load, max job)
    opt_lb = max(costs.sum() / 8, costs.max())
    assert loads.max() <= 4 / 3 * opt_lb + 1e-9
    # speed-aware: a 2x faster worker takes about twice the work
    out = lpt_assign(costs, 2, speeds=[2.0, 1.0])
    l0, l1 = costs[out == 0].sum(), costs[out == 1].sum()
    assert 1.5 < l0 / l1 < 2.6


def test_chunk_units_respects_target():
    costs = np.full(100, 0.1)
    ch = chunk_units(costs, target=1.0)
    sizes = np.bincount(ch)
    assert sizes.max() <= 11 and ch.max() + 1 >= 9


def test_place_complete_and_release_exactly():
    s = Scheduler(dead_after_s=10)
    a = s.register("h", 1000, "cuda:0")
    b = s.register("h", 1000, "cuda:1")
    units = [Unit(unit_id=f"u{i}", cost=float(10 - i), algo="RandomForestClassifier", mem_mb=100) for i in range(6)]
    plan = s.place(units)
    assert sum(len(v) for v in plan.values()) == 6
    before = {w.worker_id: w.load_seconds for w in s.alive_workers()}
    assert all(v > 0 for v in before.values())
    # calibration changes between placement and completion must not leak load (D11)
    for wid, us in plan.items():
        for u in us:
            s.observe(wid, u, seconds=0.5)
    for w in s.alive_workers():
        assert abs(w.load_seconds) < 1e-9 and w.mem_load_mb == 0
    assert s.calib["randomforestclassifier"] > 0


def test_held_when_no_workers_and_requeue_on_death():
    s = Scheduler(dead_after_s=5)
    u = [Unit(unit_id="x", cost=1.0, algo="SVC")]
    assert s.place(u) == {}
    assert [h.unit_id for h in s.take_held()] == ["x"]          # held, not dropped (D14)
    w = s.register()
    s.place(u)
    lost = s.monitor(now=s.workers[w].last_heartbeat + 6)         # silent worker
    assert [x.unit_id for x in lost] == ["x"] and not s.alive_workers()
    assert not s.heartbeat(w)                                     # must re-register (D28)


def test_algo_weight_scales_estimates():
    s = Scheduler(algo_weight={"SVC": 3.0})
    assert s.estimate("svc", 2.0) == 6.0 and s.estimate("LogisticRegression", 2.0) == 2.0


def test_calibration_is_cost_weighted_so_a_warmup_job_cannot_misprice_a_search():
    """A tiny warm-up slice (all fixed overhead: 0.3 s for 0.001 cost units) followed by
    one real slice (1.5 s for 30 units): the estimate for a 15-unit candidate must be
    near the real 0.05 s/unit, not the warm-up's 300 s/unit."""
    s = Scheduler()
    wid = s.register("local")
    s.observe(wid, Unit("warm", 0.001, algo="RandomForestClassifier"), 0.3)
    s.observe(wid, Unit("real", 30.0, algo="RandomForestClassifier"), 1.5)
    est = s.estimate("RandomForestClassifier", 15.0)
    assert 0.6 < est < 1.2, est


def test_should_recut_when_queue_far_from_target():
    from types import SimpleNamespace

    from cs230_distributed_machine_learning_amd.engine.service import should_recut

    sched = Scheduler()
    ctl = SimpleNamespace(config=SimpleNamespace(chunk_target_s=2.0), scheduler=sched)
    plan = {"model_type": "RandomForestClassifier"}
    costs = [1.0] * 10
    sched.calib["randomforestclassifier"] = 0.1                    # 0.1 s per candidate
    assert should_recut(ctl, plan, [[i] for i in range(10)], costs)           # 0.1 s slices << 2 s
    assert not should_recut(ctl, plan, [list(range(0, 5)) * 4, list(range(5, 10)) * 4], costs)   # 2 s slices
    sched.calib["randomforestclassifier"] = 5.0
    assert should_recut(ctl, plan, [[0, 1], [2, 3], [4, 5]], costs)            # 10 s slices of 2
    assert not should_recut(ctl, plan, [[0], [1], [2]], costs)                 # single candidates: nothing to split
