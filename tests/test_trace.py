"""roctx ranges + host phase timers (utils/trace.py)."""
from cs230_distributed_machine_learning_amd.utils import trace


def test_ranges_accumulate_and_nest():
    trace.summary(reset=True)
    with trace.range("slice RandomForestClassifier x4"):
        with trace.range("forest_build"):
            pass
        with trace.range("forest_build"):
            pass
    trace.mark("done")
    s = trace.summary(reset=True)
    assert s["slice"]["count"] == 1 and s["forest_build"]["count"] == 2
    assert s["slice"]["seconds"] >= s["forest_build"]["seconds"]
    assert trace.summary() == {}


def test_disabled_records_nothing():
    trace.set_enabled(False)
    try:
        with trace.range("x"):
            pass
        assert "x" not in trace.summary()
    finally:
        trace.set_enabled(True)
