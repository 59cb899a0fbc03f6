"""Host-builder criterion=absolute_error timing vs sklearn (profiles/r2_mae_host_builder_cpu_timing.log)."""
import time, numpy as np
from cs230_distributed_machine_learning_amd.engine.executor import JobSpec, run_candidates
from cs230_distributed_machine_learning_amd.data.device import DeviceData
from sklearn.ensemble import RandomForestRegressor
rng = np.random.default_rng(0)
X = rng.standard_normal((50000, 10)).astype(np.float32)
y = X[:, 0] - X[:, 1] + rng.standard_normal(50000)
spec = JobSpec("RandomForestRegressor", [{"n_estimators": 8, "criterion": "absolute_error", "max_depth": 10}], cv=3, holdout=False, random_state=0)
t = time.perf_counter(); r = run_candidates(DeviceData(X, y, False, "cpu"), spec, [0]); t1 = time.perf_counter() - t
print("ours 3 folds x 8 trees:", round(t1, 2), "s", r[0].result["cv_scores"])
t = time.perf_counter(); RandomForestRegressor(n_estimators=8, criterion="absolute_error", max_depth=10, n_jobs=8).fit(X[:33333], y[:33333]); t2 = time.perf_counter() - t
print("sklearn 1 fold x 8 trees (n_jobs=8):", round(t2, 2), "s")
