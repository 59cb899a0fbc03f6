"""End-to-end tour of the client API (the reference's demo_tests.py flow).

    python examples/quickstart.py                      # in-process engine (CPU or local GPU)
    python examples/quickstart.py http://127.0.0.1:5001  # against `python -m cs230_distributed_machine_learning_amd.serve`

Steps: register a dataset, preprocess it with the titanic-style YAML, train a plain
RandomForest, then a GridSearchCV and a RandomizedSearchCV over LogisticRegression, and
download the refitted best model.  No network: datasets come from scikit-learn's
bundled copies or a local CSV.
"""
import os
import sys
import tempfile

import numpy as np
import pandas as pd
import scipy.stats as st
from sklearn.ensemble import RandomForestClassifier
from sklearn.linear_model import LogisticRegression
from sklearn.model_selection import GridSearchCV, RandomizedSearchCV

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_ml import MLTaskManager  # noqa: E402

url = sys.argv[1] if len(sys.argv) > 1 else None
tm = MLTaskManager(url)

# a titanic-shaped table (synthetic; the reference downloads it from Kaggle)
rng = np.random.RandomState(0)
n = 891
df = pd.DataFrame({
    "PassengerId": np.arange(1, n + 1), "Pclass": rng.choice([1, 2, 3], n, p=[0.25, 0.2, 0.55]),
    "Name": [f"passenger {i}" for i in range(n)], "Sex": rng.choice(["male", "female"], n, p=[0.65, 0.35]),
    "Age": np.where(rng.rand(n) < 0.2, np.nan, rng.gamma(4, 7, n).round()), "SibSp": rng.poisson(0.5, n),
    "Parch": rng.poisson(0.4, n), "Ticket": ["T"] * n, "Fare": rng.lognormal(3, 1, n).round(2),
    "Cabin": [None] * n, "Embarked": rng.choice(["S", "C", "Q", None], n, p=[0.7, 0.19, 0.09, 0.02])})
logit = 1.5 * (df.Sex == "female") - 0.8 * (df.Pclass - 2) - 0.02 * df.Age.fillna(30) + 0.3
df["Survived"] = (rng.rand(n) < 1 / (1 + np.exp(-logit))).astype(int)
csv = os.path.join(tempfile.mkdtemp(), "titanic.csv")
df.to_csv(csv, index=False)

print(tm.download_data(csv, "titanic", "local"))
print(tm.check_data("titanic"))
yaml_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "titanic_preprocess.yaml")
print(tm.preprocess("titanic", open(yaml_path).read()))

# plain estimator: one fit + 5-fold CV (reference J1a)
out = tm.train(RandomForestClassifier(n_estimators=50), "titanic", {"test_size": 0.25, "random_state": 42,
                                                                     "target_column": "Survived"},
               wait_for_completion=True)
print("RF:", {k: out["job_result"]["results"][0][k] for k in ("accuracy", "mean_cv_score")})

grid = {"C": [0.1, 1.0, 10.0, 100], "solver": ["liblinear", "lbfgs"]}
out = tm.train(GridSearchCV(LogisticRegression(max_iter=500), grid, cv=5), "titanic",
               {"test_size": 0.25, "random_state": 42, "target_column": "Survived"}, wait_for_completion=True)
print("Grid best:", out["best_result"]["parameters"]["C"], out["best_result"]["parameters"]["solver"],
      round(out["best_result"]["mean_cv_score"], 4))

dist = {"C": st.loguniform(1e-2, 1e2), "solver": ["liblinear", "lbfgs"]}
out = tm.train(RandomizedSearchCV(LogisticRegression(max_iter=500), dist, n_iter=12, cv=5, random_state=0),
               "titanic", {"target_column": "Survived"}, wait_for_completion=True)
print("Random best:", out["best_result"]["parameters"], round(out["best_result"]["mean_cv_score"], 4))
print("model saved to", tm.download_best_model(dest=os.path.join(tempfile.mkdtemp(), "best.npz")))
