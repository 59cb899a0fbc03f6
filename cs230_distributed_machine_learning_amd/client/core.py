"""``MLTaskManager`` — the client SDK, API-compatible with ``distributed-ml`` 0.2.6.

Public surface kept from DistributedLibrary/src/distributed_ml/core.py:15-213:
``MLTaskManager(url)``, ``check_data``, ``download_data``, ``preprocess``, ``train``,
``check_job_status``, ``download_best_model`` and the J1 job JSON it sends
(``model_details`` from ``_extract_model_details``, ``train_params``, ``timestamp``).

Fixed against the reference:
* D3  — ``train`` POSTs the JSON ``/train`` route (202-style ack + job id); streaming
  progress is opt-in (``stream=True``) and parsed as SSE;
* D4  — ``check_job_status`` returns the J6 status dict (``/check_status``), so
  ``wait_for_completion`` works; raw J3 records are ``metrics(job_id)``;
* D7/D8 — ``RandomizedSearchCV.random_state`` and scipy distributions are serialised
  (``{"dist": "loguniform", "a": .., "b": ..}``) instead of ``str()``;
* D20 — session creation checks ``status in (200, 201)``;
* D21 — ``url`` is optional: ``MLTaskManager()`` runs an in-process engine on the
  local device (CPU, or the GPU when present) with the same JSON contract.
"""
from __future__ import annotations

import json
import math
import os
import time
import uuid
from datetime import datetime
from typing import Any, Dict, Optional

import numpy as np

from ..search.grid import encode_distribution


class _LocalTransport:
    """Routes SDK calls straight into an in-process Controller (no HTTP)."""

    _shared = None

    def __init__(self, controller=None):
        if controller is None:
            if _LocalTransport._shared is None:
                from ..engine.service import Controller

                _LocalTransport._shared = Controller()
            controller = _LocalTransport._shared
        self.ctl = controller

    def request(self, method: str, endpoint: str, data=None, params=None):
        parts = [p for p in endpoint.strip("/").split("/") if p]
        route, args = parts[0], parts[1:]
        c = self.ctl
        if route == "create_session":
            return c.create_session()
        if route == "check_data":
            return c.check_data(args[0], (params or {}).get("dataset_name"))
        if route == "download_data":
            return c.download_data(args[0], data)
        if route == "preprocess":
            return c.preprocess(args[0], data)
        if route == "train":
            return c.train(args[0], data)
        if route == "train_status":
            status, payload = c.train_status(args[0], data)
            if status != 200:
                return status, payload
            return status, list(payload)
        if route == "check_status":
            return c.check_status(args[0], args[1])
        if route == "metrics":
            return c.metrics(args[0], args[1], wait=(params or {}).get("wait", True) not in (False, "false"))
        if route == "download_model":
            return c.download_model(args[0], args[1], data)
        if route == "health":
            return c.health()
        raise ValueError(f"unknown endpoint {endpoint}")


class MLTaskManager:
    def __init__(self, url: Optional[str] = None, controller=None, timeout: float = 30.0):
        self.api_url = url.rstrip("/") if url else None
        self.timeout = timeout
        self._local = None if self.api_url else _LocalTransport(controller)
        self._http = None
        if self.api_url:
            import requests

            self._http = requests.Session()
        self.job_id: Optional[str] = None
        self.result = None
        self.session_id = self._create_session()

    # ---- transport ------------------------------------------------------------------------
    def _create_session(self) -> str:
        status, body = self._raw("create_session", "post")
        if status in (200, 201) and isinstance(body, dict) and body.get("session_id"):
            print(f"Session Created: {body['session_id']}")
            return body["session_id"]
        raise Exception(f"Failed to create session: {body}")

    def _raw(self, endpoint, method="post", data=None, params=None, stream=False):
        if self._local is not None:
            return self._local.request(method, endpoint, data, params)
        url = f"{self.api_url}/{endpoint.lstrip('/')}"
        r = self._http.request(method, url, json=data, params=params, timeout=None if stream else self.timeout,
                               stream=stream)
        if stream:
            return r.status_code, r
        try:
            return r.status_code, r.json()
        except ValueError:
            return r.status_code, {"raw": r.text}

    def _api_request(self, endpoint, method="post", data=None, params=None):
        """JSON request with the reference's error convention ({"status":"error",...})."""
        try:
            if data:
                data = json.loads(json.dumps(data, default=self._json_serializer))
                data = self._clean_dict(data)
            status, body = self._raw(endpoint, method, data, params)
            if status >= 400:
                msg = body.get("error") if isinstance(body, dict) else body
                return {"status": "error", "message": f"{status}: {msg}", "code": status,
                        **({"detail": body} if isinstance(body, dict) else {})}
            return body
        except Exception as e:  # network errors mirror requests.RequestException handling
            return {"status": "error", "message": str(e)}

    @staticmethod
    def _json_serializer(obj):
        if isinstance(obj, (np.floating,)):
            v = float(obj)
            return None if math.isnan(v) or math.isinf(v) else v
        if isinstance(obj, (np.integer,)):
            return int(obj)
        if isinstance(obj, np.bool_):
            return bool(obj)
        if isinstance(obj, np.ndarray):
            return obj.tolist()
        try:
            import pandas as pd

            if isinstance(obj, (pd.DataFrame, pd.Series)):
                return obj.to_dict()
        except ImportError:  # pragma: no cover
            pass
        if hasattr(obj, "rvs") and hasattr(obj, "dist"):
            return encode_distribution(obj)
        if isinstance(obj, type):
            return obj.__name__
        return str(obj)

    def _clean_dict(self, data):
        if isinstance(data, dict):
            return {k: self._clean_dict(v) for k, v in data.items()}
        if isinstance(data, list):
            return [self._clean_dict(v) for v in data]
        if isinstance(data, float) and (math.isnan(data) or math.isinf(data)):
            return None
        return data

    # ---- data -------------------------------------------------------------------------------
    def check_data(self, data_name):
        return self._api_request(f"check_data/{self.session_id}", "get", params={"dataset_name": data_name})

    def download_data(self, data_link, data_name, data_type):
        return self._api_request(f"download_data/{self.session_id}", "post", data={
            "dataset_url": data_link, "dataset_name": data_name, "dataset_type": data_type})

    def preprocess(self, dataset_name, yaml):
        """``yaml``: a file name under the server's config dir (reference), a local path,
        YAML text, or a dict (sent inline — D23)."""
        payload: Dict[str, Any] = {"dataset_id": dataset_name, "yaml_url": yaml}
        if isinstance(yaml, dict):
            payload["config"] = yaml
        elif isinstance(yaml, str) and os.path.isfile(yaml):
            with open(yaml, "r", encoding="utf-8") as f:
                payload["yaml"] = f.read()
        elif isinstance(yaml, str) and "\n" in yaml:
            payload["yaml"] = yaml
        return self._api_request(f"preprocess/{self.session_id}", "post", data=payload)

    # ---- model details (J1) -------------------------------------------------------------------
    def _extract_model_details(self, estimator) -> Dict[str, Any]:
        if isinstance(estimator, dict) and "model_type" in estimator:
            return estimator
        is_grid = hasattr(estimator, "param_grid") and hasattr(estimator, "estimator")
        is_rand = hasattr(estimator, "param_distributions") and hasattr(estimator, "estimator")
        if is_grid or is_rand:
            base = estimator.estimator
            model_type = type(base).__name__
            if is_grid:
                search_type = "GridSearchCV"
                search = {"param_grid": estimator.param_grid}
            else:
                search_type = "RandomizedSearchCV"
                rs = getattr(estimator, "random_state", None)
                search = {"param_distributions": _encode_dists(estimator.param_distributions),
                          "n_iter": estimator.n_iter, "random_state": rs if isinstance(rs, (int, type(None))) else None}
            cv_params = {k: getattr(estimator, k, None) for k in
                         ("cv", "scoring", "refit", "verbose", "error_score", "return_train_score")}
            hyper = {"base_estimator_params": {k.split("__")[-1]: v for k, v in base.get_params().items()},
                     "search_params": search, "cv_params": cv_params}
            return {"model_type": model_type, "search_type": search_type, "hyperparameters": hyper}
        return {"model_type": type(estimator).__name__, "hyperparameters": dict(estimator.get_params())}

    # ---- jobs ----------------------------------------------------------------------------------
    def train(self, estimator, dataset_name, train_params=None, wait_for_completion=False, stream=False,
              polling_interval: float = 1.0, timeout: Optional[float] = None):
        self.job_id = str(uuid.uuid4())
        train_params = dict(train_params or {})
        details = self._extract_model_details(estimator)
        if "test_size" not in train_params and "search_type" not in details:
            train_params["test_size"] = 0.2
        payload = {"job_id": self.job_id, "session_id": self.session_id, "dataset_id": dataset_name,
                   "model_details": details, "train_params": train_params, "timestamp": datetime.now().isoformat()}
        if stream:
            return self._train_stream(payload)
        resp = self._api_request(f"train/{self.session_id}", "post", data=payload)
        print("Job Created:", self.job_id)
        print(resp.get("status"))
        if wait_for_completion and resp.get("status") != "error":
            return self._wait_for_completion(self.job_id, polling_interval, timeout)
        return resp

    def _train_stream(self, payload):
        data = json.loads(json.dumps(payload, default=self._json_serializer))
        data = self._clean_dict(data)
        status, body = self._raw(f"train_status/{self.session_id}", "post", data, stream=True)
        if status != 200:
            return {"status": "error", "message": str(body if isinstance(body, dict) else body.text)}
        last = None
        events = body if isinstance(body, list) else _iter_sse(body)
        for ev in events:
            if isinstance(ev, str):
                ev = json.loads(ev[len("data: "):].strip()) if ev.startswith("data: ") else json.loads(ev)
            last = ev
        self.result = last
        return last

    def check_job_status(self, job_id=None):
        return self._api_request(f"check_status/{self.session_id}/{job_id or self.job_id}", "get")

    def metrics(self, job_id=None, wait: bool = True):
        return self._api_request(f"metrics/{self.session_id}/{job_id or self.job_id}", "get",
                                 params={"wait": "true" if wait else "false"})

    def _wait_for_completion(self, job_id, polling_interval=1.0, timeout=None):
        start = time.time()
        bar = None
        try:
            from tqdm import tqdm

            bar = tqdm(total=100, desc="Training Progress")
        except ImportError:  # pragma: no cover
            pass
        try:
            while True:
                if timeout is not None and time.time() - start > timeout:
                    return {"status": "error", "message": "Timeout exceeded"}
                status = self.check_job_status(job_id)
                progress = status.get("job_status", 0)
                if progress in ("completed", "failed"):
                    value = 100
                elif progress in ("pending", None, 0):
                    value = 0
                else:
                    try:
                        value = int(float(progress))
                    except (TypeError, ValueError):
                        value = 0
                if bar is not None:
                    bar.update(max(0, value - bar.n))
                if status.get("job_status") in ("completed", "failed") or status.get("status") == "error":
                    self.result = status
                    return status
                time.sleep(polling_interval)
        finally:
            if bar is not None:
                bar.close()

    @staticmethod
    def load_model(path: str):
        """A downloaded ``.npz`` artefact as an estimator-like object with ``predict``,
        ``predict_proba`` / ``decision_function`` (classifiers), ``score`` and ``transform``
        (PCA) -- the usable model the reference hands over as a pickle
        (DistributedLibrary/src/distributed_ml/core.py:201-206); loading executes nothing."""
        from ..engine.model_store import load_predictor

        return load_predictor(path)

    def download_best_model(self, job_id=None, model_path=None, model_id=None, dest: Optional[str] = None,
                            load: bool = False):
        """Fetch the stored best model (``.npz`` artefact); returns the local path, or with
        ``load=True`` the loaded estimator (:meth:`load_model`)."""
        out = self._download_model(job_id, model_path, model_id, dest)
        if load and isinstance(out, str):
            return self.load_model(out)
        return out

    def _download_model(self, job_id=None, model_path=None, model_id=None, dest: Optional[str] = None):
        job_id = job_id or self.job_id
        body = {"model_path": model_path, "model_id": model_id}
        if self._local is not None:
            status, payload = self._local.request("post", f"download_model/{self.session_id}/{job_id}", body)
            if status != 200:
                return {"status": "error", "message": payload}
            if dest:
                import shutil

                shutil.copy(payload["__file__"], dest)
                return dest
            return payload["__file__"]
        r = self._http.post(f"{self.api_url}/download_model/{self.session_id}/{job_id}", json=body,
                            timeout=self.timeout)
        if r.status_code != 200:
            try:
                return {"status": "error", "message": r.json()}
            except ValueError:
                return {"status": "error", "message": r.text}
        dest = dest or f"{model_id or job_id}.npz"
        with open(dest, "wb") as f:
            f.write(r.content)
        return dest


def _iter_sse(resp):
    for raw in resp.iter_lines(decode_unicode=True):
        if raw and raw.startswith("data: "):
            yield json.loads(raw[len("data: "):])


def _encode_dists(pd):
    if isinstance(pd, list):
        return [_encode_dists(x) for x in pd]
    out = {}
    for k, v in pd.items():
        out[k] = encode_distribution(v) if hasattr(v, "rvs") else v
    return out
