"""One typed configuration for controller, gateway, scheduler and workers.

Replaces the three hard-coded ``config.py`` modules and scattered env vars of the
reference (aws-prod/master/config.py:11-18, scheduler/config.py:12-19,
worker/config.py:10-15, scheduler_service.py:29-37).  Values come from
defaults < environment (``DML_*``) < explicit overrides / CLI flags.
``ALGO_WEIGHT_JSON`` is honoured for compatibility with the reference scheduler.
"""
from __future__ import annotations

import argparse
import json
import os
from dataclasses import asdict, dataclass, field, fields
from typing import Any, Dict, Optional


@dataclass
class Config:
    data_root: str = "./dml_data"
    journal: Optional[str] = None          # JSONL job journal (resume after restart)
    device: str = "auto"                   # auto | cpu | cuda | cuda:N
    host: str = "127.0.0.1"
    port: int = 5001
    sse_interval_s: float = 1.5            # master.py:266
    heartbeat_s: float = 5.0               # worker.py:33
    dead_after_s: float = 10.0             # scheduler_service.py:214
    monitor_tick_s: float = 2.0            # faster than the reference's 15 s (worst case 25 s)
    keep_models: str = "best"              # none | best | all
    refit: bool = True
    max_retries: int = 2
    chunk_target_s: float = 2.0            # progress granularity of a worker slice
    hbm_budget_gb: Optional[float] = None  # forest batch budget (default: 55% of free HBM)
    # parallelism 'auto': a data-parallel-capable job runs row-sharded when its table is
    # at least dp_min_cells cells AND (fewer candidates than ranks OR > dp_auto_gb of fp32)
    dp_auto_gb: float = 48.0
    dp_min_cells: int = 50_000_000
    algo_weight: Dict[str, float] = field(default_factory=dict)
    log_dir: Optional[str] = None
    deterministic: bool = True

    @property
    def models_dir(self) -> str:
        return os.path.join(os.path.abspath(self.data_root), "models")

    @classmethod
    def from_env(cls, **overrides) -> "Config":
        cfg = cls()
        for f in fields(cls):
            env = os.environ.get("DML_" + f.name.upper())
            if env is None:
                continue
            setattr(cfg, f.name, _coerce(f.type, env))
        aw = os.environ.get("ALGO_WEIGHT_JSON")
        if aw:
            try:
                cfg.algo_weight = {k.lower(): float(v) for k, v in json.loads(aw).items()}
            except (ValueError, AttributeError):
                pass
        for k, v in overrides.items():
            if v is not None and hasattr(cfg, k):
                setattr(cfg, k, v)
        return cfg

    @staticmethod
    def add_cli(ap: argparse.ArgumentParser) -> None:
        ap.add_argument("--data-root")
        ap.add_argument("--journal")
        ap.add_argument("--device")
        ap.add_argument("--host")
        ap.add_argument("--port", type=int)
        ap.add_argument("--keep-models", choices=["none", "best", "all"])
        ap.add_argument("--hbm-budget-gb", type=float)
        ap.add_argument("--log-dir")

    @classmethod
    def from_args(cls, ns: argparse.Namespace) -> "Config":
        return cls.from_env(**{k: getattr(ns, k, None) for k in
                               ("data_root", "journal", "device", "host", "port", "keep_models", "hbm_budget_gb",
                                "log_dir")})

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        try:
            import torch

            return "cuda" if torch.cuda.is_available() else "cpu"
        except Exception:
            return "cpu"

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


def _coerce(tp, s: str):
    t = str(tp)
    if "bool" in t:
        return s.lower() in ("1", "true", "yes")
    if "int" in t and "Optional" not in t:
        return int(s)
    if "float" in t:
        return float(s)
    if "Dict" in t:
        return json.loads(s)
    return s
