"""One typed configuration for controller, gateway, scheduler and workers.

Replaces the three hard-coded ``config.py`` modules and scattered env vars of the
reference (aws-prod/master/config.py:11-18, scheduler/config.py:12-19,
worker/config.py:10-15, scheduler_service.py:29-37).  Values come from
defaults < YAML file (``--config`` / ``DML_CONFIG``) < environment (``DML_*``) <
explicit overrides / CLI flags.
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
    # tree jobs on a table whose float32 copy exceeds this fraction of the device's free
    # HBM keep only the uint8 bins resident (DeviceData binned_only: streamed binning)
    stream_binned_fraction: float = 0.5
    algo_weight: Dict[str, float] = field(default_factory=dict)
    log_dir: Optional[str] = None
    # (no "deterministic" switch: every tree builder is deterministic by construction --
    # classification histograms are integer counts, regression histograms exact 64-bit
    # fixed-point sums, forest_common.h -- so there is no faster non-deterministic mode)

    @property
    def models_dir(self) -> str:
        return os.path.join(os.path.abspath(self.data_root), "models")

    @classmethod
    def from_env(cls, config_file: Optional[str] = None, **overrides) -> "Config":
        cfg = cls()
        path = config_file or os.environ.get("DML_CONFIG")
        if path:
            cfg._apply_file(path)
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

    def _apply_file(self, path: str) -> None:
        """YAML (or JSON) mapping of field names; unknown keys are an error."""
        import yaml

        with open(path) as f:
            doc = yaml.safe_load(f) or {}
        if not isinstance(doc, dict):
            raise ValueError(f"config file {path} must hold a mapping")
        known = {f.name: f for f in fields(self)}
        bad = sorted(k for k in doc if k.replace("-", "_") not in known)
        if bad:
            raise ValueError(f"unknown config keys in {path}: {bad}")
        for k, v in doc.items():
            f = known[k.replace("-", "_")]
            if isinstance(v, str) and "str" not in str(f.type):
                v = _coerce(f.type, v)
            if f.name == "algo_weight" and v is not None:
                v = {str(a).lower(): float(w) for a, w in dict(v).items()}
            setattr(self, f.name, v)

    @staticmethod
    def add_cli(ap: argparse.ArgumentParser) -> None:
        ap.add_argument("--config", help="YAML config file (keys = Config fields)")
        ap.add_argument("--data-root")
        ap.add_argument("--journal")
        ap.add_argument("--device")
        ap.add_argument("--host")
        ap.add_argument("--port", type=int)
        ap.add_argument("--keep-models", choices=["none", "best", "all"])
        ap.add_argument("--hbm-budget-gb", type=float)
        ap.add_argument("--log-dir")
        ap.add_argument("--chunk-target-s", type=float)
        ap.add_argument("--max-retries", type=int)
        ap.add_argument("--dp-auto-gb", type=float)
        ap.add_argument("--dp-min-cells", type=int)

    @classmethod
    def from_args(cls, ns: argparse.Namespace) -> "Config":
        return cls.from_env(config_file=getattr(ns, "config", None),
                            **{k: getattr(ns, k, None) for k in
                               ("data_root", "journal", "device", "host", "port", "keep_models", "hbm_budget_gb",
                                "log_dir", "chunk_target_s", "max_retries", "dp_auto_gb", "dp_min_cells")})

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
