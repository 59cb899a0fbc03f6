"""Declarative preprocessing (the ``/preprocess`` YAML), reference C11/C12 semantics.

Steps and order follow aws-prod/master/dataset_util.py:43-116 (drop columns, drop
nulls or impute mean/median/mode, outliers clip/iqr, dedupe, categorical
onehot/label/freq, standard scaling, target moved last), with two fixes:

* D22 — ``categorical`` may be a mapping OR a list of single-key mappings (the shipped
  ``titanic_preprocess.yaml:19-22`` uses the list form, which the reference crashes on);
* D23 — the YAML may be passed inline (text or dict) instead of being pre-placed on
  the shared volume.

Additional scaling methods (``minmax``) are accepted.
"""
from __future__ import annotations

from typing import Any, Dict, Mapping

import numpy as np
import pandas as pd
import yaml


def load_config(cfg: Any) -> Dict[str, Any]:
    if cfg is None:
        return {}
    if isinstance(cfg, Mapping):
        return dict(cfg)
    if isinstance(cfg, str):
        text = cfg
        if "\n" not in cfg and (cfg.endswith(".yaml") or cfg.endswith(".yml")):
            with open(cfg, "r", encoding="utf-8") as f:
                text = f.read()
        out = yaml.safe_load(text)
        return dict(out or {})
    raise ValueError(f"unsupported preprocessing config {type(cfg).__name__}")


def _pairs(section: Any):
    """Mapping or list-of-mappings -> iterable of (column, method)."""
    if section is None:
        return []
    if isinstance(section, Mapping):
        return list(section.items())
    if isinstance(section, list):
        out = []
        for item in section:
            if isinstance(item, Mapping):
                out.extend(item.items())
            elif isinstance(item, str):
                out.append((item, None))
        return out
    raise ValueError(f"expected mapping or list, got {section!r}")


def preprocess_frame(df: pd.DataFrame, config: Mapping[str, Any]) -> pd.DataFrame:
    df = df.copy()
    if config.get("drop_columns"):
        df = df.drop(columns=list(config["drop_columns"]), errors="ignore")
    if config.get("drop_null", False):
        df = df.dropna()
    else:
        for col, method in _pairs(config.get("impute")):
            if col not in df.columns:
                continue
            if method == "mean":
                df[col] = df[col].fillna(df[col].mean())
            elif method == "median":
                df[col] = df[col].fillna(df[col].median())
            elif method == "mode":
                m = df[col].mode()
                if len(m):
                    df[col] = df[col].fillna(m.iloc[0])
            elif method is not None:
                df[col] = df[col].fillna(method)
    for col, method in _pairs(config.get("outliers")):
        if col not in df.columns:
            continue
        if method == "clip":
            lo, hi = df[col].quantile(0.01), df[col].quantile(0.99)
            df[col] = df[col].clip(lo, hi)
        elif method == "iqr":
            q1, q3 = df[col].quantile(0.25), df[col].quantile(0.75)
            iqr = q3 - q1
            df = df[(df[col] >= q1 - 1.5 * iqr) & (df[col] <= q3 + 1.5 * iqr)]
    if config.get("drop_duplicates", False):
        df = df.drop_duplicates()
    for col, method in _pairs(config.get("categorical")):
        if col not in df.columns:
            continue
        if method == "onehot":
            dummies = pd.get_dummies(df[col], prefix=col, drop_first=False).astype(np.int64)
            df = pd.concat([df.drop(columns=[col]), dummies], axis=1)
        elif method == "label":
            codes, _ = pd.factorize(df[col].astype(str), sort=True)
            df[col] = codes
        elif method == "freq":
            df[col] = df[col].map(df[col].value_counts(normalize=True))
    scale = config.get("scale") or {}
    method = scale.get("method")
    for col in scale.get("columns", []) or []:
        if col not in df.columns:
            continue
        if method == "standard":
            std = df[col].std()
            df[col] = (df[col] - df[col].mean()) / std if std else 0
        elif method == "minmax":
            lo, hi = df[col].min(), df[col].max()
            df[col] = (df[col] - lo) / (hi - lo) if hi > lo else 0
    target = config.get("target_column")
    if target and target in df.columns:
        df[target] = df.pop(target)
    return df.reset_index(drop=True)
