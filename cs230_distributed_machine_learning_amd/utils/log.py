"""Logging: console + daily-rotated file (reference */logger_util.py: midnight, 7 backups)."""
from __future__ import annotations

import logging
import os
from logging.handlers import TimedRotatingFileHandler
from typing import Optional

_FMT = "%(asctime)s %(levelname)s [%(name)s] %(message)s"


def get_logger(name: str = "dml", log_dir: Optional[str] = None) -> logging.Logger:
    logger = logging.getLogger(name)
    if getattr(logger, "_dml_configured", False):
        return logger
    logger.setLevel(os.environ.get("DML_LOG_LEVEL", "INFO"))
    logger.propagate = False
    sh = logging.StreamHandler()
    sh.setFormatter(logging.Formatter(_FMT))
    logger.addHandler(sh)
    if log_dir:
        os.makedirs(log_dir, exist_ok=True)
        fh = TimedRotatingFileHandler(os.path.join(log_dir, "app.log"), when="midnight", backupCount=7)
        fh.setFormatter(logging.Formatter(_FMT))
        logger.addHandler(fh)
    logger._dml_configured = True  # type: ignore[attr-defined]
    return logger
