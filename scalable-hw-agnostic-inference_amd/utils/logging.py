"""Structured logging.

The reference logs with ``print`` and publishes per-request CloudWatch metrics
(`app/run-sd.py:25-37,166-173`).  Here every component logs through ``get_logger``:

* ``SHAI_LOG_FORMAT=json`` (default for workers launched by the supervisor) emits one JSON
  object per line: ``ts``, ``level``, ``logger``, ``msg``, ``pid`` plus the worker identity
  (``app``, ``pod``, ``rank``) and any ``extra={...}`` fields -- greppable and machine-readable
  without a log shipper.
* ``SHAI_LOG_FORMAT=text`` (default interactively) is the usual human format.
* ``SHAI_LOG_LEVEL`` sets the level (INFO).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import time

_STD = set(vars(logging.LogRecord("", 0, "", 0, "", (), None))) | {"message", "asctime"}


class JsonFormatter(logging.Formatter):
    def __init__(self, static: dict | None = None):
        super().__init__()
        self.static = static or {}

    def format(self, r: logging.LogRecord) -> str:
        d = {"ts": round(r.created, 6), "time": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(r.created)),
             "level": r.levelname, "logger": r.name, "msg": r.getMessage(), "pid": r.process}
        d.update(self.static)
        for k, v in vars(r).items():
            if k not in _STD and not k.startswith("_"):
                d[k] = v if isinstance(v, (int, float, str, bool, type(None), list, dict)) else repr(v)
        if r.exc_info:
            d["exc"] = self.formatException(r.exc_info)
        return json.dumps(d, default=str)


def _identity() -> dict:
    e = os.environ
    ident = {"app": e.get("APP"), "pod": e.get("POD_NAME"), "rank": e.get("RANK")}
    return {k: v for k, v in ident.items() if v}


_configured = False


def configure(fmt: str | None = None, level: str | None = None, stream=None) -> None:
    """(Re)configure the ``shai`` logger tree."""
    global _configured
    fmt = (fmt or os.environ.get("SHAI_LOG_FORMAT", "text")).lower()
    level = (level or os.environ.get("SHAI_LOG_LEVEL", "INFO")).upper()
    root = logging.getLogger("shai")
    for h in list(root.handlers):
        root.removeHandler(h)
    h = logging.StreamHandler(stream or sys.stderr)
    if fmt == "json":
        h.setFormatter(JsonFormatter(_identity()))
    else:
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root.addHandler(h)
    root.setLevel(level)
    root.propagate = False
    _configured = True


def get_logger(name: str) -> logging.Logger:
    if not _configured:
        configure()
    return logging.getLogger(name if name.startswith("shai") else f"shai.{name}")
