"""Structured logging with DryadLINQ-compatible levels.

Reference: DryadLinqLog levels Off/Critical/Error/Warning/Information/Verbose = 0/1/3/7/15/31
(LinqToDryad/Constants.cs:72-112, QueryTraceLevel.cs:30-37); workers read ``DRYAD_LOGGING_LEVEL``
(LocalJobSubmission.cs:103,128).  Levels map onto Python logging.
"""
from __future__ import annotations

import logging
import os

_MAP = {0: logging.CRITICAL + 10, 1: logging.CRITICAL, 3: logging.ERROR, 7: logging.WARNING, 15: logging.INFO,
        31: logging.DEBUG}


def level_from_env() -> int:
    v = os.environ.get("DRYAD_LOGGING_LEVEL")
    if v is None:
        return logging.WARNING
    try:
        return _MAP.get(int(v), logging.INFO)
    except ValueError:
        return getattr(logging, v.upper(), logging.WARNING)


def get_logger(name: str) -> logging.Logger:
    lg = logging.getLogger("dryad." + name)
    if not logging.getLogger("dryad").handlers:
        h = logging.StreamHandler()
        h.setFormatter(logging.Formatter("[%(asctime)s %(name)s %(levelname)s] %(message)s"))
        root = logging.getLogger("dryad")
        root.addHandler(h)
        root.setLevel(level_from_env())
        root.propagate = False
    return lg


def set_level(dryad_level: int):
    logging.getLogger("dryad").setLevel(_MAP.get(int(dryad_level), logging.INFO))
