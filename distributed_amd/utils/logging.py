"""Logging with TF-style INFO/WARNING lines (reference README.md:395-412)."""
from __future__ import annotations

import logging as _logging
import os
import sys

_LOGGER = None


def get_logger() -> _logging.Logger:
    global _LOGGER
    if _LOGGER is None:
        lg = _logging.getLogger("distributed_amd")
        if not lg.handlers:
            h = _logging.StreamHandler(sys.stderr)
            h.setFormatter(_logging.Formatter("%(levelname)s:distributed_amd:%(message)s"))
            lg.addHandler(h)
        lg.setLevel(os.environ.get("DAMD_LOG_LEVEL", "INFO").upper())
        lg.propagate = False
        _LOGGER = lg
    return _LOGGER


def info(msg, *a):
    get_logger().info(msg, *a)


def warning(msg, *a):
    get_logger().warning(msg, *a)


def debug(msg, *a):
    get_logger().debug(msg, *a)


def error(msg, *a):
    get_logger().error(msg, *a)
