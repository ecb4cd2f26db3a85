"""Logging configuration: the reference's log4j layout in Python ``logging``.

The reference ships three log4j property files (``config/log4j_master.properties``,
``config/log4j_slave.properties``, ``config/log4j.properties``, each lines 1-35): the root
logger writes to stdout and to three daily-rolling files split by threshold —

    log/<role>.log          DEBUG and above   (appender "info",  datePattern '-'yyyy-MM-dd)
    log/<role>_warn.log     WARN and above    (appender "warn")
    log/<role>_error.log    ERROR and above   (appender "error")

with the pattern ``%d{yyyy-MM-dd HH:mm:ss} %5p %c{1}:%L - %m%n``.  :func:`configure_logging`
builds the same thing (``TimedRotatingFileHandler`` at midnight, suffix ``-%Y-%m-%d``).

Configuration sources, first match wins:

* ``MP4X_LOG_CONFIG=<file>``: a standard ``logging.config`` file — ``.ini``/``.conf``
  (``fileConfig``), ``.json`` or ``.yaml``/``.yml`` (``dictConfig``; YAML via ``safe_load``).
  ``config/logging_master.ini`` and ``config/logging_slave.ini`` in the repo are the
  log4j-equivalent defaults in that format (the reference's
  ``-Dlog4j.configuration=file:config/log4j_master.properties``, README.md:24);
* otherwise the built-in layout above, in ``MP4X_LOG_DIR`` (default ``log``), at
  ``MP4X_LOG_LEVEL`` (default INFO).  ``MP4X_LOG_DIR=-`` keeps stdout only.
"""
from __future__ import annotations

import json
import logging
import logging.config
import logging.handlers
import os
import sys
from typing import Optional

PATTERN = "%(asctime)s %(levelname)5s %(name)s:%(lineno)d - %(message)s"
DATEFMT = "%Y-%m-%d %H:%M:%S"

_HANDLER_TAG = "_mp4x_logconf"


def _daily(path: str, threshold: int, fmt: logging.Formatter) -> logging.Handler:
    h = logging.handlers.TimedRotatingFileHandler(path, when="midnight", encoding="utf-8")
    h.suffix = "-%Y-%m-%d"         # log4j datePattern '-'yyyy-MM-dd
    h.setLevel(threshold)
    h.setFormatter(fmt)
    return h


def _load_file(path: str) -> None:
    low = path.lower()
    if low.endswith(".json"):
        with open(path) as f:
            logging.config.dictConfig(json.load(f))
    elif low.endswith((".yaml", ".yml")):
        import yaml
        with open(path) as f:
            logging.config.dictConfig(yaml.safe_load(f))
    else:
        logging.config.fileConfig(path, disable_existing_loggers=False)


def configure_logging(role: str = "slave", log_dir: Optional[str] = None, level: Optional[str] = None,
                      config_file: Optional[str] = None, stream=None) -> logging.Logger:
    """Install the reference's stdout + info/warn/error daily-rolling layout on the root logger.

    ``role`` names the files (``master`` → ``log/master.log``, ``master_warn.log``,
    ``master_error.log``).  Idempotent: handlers installed by an earlier call are replaced,
    handlers installed by the application are left alone.  Returns the root logger."""
    config_file = config_file or os.environ.get("MP4X_LOG_CONFIG")
    root = logging.getLogger()
    if config_file:
        _load_file(config_file)
        return root
    level = (level or os.environ.get("MP4X_LOG_LEVEL", "INFO")).upper()
    log_dir = log_dir if log_dir is not None else os.environ.get("MP4X_LOG_DIR", "log")
    for h in list(root.handlers):
        if getattr(h, _HANDLER_TAG, False):
            root.removeHandler(h)
            h.close()
    fmt = logging.Formatter(PATTERN, DATEFMT)
    handlers = []
    out = logging.StreamHandler(stream or sys.stdout)
    out.setFormatter(fmt)
    handlers.append(out)
    if log_dir and log_dir != "-":
        os.makedirs(log_dir, exist_ok=True)
        handlers.append(_daily(os.path.join(log_dir, f"{role}.log"), logging.DEBUG, fmt))
        handlers.append(_daily(os.path.join(log_dir, f"{role}_warn.log"), logging.WARNING, fmt))
        handlers.append(_daily(os.path.join(log_dir, f"{role}_error.log"), logging.ERROR, fmt))
    for h in handlers:
        setattr(h, _HANDLER_TAG, True)
        root.addHandler(h)
    root.setLevel(level)
    return root
