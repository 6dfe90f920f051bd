"""Logging helpers with the reference's file layout (reference utils/logging_utils.py:8-99):
artifacts/highway-ppo/logs/<timestamp>_<pid>_{master,experiment_<id>}.log."""

from __future__ import annotations

import logging
import os
import sys
from datetime import datetime

ARTIFACTS_DIR = os.path.join("artifacts", "highway-ppo")
LOGS_DIR = os.path.join(ARTIFACTS_DIR, "logs")


def ensure_artifacts_dir(custom_path=None):
    path = custom_path or ARTIFACTS_DIR
    os.makedirs(path, exist_ok=True)
    return path


def _stamp() -> str:
    return datetime.now().strftime("%Y%m%d_%H%M%S_%f")[:-3]


def _make_logger(name, path, level, console_level, console_fmt, console_datefmt):
    logger = logging.getLogger(name)
    logger.setLevel(level)
    logger.handlers = []
    fh = logging.FileHandler(path)
    fh.setLevel(level)
    fh.setFormatter(logging.Formatter("%(asctime)s | %(levelname)s | %(message)s"))
    logger.addHandler(fh)
    ch = logging.StreamHandler(sys.stdout)
    ch.setLevel(console_level)
    ch.setFormatter(logging.Formatter(console_fmt, console_datefmt))
    logger.addHandler(ch)
    return logger


def setup_master_logger(log_level=logging.INFO):
    os.makedirs(LOGS_DIR, exist_ok=True)
    path = os.path.join(LOGS_DIR, f"{_stamp()}_{os.getpid()}_master.log")
    logger = _make_logger("master_logger", path, log_level, log_level,
                          "%(asctime)s | %(levelname)s | %(message)s", "%H:%M:%S")
    logger.info(f"Master logger initialized. Log file: {path}")
    return logger


def setup_experiment_logger(experiment_id, log_level=logging.INFO, console_level=logging.WARNING):
    os.makedirs(LOGS_DIR, exist_ok=True)
    name = f"experiment_{experiment_id}"
    path = os.path.join(LOGS_DIR, f"{_stamp()}_{os.getpid()}_{name}.log")
    logger = _make_logger(name, path, log_level, console_level,
                          "%(asctime)s | %(name)s | %(levelname)s | %(message)s", "%H:%M:%S")
    logger.info(f"Experiment logger initialized for {name}. Log file: {path}")
    return logger


def setup_logger(experiment_name="", log_level=logging.INFO):
    if experiment_name:
        return setup_experiment_logger(experiment_name, log_level)
    return setup_master_logger(log_level)
