"""Process-wide logger with millisecond timestamps (reference:
metisfl/utils/metis_logger.py:10-75).  The figlet banner of the reference
needs pyfiglet/termcolor, which are not installed; the banner is a plain
text header instead."""
from __future__ import annotations

import datetime as dt
import logging
import sys
import threading


class _MsFormatter(logging.Formatter):
    def formatTime(self, record, datefmt=None):  # noqa: N802 (logging API)
        ct = dt.datetime.fromtimestamp(record.created)
        return "%s,%03d" % (ct.strftime("%Y-%m-%d %H:%M:%S"), record.msecs)


class MetisASCIIArt:
    @classmethod
    def print(cls):
        print("=" * 60 + "\n  METIS Federated Learning -- MI355X-native engine\n" + "=" * 60,
              file=sys.stderr, flush=True)


class MetisLogger:
    _logger = logging.getLogger("Metis")
    _lock = threading.Lock()
    if not _logger.handlers:
        _h = logging.StreamHandler(stream=sys.stderr)
        _h.setFormatter(_MsFormatter("%(asctime)s: %(name)s: %(levelname)s: %(message)s"))
        _logger.addHandler(_h)
        _logger.setLevel("INFO")
        _logger.propagate = False

    @classmethod
    def getlogger(cls) -> logging.Logger:
        with cls._lock:
            return cls._logger

    @classmethod
    def set_level(cls, level) -> None:
        cls._logger.setLevel(level)

    @classmethod
    def log(cls, level, msg, *args, **kwargs):
        cls.getlogger().log(level, msg, *args, **kwargs)

    @classmethod
    def debug(cls, msg, *args, **kwargs):
        cls.getlogger().debug(msg, *args, **kwargs)

    @classmethod
    def info(cls, msg, *args, **kwargs):
        cls.getlogger().info(msg, *args, **kwargs)

    @classmethod
    def warning(cls, msg, *args, **kwargs):
        cls.getlogger().warning(msg, *args, **kwargs)

    @classmethod
    def error(cls, msg, *args, **kwargs):
        cls.getlogger().error(msg, *args, **kwargs)

    @classmethod
    def fatal(cls, msg, *args, **kwargs):
        cls.getlogger().critical(msg, *args, **kwargs)
