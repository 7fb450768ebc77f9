"""Logger factory with the reference's format and noise policy (``config.py:49-80``)."""
from __future__ import annotations

import logging
import os

LOG_FORMAT = "[%(levelname)s] %(asctime)s |%(name)s| %(message)s"
_QUIET = ("pymongo", "pymongo.topology", "confluent_kafka", "uvicorn", "uvicorn.access")


def get_logger(name: str) -> logging.Logger:
    level = os.getenv("LOG_LEVEL", "INFO").upper()
    if level not in ("DEBUG", "INFO", "WARNING", "ERROR"):
        level = "INFO"
    root = logging.getLogger()
    if not root.handlers:
        logging.basicConfig(level=getattr(logging, level), format=LOG_FORMAT)
        for n in _QUIET:
            logging.getLogger(n).setLevel(logging.WARNING)
    return logging.getLogger(name)
