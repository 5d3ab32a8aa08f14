"""stdlib logging helpers (reference divrec/utils/divrec_logger.py:4-27)."""
import logging
from typing import Optional

LOG_FORMAT = "%(asctime)s %(name)s [%(levelname)s] %(message)s"


def _handler(h: logging.Handler) -> logging.Handler:
    h.setLevel(logging.INFO)
    h.setFormatter(logging.Formatter(LOG_FORMAT))
    return h


def get_file_handler(filepath: str) -> logging.Handler:
    return _handler(logging.FileHandler(filepath))


def get_stream_handler() -> logging.Handler:
    return _handler(logging.StreamHandler())


def get_logger(name: str, filepath: Optional[str] = None) -> logging.Logger:
    logger = logging.getLogger(name)
    logger.setLevel(logging.INFO)
    if filepath is not None:
        logger.addHandler(get_file_handler(filepath))
    logger.addHandler(get_stream_handler())
    return logger
