"""Rank-aware logger with TRAIN / EVAL levels.

Parity: reference ``ppfleetx/utils/log.py:30-175`` (custom TRAIN=21 / EVAL=22
levels, ``advertise()`` banner).  Unlike the reference, only the ranks selected
by ``FLEETX_LOG_ALL_RANKS`` (default: every rank logs, prefixed by its rank)
emit, and there is no colorlog dependency.
"""
import logging
import os
import sys
import threading
import time

TRAIN = 21
EVAL = 22
logging.addLevelName(TRAIN, "TRAIN")
logging.addLevelName(EVAL, "EVAL")


def _rank():
    return int(os.environ.get("RANK", os.environ.get("PADDLE_TRAINER_ID", "0")))


class _RankFilter(logging.Filter):
    def filter(self, record):
        record.rank = _rank()
        return True


class Logger:
    """Thin wrapper over :mod:`logging` with ``train``/``eval`` helpers."""

    def __init__(self, name="FleetX-AMD"):
        self.logger = logging.getLogger(name)
        self.logger.propagate = False
        if not self.logger.handlers:
            handler = logging.StreamHandler(sys.stdout)
            handler.setFormatter(logging.Formatter(
                "[%(asctime)s] [%(levelname)8s] [rank %(rank)s] - %(message)s",
                datefmt="%Y/%m/%d %H:%M:%S"))
            handler.addFilter(_RankFilter())
            self.logger.addHandler(handler)
        self.logger.setLevel(os.environ.get("FLEETX_LOG_LEVEL", "INFO"))
        self._enabled = True

    def _emit(self, level, msg, *args):
        if not self._enabled:
            return
        if os.environ.get("FLEETX_LOG_RANK0_ONLY", "0") == "1" and _rank() != 0:
            return
        self.logger.log(level, msg, *args)

    def info(self, msg, *args):
        self._emit(logging.INFO, msg, *args)

    def debug(self, msg, *args):
        self._emit(logging.DEBUG, msg, *args)

    def warning(self, msg, *args):
        self._emit(logging.WARNING, msg, *args)

    warn = warning

    def error(self, msg, *args):
        self._emit(logging.ERROR, msg, *args)

    def train(self, msg, *args):
        self._emit(TRAIN, msg, *args)

    def eval(self, msg, *args):
        self._emit(EVAL, msg, *args)

    def enable(self):
        self._enabled = True

    def disable(self):
        self._enabled = False

    def processing(self, msg, interval=0.5):
        """Context manager printing a spinner while a slow host step runs."""
        outer = self

        class _Spinner:
            def __enter__(self):
                self._stop = threading.Event()

                def run():
                    marks = "|/-\\"
                    i = 0
                    while not self._stop.is_set():
                        if outer._enabled:
                            sys.stdout.write("\r{} {}".format(msg, marks[i % 4]))
                            sys.stdout.flush()
                        i += 1
                        time.sleep(interval)

                self._t = threading.Thread(target=run, daemon=True)
                self._t.start()
                return self

            def __exit__(self, *exc):
                self._stop.set()
                self._t.join()
                if outer._enabled:
                    sys.stdout.write("\r")
                return False

        return _Spinner()


logger = Logger()


def advertise():
    """Start-of-run banner (reference ``log.py:150-175``)."""
    lines = [
        "FleetX-AMD: MI355X-native large-model training toolkit",
        "PyTorch-ROCm + HIP/CDNA4 kernels + RCCL over xGMI",
    ]
    width = max(len(l) for l in lines) + 8
    logger.info("=" * width)
    for l in lines:
        logger.info("=={}==".format(l.center(width - 4)))
    logger.info("=" * width)
