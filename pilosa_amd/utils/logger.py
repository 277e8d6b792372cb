"""Logger (reference: logger/logger.go): nop / standard / verbose / capture."""
from __future__ import annotations

import sys
import threading
import time


class NopLogger:
    def printf(self, fmt, *args):
        pass

    def debugf(self, fmt, *args):
        pass


class StandardLogger(NopLogger):
    def __init__(self, stream=None, verbose=False):
        self.stream = stream or sys.stderr
        self.verbose = verbose
        self.mu = threading.Lock()

    def printf(self, fmt, *args):
        msg = (fmt % args) if args else fmt
        with self.mu:
            self.stream.write(time.strftime("%Y/%m/%d %H:%M:%S ") + msg.rstrip("\n") + "\n")
            self.stream.flush()

    def debugf(self, fmt, *args):
        if self.verbose:
            self.printf(fmt, *args)


class CaptureLogger(NopLogger):
    """Keeps messages in memory (tests)."""

    def __init__(self):
        self.prints = []
        self.debugs = []

    def printf(self, fmt, *args):
        self.prints.append((fmt % args) if args else fmt)

    def debugf(self, fmt, *args):
        self.debugs.append((fmt % args) if args else fmt)
