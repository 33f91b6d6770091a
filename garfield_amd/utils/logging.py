"""Contextual, thread-aware console logging and the user-facing exception type.

Reference: ``pytorch_impl/libs/tools/__init__.py:26-246`` (``Context`` with coloured,
per-thread prefixes wrapping stdout/stderr, ``UserException``, ``info``/``warning``/
``error``/``fatal``/``trace`` and a custom excepthook). Same API; the prefix stack is
a ``threading.local`` and output goes through one lock so lines from RPC handler
threads never interleave mid-line.
"""
from __future__ import annotations

import os
import sys
import threading
import traceback

__all__ = ["UserException", "Context", "context", "info", "warning", "error", "fatal", "trace",
           "set_rank_prefix", "install_excepthook"]


class UserException(Exception):
    """An error caused by user input (bad flags, bad GAR parameters, ...)."""


_COLORS = {"header": "\033[1;30m", "red": "\033[1;31m", "green": "\033[1;32m", "yellow": "\033[1;33m",
           "blue": "\033[1;34m", "gray": "\033[0;90m", None: ""}
_RESET = "\033[0m"
_local = threading.local()
_lock = threading.Lock()
_rank_prefix = ""
_use_color = sys.stdout.isatty() and os.environ.get("NO_COLOR") is None


def _stack():
    s = getattr(_local, "stack", None)
    if s is None:
        s = []
        _local.stack = s
    return s


def set_rank_prefix(prefix: str) -> None:
    """Global prefix (e.g. ``"[rank 3] "``) for multi-process runs."""
    global _rank_prefix
    _rank_prefix = prefix


class Context:
    """``with Context("name", "green"):`` prefixes every message printed inside."""

    def __init__(self, name: str | None, color: str | None = None):
        self.name = name
        self.color = color

    def __enter__(self):
        _stack().append((self.name, self.color))
        return self

    def __exit__(self, *exc):
        _stack().pop()
        return False


context = Context


def _prefix(color_default: str | None) -> str:
    parts = []
    for name, color in _stack():
        if name is None:
            continue
        if _use_color and color:
            parts.append(f"{_COLORS.get(color, '')}[{name}]{_RESET}")
        else:
            parts.append(f"[{name}]")
    return _rank_prefix + (" ".join(parts) + " " if parts else "")


def _emit(stream, tag: str | None, color: str | None, *args) -> None:
    msg = " ".join(str(a) for a in args)
    pre = _prefix(color)
    if tag:
        pre += (f"{_COLORS[color]}{tag}{_RESET} " if _use_color and color else f"{tag} ")
    with _lock:
        for line in msg.split("\n") or [""]:
            stream.write(pre + line + "\n")
        stream.flush()


def info(*args) -> None:
    _emit(sys.stdout, None, None, *args)


def warning(*args) -> None:
    _emit(sys.stderr, "(warning)", "yellow", *args)


def error(*args) -> None:
    _emit(sys.stderr, "(error)", "red", *args)


def trace(*args) -> None:
    if os.environ.get("GARFIELD_TRACE", "0") == "1":
        _emit(sys.stderr, "(trace)", "gray", *args)


def fatal(*args, code: int = 1) -> None:
    _emit(sys.stderr, "(fatal)", "red", *args)
    raise SystemExit(code)


def install_excepthook() -> None:
    """Print UserException as a one-line fatal message, other exceptions with a traceback."""

    def hook(typ, value, tb):
        if issubclass(typ, UserException):
            _emit(sys.stderr, "(fatal)", "red", str(value))
        else:
            _emit(sys.stderr, "(fatal)", "red", "".join(traceback.format_exception(typ, value, tb)).rstrip())

    sys.excepthook = hook
