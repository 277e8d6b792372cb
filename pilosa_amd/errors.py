"""Sentinel errors and HTTP-mapped wrappers (reference: pilosa.go:25-118)."""
from __future__ import annotations

import re


class PilosaError(Exception):
    """Base error; ``str(e)`` is the reference's message."""


class BadRequestError(PilosaError):
    """Maps to HTTP 400."""

    def __init__(self, err):
        super().__init__(str(err))
        self.err = err


class ConflictError(PilosaError):
    """Maps to HTTP 409."""

    def __init__(self, err):
        super().__init__(str(err))
        self.err = err


class NotFoundError(PilosaError):
    """Maps to HTTP 404."""

    def __init__(self, err):
        super().__init__(str(err))
        self.err = err


class APIMethodNotAllowedError(PilosaError):
    """Maps to HTTP 405 (method not allowed in the current cluster state)."""

    def __init__(self, err):
        super().__init__(str(err))
        self.err = err


def _e(msg):
    return PilosaError(msg)


def cause(err: BaseException) -> BaseException:
    """errors.Cause: the innermost error behind :func:`wrap` layers."""
    while getattr(err, "cause", None) is not None and err.cause is not err:
        err = err.cause
    return err


def wrap(err: BaseException, prefix: str) -> PilosaError:
    """errors.Wrap: ``"<prefix>: <err>"`` of the same class (so the same HTTP
    status), with the original reachable through :func:`cause`."""
    cls = type(err) if isinstance(err, PilosaError) else PilosaError
    out = cls.__new__(cls)
    Exception.__init__(out, f"{prefix}: {err}")
    if hasattr(err, "err"):
        out.err = err.err
    out.cause = err
    return out


ErrHostRequired = _e("host required")
ErrIndexRequired = _e("index required")
ErrIndexExists = _e("index already exists")
ErrIndexNotFound = _e("index not found")
ErrFieldRequired = _e("field required")
ErrFieldExists = _e("field already exists")
ErrFieldNotFound = _e("field not found")
ErrBSIGroupNotFound = _e("bsigroup not found")
ErrBSIGroupExists = _e("bsigroup already exists")
ErrBSIGroupNameRequired = _e("bsigroup name required")
ErrInvalidBSIGroupType = _e("invalid bsigroup type")
ErrInvalidBSIGroupRange = _e("invalid bsigroup range")
ErrInvalidBSIGroupValueType = _e("invalid bsigroup value type")
ErrBSIGroupValueTooLow = _e("bsigroup value too low")
ErrBSIGroupValueTooHigh = _e("bsigroup value too high")
ErrInvalidRangeOperation = _e("invalid range operation")
ErrInvalidBetweenValue = _e("invalid value for between operation")
ErrInvalidView = _e("invalid view")
ErrInvalidCacheType = _e("invalid cache type")
ErrName = _e("invalid index or field name, must match [a-z][a-z0-9_-]* and contain at most 64 characters")
ErrLabel = _e("invalid row or column label, must match [A-Za-z0-9_-]")
ErrFragmentNotFound = _e("fragment not found")
ErrQueryRequired = _e("query required")
ErrQueryCancelled = _e("query cancelled")
ErrQueryTimeout = _e("query timeout")
ErrTooManyWrites = _e("too many write commands")
ErrClusterDoesNotOwnShard = _e("node does not own shard")
ErrNodeIDNotExists = _e("node with provided ID does not exist")
ErrNodeNotCoordinator = _e("node is not the coordinator")
ErrResizeNotRunning = _e("no resize job currently running")
ErrNotImplemented = _e("not implemented")
ErrFieldsArgumentRequired = _e("fields argument required")
ErrExpectedFieldListArgument = _e("expected field list argument")
ErrInvalidTimeQuantum = _e("invalid time quantum")
ErrTranslateStoreReadOnly = _e("translate store could not find or create key, translate store read only")
ErrTranslatingKeyNotFound = _e("translating key not found")

_NAME_RE = re.compile(r"^[a-z][a-z0-9_-]{0,63}$")
_LABEL_RE = re.compile(r"^[A-Za-z][A-Za-z0-9_-]{0,63}$")


def validate_name(name: str) -> None:
    """Index/field name rule (pilosa.go validateName)."""
    if not _NAME_RE.match(name or ""):
        raise ErrName


def validate_label(label: str) -> None:
    if not _LABEL_RE.match(label or ""):
        raise ErrLabel
