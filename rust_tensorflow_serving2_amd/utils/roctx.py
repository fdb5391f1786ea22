"""roctx ranges for the Python serving path (opt-in: ``TFSERVE_ROCTX=1``).

The C++ native lanes push the same kind of ranges (``csrc/server.cpp``,
``struct Roctx``): under ``rocprofv3 --marker-trace`` each slow-path RPC
(``tfs.rpc <method>``) and each Python-executed batch (``tfs.batch``) shows
up on the host timeline above the kernels it launched.  SURVEY.md §5
"Tracing / profiling".  Disabled (or without the library), :func:`range`
is a shared no-op context manager.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
if os.environ.get("TFSERVE_ROCTX", "0") not in ("", "0"):
    for _name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so"):
        try:
            _lib = ctypes.CDLL(_name, mode=ctypes.RTLD_GLOBAL)
            _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            break
        except (OSError, AttributeError):
            _lib = None

NULL = contextlib.nullcontext()


def enabled() -> bool:
    return _lib is not None


@contextlib.contextmanager
def _range(msg: str):
    _lib.roctxRangePushA(msg.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()


def range(msg: str):  # noqa: A001 - mirrors roctx naming
    return _range(msg) if _lib is not None else NULL
