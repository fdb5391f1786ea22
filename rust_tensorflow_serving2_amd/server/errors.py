"""Canonical error space (tensorflow.error.Code == grpc status codes).

The reference surfaces every non-OK gRPC status as ``Box<dyn Error>``
(``src/lib.rs:265,295,310,332``); the server therefore uses canonical codes
(SURVEY.md §2.3): NOT_FOUND for unknown model/version, INVALID_ARGUMENT for bad
input/signature, UNAVAILABLE while loading, FAILED_PRECONDITION for bad reloads.
"""
from __future__ import annotations

OK = 0
CANCELLED = 1
UNKNOWN = 2
INVALID_ARGUMENT = 3
DEADLINE_EXCEEDED = 4
NOT_FOUND = 5
ALREADY_EXISTS = 6
PERMISSION_DENIED = 7
RESOURCE_EXHAUSTED = 8
FAILED_PRECONDITION = 9
ABORTED = 10
OUT_OF_RANGE = 11
UNIMPLEMENTED = 12
INTERNAL = 13
UNAVAILABLE = 14
DATA_LOSS = 15
UNAUTHENTICATED = 16

CODE_NAMES = {v: k for k, v in dict(globals()).items() if isinstance(v, int) and k.isupper()}


class ServingError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
        self.message = message

    def __repr__(self):
        return f"ServingError({CODE_NAMES.get(self.code, self.code)}, {self.message!r})"


def invalid(msg):
    return ServingError(INVALID_ARGUMENT, msg)


def not_found(msg):
    return ServingError(NOT_FOUND, msg)


def unavailable(msg):
    return ServingError(UNAVAILABLE, msg)


def internal(msg):
    return ServingError(INTERNAL, msg)


def failed_precondition(msg):
    return ServingError(FAILED_PRECONDITION, msg)


def unimplemented(msg):
    return ServingError(UNIMPLEMENTED, msg)
