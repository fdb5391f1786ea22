"""gRPC transport on grpcio (C-core HTTP/2) with raw-bytes generic handlers.

Messages are never (de)serialised by grpcio: request bytes go straight to
:class:`~.core.ServingCore`, whose hot path is the native codec.  This is the
portable transport; the native HTTP/2 front end (``server/native_transport.py``)
is the fast one.  Both speak the wire protocol the reference's tonic client
uses (plaintext HTTP/2, ``/tensorflow.serving.<Service>/<Method>``).
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
from typing import Optional

import grpc

from ..schema import MODEL_SERVICE, PREDICTION_SERVICE
from . import errors as E
from .core import ServingCore

log = logging.getLogger("tfserve.grpc")

_STATUS = {c.value[0]: c for c in grpc.StatusCode}

MAX_MESSAGE = 2 ** 31 - 1


def grpc_options(max_message: int = MAX_MESSAGE):
    return [("grpc.max_receive_message_length", max_message),
            ("grpc.max_send_message_length", max_message),
            ("grpc.so_reuseport", 1)]


class GrpcTransport:
    def __init__(self, core: ServingCore, port: int, host: str = "0.0.0.0", workers: int = 64,
                 max_message: int = MAX_MESSAGE):
        self.core = core
        self._pool = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="tfs-grpc")
        self.server = grpc.server(self._pool, options=grpc_options(max_message),
                                  maximum_concurrent_rpcs=None)
        handlers = {}
        for path in core.handlers:
            svc, meth = path.strip("/").split("/")
            handlers.setdefault(svc, {})[meth] = grpc.unary_unary_rpc_method_handler(self._make(path))
        for svc, meths in handlers.items():
            self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(svc, meths),))
        self.port = self.server.add_insecure_port(f"{host}:{port}")
        if self.port == 0:
            raise OSError(f"could not bind gRPC port {host}:{port}")

    def _make(self, path):
        core = self.core

        def handler(request: bytes, context: grpc.ServicerContext):
            try:
                return core.handle(path, request)
            except E.ServingError as e:
                context.abort(_STATUS.get(e.code, grpc.StatusCode.UNKNOWN), e.message)
        return handler

    def start(self):
        self.server.start()
        return self

    def stop(self, grace: Optional[float] = 1.0):
        self.server.stop(grace).wait()
        self._pool.shutdown(wait=False)
