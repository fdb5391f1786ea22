"""Per-model request logging driven by ``ModelConfig.logging_config``.

``LoggingConfig{log_collector_config{type, filename_prefix}, sampling_config
{sampling_rate}}`` (reference ``logging_config.proto:8-18``,
``log_collector_config.proto:6-12``, ``model_server_config.proto:67``; passed
through by the client at ``examples/model_info.rs:47``).  Sampled requests
are written as ``PredictionLog`` records into one TFRecord file per model and
process (``<prefix>.<pid>.tfrecord``): u64 length, masked crc32c(length),
payload, masked crc32c(payload).

Every record goes through ONE native writer per model (``_C.RequestLog``,
``csrc/request_log.h``): the C++ fast path samples and submits Predicts from
its lane threads (the GPU path never enters Python), the Python slow path
(Classify / Regress / non-fast-pathable Predicts) submits its serialised
records to the same writer.  The writer thread does framing, CRCs and IO.
"""
from __future__ import annotations

import os
import struct
import threading
from typing import Callable, Dict, List, Optional

from .. import native
from ..schema import serving


def _frame(payload: bytes) -> bytes:
    hdr = struct.pack("<Q", len(payload))
    return hdr + struct.pack("<I", native.crc32c_mask(native.crc32c(hdr))) + payload + \
        struct.pack("<I", native.crc32c_mask(native.crc32c(payload)))


class TFRecordWriter:
    """Plain synchronous TFRecord writer (tools and tests; serving uses the native one)."""

    def __init__(self, path: str):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._f = open(path, "ab")
        self._lock = threading.Lock()

    def write(self, payload: bytes):
        rec = _frame(payload)
        with self._lock:
            self._f.write(rec)
            self._f.flush()

    def close(self):
        with self._lock:
            self._f.close()


def read_tfrecords(path: str):
    with open(path, "rb") as f:
        data = f.read()
    off = 0
    while off < len(data):
        if off + 12 > len(data):
            raise IOError("truncated TFRecord header")
        (n,) = struct.unpack_from("<Q", data, off)
        (hc,) = struct.unpack_from("<I", data, off + 8)
        if native.crc32c_mask(native.crc32c(data[off:off + 8])) != hc:
            raise IOError("corrupt TFRecord length")
        if off + 16 + n > len(data):
            raise IOError("truncated TFRecord payload")
        payload = data[off + 12: off + 12 + n]
        (pc,) = struct.unpack_from("<I", data, off + 12 + n)
        if native.crc32c_mask(native.crc32c(payload)) != pc:
            raise IOError("corrupt TFRecord payload")
        yield payload
        off += 16 + n


def _key(cfg) -> tuple:
    return (cfg.log_collector_config.type, cfg.log_collector_config.filename_prefix,
            float(cfg.sampling_config.sampling_rate))


class RequestLogger:
    def __init__(self, model: str, cfg):
        from .. import _C
        self.model = model
        self.rate = float(cfg.sampling_config.sampling_rate)
        prefix = cfg.log_collector_config.filename_prefix or f"/tmp/tfserve_requests_{model}"
        kind = cfg.log_collector_config.type or "tfrecord"
        if kind not in ("tfrecord", "file", "disk"):
            raise ValueError(f"unsupported log collector type {kind!r}")
        self.path = f"{prefix}.{os.getpid()}.tfrecord"
        os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
        self.native = _C.RequestLog(self.path, self.rate)
        self.cfg = cfg
        self.key = _key(cfg)

    def log(self, kind: str, request: bytes, response: bytes):
        if not self.native.sample():
            return
        pl = serving.PredictionLog()
        pl.log_metadata.sampling_config.CopyFrom(self.cfg.sampling_config)
        if kind == "predict":
            pl.predict_log.request.ParseFromString(request)
            pl.predict_log.response.ParseFromString(response)
            pl.log_metadata.model_spec.CopyFrom(pl.predict_log.response.model_spec)
        elif kind == "classify":
            pl.classify_log.request.ParseFromString(request)
            pl.classify_log.response.ParseFromString(response)
            pl.log_metadata.model_spec.CopyFrom(pl.classify_log.response.model_spec)
        elif kind == "regress":
            pl.regress_log.request.ParseFromString(request)
            pl.regress_log.response.ParseFromString(response)
            pl.log_metadata.model_spec.CopyFrom(pl.regress_log.response.model_spec)
        else:
            return
        pl.log_metadata.saved_model_tags.append("serve")
        self.native.submit_record(pl.SerializeToString())

    def flush(self):
        self.native.flush()

    def stats(self) -> dict:
        return self.native.stats()

    def close(self):
        self.native.close()


class RequestLoggerRegistry:
    """model name -> RequestLogger.  ``listeners`` (the native transport) are
    told when a model's logger changes so its fast-path endpoints follow."""

    def __init__(self):
        self._loggers: Dict[str, RequestLogger] = {}
        self._lock = threading.Lock()
        self.listeners: List[Callable[[str, Optional[RequestLogger]], None]] = []

    def configure(self, model: str, cfg) -> Optional[RequestLogger]:
        with self._lock:
            cur = self._loggers.get(model)
            if cur is not None and cur.key == _key(cfg):
                return cur                 # a new version of the model: same file, same writer
            old = self._loggers.pop(model, None)
            lg = RequestLogger(model, cfg) if cfg.sampling_config.sampling_rate > 0 else None
            if lg is not None:
                self._loggers[model] = lg
        for fn in list(self.listeners):
            fn(model, lg)
        if old is not None:
            old.close()                    # drains what the fast path submitted before the switch
        return lg

    def get(self, model: str) -> Optional[RequestLogger]:
        return self._loggers.get(model)

    def log(self, kind: str, model: str, request: bytes, response: bytes):
        lg = self._loggers.get(model)
        if lg is not None:
            lg.log(kind, request, response)

    def flush(self):
        for lg in list(self._loggers.values()):
            lg.flush()

    def close(self):
        with self._lock:
            loggers = list(self._loggers.values())
            self._loggers.clear()
        for lg in loggers:
            lg.close()
