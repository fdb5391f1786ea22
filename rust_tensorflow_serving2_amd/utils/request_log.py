"""Per-model request logging driven by ``ModelConfig.logging_config``.

``LoggingConfig{log_collector_config{type, filename_prefix}, sampling_config
{sampling_rate}}`` (reference ``logging_config.proto:8-18``,
``log_collector_config.proto:6-12``; passed through by the client at
``examples/model_info.rs:47``).  Sampled requests are written as
``PredictionLog`` records into TFRecord files (``<prefix>.<pid>.tfrecord``):
u64 length, masked crc32c(length), payload, masked crc32c(payload).
"""
from __future__ import annotations

import os
import random
import struct
import threading
from typing import Dict, Optional

from .. import native
from ..schema import serving


class TFRecordWriter:
    def __init__(self, path: str):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        self._f = open(path, "ab")
        self._lock = threading.Lock()

    def write(self, payload: bytes):
        hdr = struct.pack("<Q", len(payload))
        rec = hdr + struct.pack("<I", native.crc32c_mask(native.crc32c(hdr))) + payload + \
            struct.pack("<I", native.crc32c_mask(native.crc32c(payload)))
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
        (n,) = struct.unpack_from("<Q", data, off)
        (hc,) = struct.unpack_from("<I", data, off + 8)
        if native.crc32c_mask(native.crc32c(data[off:off + 8])) != hc:
            raise IOError("corrupt TFRecord length")
        payload = data[off + 12: off + 12 + n]
        (pc,) = struct.unpack_from("<I", data, off + 12 + n)
        if native.crc32c_mask(native.crc32c(payload)) != pc:
            raise IOError("corrupt TFRecord payload")
        yield payload
        off += 16 + n


class RequestLogger:
    def __init__(self, model: str, cfg):
        self.model = model
        self.rate = cfg.sampling_config.sampling_rate
        prefix = cfg.log_collector_config.filename_prefix or f"/tmp/tfserve_requests_{model}"
        kind = cfg.log_collector_config.type or "tfrecord"
        if kind not in ("tfrecord", "file", "disk"):
            raise ValueError(f"unsupported log collector type {kind!r}")
        self.writer = TFRecordWriter(f"{prefix}.{os.getpid()}.tfrecord")
        self.cfg = cfg

    def log(self, kind: str, request: bytes, response: bytes):
        if self.rate <= 0 or random.random() >= self.rate:
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
        self.writer.write(pl.SerializeToString())

    def close(self):
        self.writer.close()


class RequestLoggerRegistry:
    def __init__(self):
        self._loggers: Dict[str, RequestLogger] = {}
        self._lock = threading.Lock()

    def configure(self, model: str, cfg) -> Optional[RequestLogger]:
        with self._lock:
            old = self._loggers.pop(model, None)
            if old is not None:
                old.close()
            if cfg.sampling_config.sampling_rate <= 0:
                return None
            lg = RequestLogger(model, cfg)
            self._loggers[model] = lg
            return lg

    def log(self, kind: str, model: str, request: bytes, response: bytes):
        lg = self._loggers.get(model)
        if lg is not None:
            lg.log(kind, request, response)

    def close(self):
        with self._lock:
            for lg in self._loggers.values():
                lg.close()
            self._loggers.clear()
