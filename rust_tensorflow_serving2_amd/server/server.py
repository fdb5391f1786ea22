"""Model server assembly: manager + core + transports (+ batching, metrics, logs).

Equivalent of the stock ``tensorflow/serving`` container the reference starts
(``serving/rundocker.sh:15``: gRPC 8500, REST 8501, ``MODEL_NAME=resnet``,
``/models/resnet``), rebuilt MI355X-first: servables run on the local GPU with
fused HIP kernels; one server process per GPU (``parallel/``) shares the
listening port via SO_REUSEPORT.
"""
from __future__ import annotations

import logging
import os
import threading
from dataclasses import dataclass, field
from typing import Optional

from ..schema import serving
from . import errors as E
from .core import ServingCore
from .manager import ModelManager
from .servable import Servable, ServableOptions

log = logging.getLogger("tfserve.server")


@dataclass
class ServerOptions:
    port: int = 8500
    rest_api_port: int = 0                         # 0 = off, -1 = ephemeral
    host: str = "0.0.0.0"
    model_name: str = ""
    model_base_path: str = ""
    model_config: Optional[object] = None          # serving.ModelServerConfig
    device: str = "cpu"
    enable_batching: bool = False
    batching_parameters: Optional[object] = None   # serving.BatchingParameters
    transport: str = "grpc"                        # "grpc" | "native"
    file_system_poll_wait_seconds: float = 1.0
    grpc_workers: int = 64
    io_threads: int = 4                            # native transport epoll threads
    batch_timeout_us: int = 2000                   # native fast-path batch window
    idle_dispatch: bool = True                     # run a partial batch at once when the device idles
    servable: ServableOptions = field(default_factory=ServableOptions)
    monitoring: bool = True
    weight_source: Optional[object] = None         # parallel.weights.ReplicatedWeightSource (N replicas)
    replicas: Optional[object] = None              # parallel.replicas.ReplicaControl (N replicas)
    model_config_file: str = ""                    # text-format ModelServerConfig
    model_config_file_poll_wait_seconds: float = 0.0
    trace_dir: str = ""                            # request/batch timeline (utils/tracing.py)
    health_failure_threshold: int = 8              # consecutive failed batches -> reload (0 = off)
    health_max_recoveries: int = 3                 # reloads per version before quarantine
    router: Optional[tuple] = None                 # (group, rank, world): cross-replica stream routing


class ModelServer:
    def __init__(self, opts: ServerOptions):
        self.opts = opts
        opts.servable.device = opts.device
        self.metrics = None
        if opts.monitoring:
            from ..utils.metrics import Metrics
            self.metrics = Metrics()
        self.batcher = None
        if opts.enable_batching:
            from .batching import BatchingSession
            self.batcher = BatchingSession(opts.batching_parameters, metrics=self.metrics)
        from ..utils.request_log import RequestLoggerRegistry
        self.request_logs = RequestLoggerRegistry()
        self.manager = ModelManager(self._load, poll_wait_seconds=opts.file_system_poll_wait_seconds)
        self.core = ServingCore(self.manager, self.batcher, self.request_logs, self.metrics)
        self.core.replicas = opts.replicas
        self.tracer = None
        if opts.trace_dir:
            from ..utils.tracing import Tracer
            self.tracer = Tracer(opts.trace_dir)
            self.core.tracer = self.tracer
        self.health = None
        if opts.health_failure_threshold > 0:
            from .health import HealthMonitor
            self.health = HealthMonitor(self.manager, opts.health_failure_threshold, opts.health_max_recoveries,
                                        metrics=self.metrics)
            self.core.health = self.health
        self.transports = []
        self._cfg_thread = None
        self._cfg_stop = threading.Event()
        self._cfg_text = None

    def _load(self, name: str, version: int, path: str, cfg) -> Servable:
        so = self.opts.servable
        if self.batcher is not None:
            so.max_batch_size = self.batcher.max_batch_size
            so.allowed_batch_sizes = tuple(self.batcher.allowed_batch_sizes)
        bundle = None
        if self.opts.weight_source is not None:
            bundle = self.opts.weight_source.load(name, version, path)
        s = Servable(name, version, path, so, bundle, weight_source=self.opts.weight_source)
        s.warmup()
        if cfg is not None and cfg.HasField("logging_config"):
            self.request_logs.configure(name, cfg.logging_config)
        return s

    def _read_config_file(self):
        from google.protobuf import text_format
        with open(self.opts.model_config_file) as f:
            text = f.read()
        cfg = serving.ModelServerConfig()
        try:
            text_format.Parse(text, cfg)
        except text_format.ParseError as e:
            raise E.invalid(f"could not parse --model_config_file {self.opts.model_config_file}: {e}") from None
        return text, cfg

    def _poll_config_file(self):
        """TF Serving's --model_config_file_poll_wait_seconds: re-apply the file when it changes."""
        while not self._cfg_stop.wait(self.opts.model_config_file_poll_wait_seconds):
            try:
                text, cfg = self._read_config_file()
            except (OSError, E.ServingError) as e:
                log.error("model config file poll: %s", e)
                continue
            if text != self._cfg_text:
                self._cfg_text = text
                log.info("model config file changed; applying")
                for err in self.manager.apply_config(cfg, wait=True):
                    log.error("model load error: %s", err.message)

    def initial_config(self):
        o = self.opts
        if o.model_config is not None:
            return o.model_config
        if o.model_config_file:
            self._cfg_text, cfg = self._read_config_file()
            return cfg
        cfg = serving.ModelServerConfig()
        if o.model_base_path:
            mc = cfg.model_config_list.config.add()
            mc.name = o.model_name or "default"
            mc.base_path = o.model_base_path
            mc.model_platform = "tensorflow"
        return cfg

    def start(self, wait_for_models: bool = True):
        cfg = self.initial_config()
        if cfg.WhichOneof("config"):
            errs = self.manager.apply_config(cfg, wait=wait_for_models)
            for e in errs:
                log.error("model load error: %s", e.message)
        self.manager.start_polling()
        if self.opts.replicas is not None:
            self.opts.replicas.attach(self.manager)
        if self.opts.model_config_file and self.opts.model_config_file_poll_wait_seconds > 0:
            self._cfg_thread = threading.Thread(target=self._poll_config_file, name="tfs-cfgfile", daemon=True)
            self._cfg_thread.start()
        if self.opts.transport == "native":
            from .native_transport import NativeTransport
            t = NativeTransport(self.core, self.opts.port, self.opts.host, batcher=self.batcher,
                                io_threads=self.opts.io_threads, batch_timeout_us=self.opts.batch_timeout_us,
                                idle_dispatch=self.opts.idle_dispatch, router=self.opts.router)
        else:
            from .grpc_transport import GrpcTransport
            t = GrpcTransport(self.core, self.opts.port, self.opts.host, self.opts.grpc_workers)
        self.transports.append(t.start())
        self.port = t.port
        if self.health is not None and hasattr(t, "health_rows"):
            self.health.add_source(t.health_rows)
        if self.tracer is not None and self.opts.transport == "native":
            self.tracer.attach_native(t.srv)
        if self.opts.rest_api_port:
            from .rest import RestTransport
            # 0 = disabled (TF Serving convention); -1 = any free port (tests)
            r = RestTransport(self.core, max(0, self.opts.rest_api_port), self.opts.host, self.metrics)
            self.transports.append(r.start())
            self.rest_port = r.port
        log.info("serving on port %d", self.port)
        return self

    def stop(self):
        self._cfg_stop.set()
        if self.opts.replicas is not None:
            self.opts.replicas.close()
        if self.opts.weight_source is not None and hasattr(self.opts.weight_source, "close"):
            self.opts.weight_source.close()
        for t in self.transports:
            t.stop()
        self.transports.clear()
        if self.health is not None:
            self.health.close()
        if self.batcher is not None:
            self.batcher.stop()
        self.manager.stop()
        self.request_logs.close()
        if self.tracer is not None:
            self.tracer.close()
