"""Native HTTP/2 gRPC transport (``_C.Http2Server``) + Predict fast path.

* IO threads (C++, epoll, libnghttp2) terminate gRPC; each owns an
  SO_REUSEPORT listener so connections spread over threads and over the
  per-GPU server processes sharing the port.
* Predict calls that match a registered *endpoint* never touch Python per
  request: decoded + validated + copied into a pinned batch slot on the IO
  thread, batched, executed by a GPU lane worker (one HIP-graph replay per
  batch), encoded and answered from C++.
* Every other call (control plane, Classify/Regress, unusual Predicts) is
  queued to Python worker threads that run :class:`~.core.ServingCore`.
"""
from __future__ import annotations

import logging
import os
import threading
from typing import Dict, List, Optional

import numpy as np

from .. import native  # noqa: F401  (loads _C)
from .. import _C
from . import errors as E
from .manager import AVAILABLE, END, UNLOADING
from .servable import PREDICT_METHOD

NATIVE_LANES = os.environ.get("TFSERVE_NATIVE_LANES", "1") != "0"
# CPU servables with batched signatures get the C++ fast path too (Python runs
# once per batch: cpu_runtime.CpuRunner); TFSERVE_CPU_FAST_PATH=0 keeps them on
# the per-request Python path
CPU_FAST_PATH = os.environ.get("TFSERVE_CPU_FAST_PATH", "1") != "0"

log = logging.getLogger("tfserve.native")


class FastEndpoint:
    """A (servable, signature) served by the C++ fast path on the GPU runner's lanes."""

    def __init__(self, transport: "NativeTransport", servable, sig_name: str, timeout_us: int):
        self.t = transport
        self.servable = servable
        self.sig = sig_name
        self._closed = False
        # the lanes replay graphs and read/write pinned buffers the servable
        # owns: hold a reference until close() has joined them, so the
        # manager's unload (which drains references) cannot free them early
        servable.acquire()
        try:
            self._setup(transport, servable, sig_name, timeout_us)
        except BaseException:
            self.close()
            raise

    def _setup(self, transport, servable, sig_name: str, timeout_us: int):
        self.id = -1
        self.workers: List[threading.Thread] = []
        self._stop = threading.Event()
        srv = transport.srv
        sig = servable.signatures[sig_name]
        in_specs = servable.input_specs(sig_name)
        out_specs = servable.output_specs(sig_name)
        in_aliases = sorted(in_specs)
        out_aliases = sorted(out_specs)
        self.runner = servable.runner(sig_name, in_aliases, out_aliases)
        self.max_rows = self.runner.buckets[-1]
        # 4th field: the batch-slot row dtype (bf16 for an fp32 input converted on ingest)
        slot_dt = getattr(self.runner, "slot_dtypes", None) or [in_specs[a].dtype for a in in_aliases]
        ins = [(a, in_specs[a].dtype, list(in_specs[a].shape[1:]), dt) for a, dt in zip(in_aliases, slot_dt)]
        outs = [(a, out_specs[a].dtype, list(out_specs[a].shape[1:])) for a in out_aliases]
        self.id = srv.add_endpoint(servable.name, servable.version, sig_name, ins, outs, self.max_rows, timeout_us)
        srv.set_idle_dispatch(self.id, transport.idle_dispatch)
        lg = transport.request_logs.get(servable.name) if transport.request_logs is not None else None
        if lg is not None:            # logging_config: the lanes sample and submit natively
            srv.set_endpoint_log(self.id, lg.native)
        io_in, io_out = srv.endpoint_io_order(self.id)
        assert list(io_in) == in_aliases and list(io_out) == out_aliases
        lanes = self.runner.fast_lanes()
        for lane_idx in lanes:
            in_ptrs, out_ptrs = self.runner.lane_host_pointers(lane_idx)
            srv.set_slot_buffers(self.id, lane_idx, in_ptrs, out_ptrs)
        self.native_lanes = 0
        slots = 0
        for lane_idx in lanes:
            self.runner.claim(lane_idx)
            # C++ lane worker (graph launch without Python) when every bucket graph
            # carries its own host copies; the Python worker otherwise
            spec = self.runner.native_lane_spec(lane_idx) if NATIVE_LANES else None
            if spec is not None and srv.start_native_lane(self.id, lane_idx, *spec):
                self.native_lanes += 1
                slots += 1
                continue
            slots += 1
            th = threading.Thread(target=self._work, args=(lane_idx,), daemon=True,
                                  name=f"tfs-gpu-{servable.name}-{lane_idx}")
            th.start()
            self.workers.append(th)
        transport.pipeline_rows(self.id, self.max_rows * slots)

    def _work(self, lane_idx: int):
        _C.set_thread_name(f"tfs-lane{lane_idx}")
        srv = self.t.srv
        while not self._stop.is_set():
            n = srv.acquire(self.id, lane_idx, 100)
            if n < 0:
                return
            if n == 0:
                continue
            try:
                if self.servable.fault is not None:
                    self.servable.fault.check()
                self.runner.run_lane(lane_idx, n)
            except Exception as e:  # report to every caller of the batch
                log.exception("fast-path batch failed")
                srv.fail(self.id, lane_idx, E.INTERNAL, f"{type(e).__name__}: {e}")
                continue
            srv.complete(self.id, lane_idx)
            if self.t.metrics is not None:
                self.t.metrics.observe_batch(n, 0.0, str(self.servable.options.device))

    def close(self):
        """Close the endpoint (requests that have not started are answered
        UNAVAILABLE), join its lanes, then drop the servable reference."""
        if self._closed:
            return
        self._closed = True
        self._stop.set()
        try:
            if self.id >= 0:
                self.t.srv.remove_endpoint(self.id)
                self.t.pipeline_rows(self.id, None)
            for th in self.workers:
                th.join(timeout=5)
        finally:
            self.servable.release()


class NativeTransport:
    def __init__(self, core, port: int, host: str = "0.0.0.0", batcher=None, io_threads: int = 4,
                 py_workers: int = 16, fast_path: bool = True, batch_timeout_us: int = 2000,
                 max_message: int = 2 ** 31 - 1, metrics=None, idle_dispatch: bool = True,
                 router: Optional[tuple] = None):
        self.core = core
        self.srv = _C.Http2Server(host, port, io_threads, max_message)
        self.port = self.srv.port
        self._router = router is not None
        self._cap_lock = threading.Lock()
        self._pipe_rows: dict = {}
        if router is not None:
            # (group, rank, world): per-stream routing over shared memory rings
            # (csrc/router.h); sizes from the environment for unusual models
            group, rank, world = router
            self.srv.enable_router(group, int(rank), int(world),
                                   ncells=int(os.environ.get("TFSERVE_ROUTE_CELLS", "64")),
                                   req_cap=int(os.environ.get("TFSERVE_ROUTE_REQ_BYTES", str(1 << 20))),
                                   resp_cap=int(os.environ.get("TFSERVE_ROUTE_RESP_BYTES", str(256 << 10))),
                                   margin=int(os.environ.get("TFSERVE_ROUTE_MARGIN", "8")))
        self.metrics = metrics if metrics is not None else getattr(core, "metrics", None)
        if self.metrics is not None:
            self.metrics.collectors.append(self.prometheus_lines)
        self.fast_path = fast_path
        self.request_logs = getattr(core, "request_logger", None)
        self.idle_dispatch = idle_dispatch
        self.batch_timeout_us = batch_timeout_us
        if batcher is not None:
            self.batch_timeout_us = int(getattr(batcher, "timeout_us", batch_timeout_us))
        self._workers = [threading.Thread(target=self._serve, daemon=True, name=f"tfs-py-{i}")
                         for i in range(py_workers)]
        self._stop = threading.Event()
        self._eps: Dict[tuple, FastEndpoint] = {}
        self._eps_lock = threading.Lock()
        # fast-path registrations run in background threads (graph capture takes
        # a while); a version that starts unloading meanwhile is cancelled, and
        # stop() waits for them so no capture outlives the transport
        self._reg_threads: List[threading.Thread] = []
        self._cancelled: set = set()
        # endpoint teardown (closing + joining lanes) runs off the manager's
        # listener call, which holds the manager lock: only the route removal
        # is synchronous, so resolve() / GetModelStatus never wait on a lane
        self._teardown: List[threading.Thread] = []

    # ------------------------------------------------------------ slow path
    def _serve(self):
        _C.set_thread_name("tfs-py")
        srv, core = self.srv, self.core
        while not self._stop.is_set():
            call = srv.next_call(100)
            if call is None:
                continue
            if call.expired:                      # the client's grpc-timeout already passed
                srv.respond(call, E.DEADLINE_EXCEEDED, "Deadline Exceeded", b"")
                continue
            try:
                body = core.handle(call.method, call.body)
                if call.expired:
                    srv.respond(call, E.DEADLINE_EXCEEDED, "Deadline Exceeded", b"")
                    continue
                srv.respond(call, 0, "", body)
            except E.ServingError as e:
                srv.respond(call, e.code, e.message, b"")
            except Exception as e:  # pragma: no cover - defensive
                srv.respond(call, E.INTERNAL, str(e), b"")

    # ------------------------------------------------------------ fast path wiring
    def _on_state(self, name: str, version: int, state: int):
        if not self.fast_path:
            return
        if state == AVAILABLE:
            with self._eps_lock:
                self._cancelled.discard((name, version))
                self._reg_threads = [t for t in self._reg_threads if t.is_alive()]
                th = threading.Thread(target=self._register, args=(name, version), daemon=True,
                                      name=f"tfs-fastreg-{name}-{version}")
                self._reg_threads.append(th)
            th.start()
        elif state in (UNLOADING, END):
            with self._eps_lock:
                self._cancelled.add((name, version))
            self._unregister(name, version)

    def _reg_cancelled(self, name: str, version: int) -> bool:
        return self._stop.is_set() or (name, version) in self._cancelled

    def _register(self, name: str, version: int):
        mgr = self.core.manager
        try:
            servable = mgr.resolve(name, version)
        except E.ServingError:
            return
        try:
            if not servable.options.is_gpu and not CPU_FAST_PATH:
                return
            for sig_name, sig in servable.signatures.items():
                if sig.method_name != PREDICT_METHOD or self._reg_cancelled(name, version):
                    continue
                ins = servable.input_specs(sig_name)
                if not all(s.shape and s.shape[0] == -1 and all(d >= 0 for d in s.shape[1:]) for s in ins.values()):
                    continue
                outs = servable.output_specs(sig_name)
                if not all(s.shape and s.shape[0] == -1 and all(d >= 0 for d in s.shape[1:]) for s in outs.values()):
                    continue
                if not servable.options.is_gpu and \
                        not hasattr(servable.runner(sig_name, sorted(ins), sorted(outs)), "fast_lanes"):
                    continue      # a CPU signature the batched runner does not take: Python path
                try:
                    ep = FastEndpoint(self, servable, sig_name, self.batch_timeout_us)
                except Exception:
                    log.exception("fast path unavailable for %s/%s", name, sig_name)
                    continue
                with self._eps_lock:
                    cancelled = self._reg_cancelled(name, version)
                    if not cancelled:
                        self._eps[(name, version, sig_name)] = ep
                if cancelled:   # the version began unloading while its graphs were captured
                    ep.close()
                    continue
                self.srv.set_route(name, sig_name, version, ep.id)
                log.info("fast path: %s v%d %s -> endpoint %d", name, version, sig_name, ep.id)
            self._refresh_latest(name)
        finally:
            servable.release()

    def _refresh_latest(self, name: str):
        with self._eps_lock:
            versions = sorted({v for (n, v, _s) in self._eps if n == name})
            sigs = {}
            for (n, v, s), ep in self._eps.items():
                if n == name:
                    sigs.setdefault(s, {})[v] = ep
        latest_avail = max((v for n, v, _ in self.core.manager.available() if n == name), default=None)
        for s, byv in sigs.items():
            if latest_avail is not None and latest_avail in byv:
                self.srv.set_route(name, s, -1, byv[latest_avail].id)
            else:
                self.srv.set_route(name, s, -1, -1)   # latest not fast-pathable: python decides

    def _unregister(self, name: str, version: int):
        with self._eps_lock:
            keys = [k for k in self._eps if k[0] == name and k[1] == version]
            eps = [self._eps.pop(k) for k in keys]
        for k, ep in zip(keys, eps):
            self.srv.set_route(name, k[2], version, -1)
        self._refresh_latest(name)
        if not eps:
            return
        th = threading.Thread(target=lambda: [ep.close() for ep in eps], daemon=True,
                              name=f"tfs-teardown-{name}-{version}")
        with self._eps_lock:
            self._teardown = [t for t in self._teardown if t.is_alive()] + [th]
        th.start()

    def _on_log_config(self, name: str, lg):
        """A model's logging_config changed: its fast-path endpoints follow."""
        with self._eps_lock:
            eps = [ep for (n, _v, _s), ep in self._eps.items() if n == name]
        for ep in eps:
            try:
                self.srv.set_endpoint_log(ep.id, lg.native if lg is not None else None)
            except ValueError:
                pass                  # removed meanwhile

    # ------------------------------------------------------------ lifecycle
    def start(self):
        if self.request_logs is not None:
            self.request_logs.listeners.append(self._on_log_config)
        self.srv.start()
        for w in self._workers:
            w.start()
        mgr = self.core.manager
        mgr.listeners.append(self._on_state)
        for name, version, _s in mgr.available():
            self._register(name, version)
        return self

    def stop(self, grace: Optional[float] = 1.0):
        self._stop.set()
        if self.request_logs is not None and self._on_log_config in self.request_logs.listeners:
            self.request_logs.listeners.remove(self._on_log_config)
        with self._eps_lock:
            regs = list(self._reg_threads)
        for th in regs:   # in-flight registrations see _stop and close what they built
            th.join(timeout=120)
        with self._eps_lock:
            eps = list(self._eps.values())
            self._eps.clear()
            teardown = list(self._teardown)
        for ep in eps:
            ep.close()
        for th in teardown:
            th.join(timeout=60)
        self.srv.stop_router()          # peers see this replica go; its forwarded calls are answered
        self.srv.stop()
        for w in self._workers:
            w.join(timeout=2)
        try:
            self.core.manager.listeners.remove(self._on_state)
        except ValueError:
            pass

    def pipeline_rows(self, ep_id: int, rows: Optional[int]) -> None:
        """A fast endpoint's batch pipeline (lanes x max batch): the router keeps
        calls local until that many are outstanding (TFSERVE_ROUTE_LOCAL_CAP
        overrides; 0 = route on load difference alone)."""
        if not self._router:
            return
        with self._cap_lock:
            if rows is None:
                self._pipe_rows.pop(ep_id, None)
            else:
                self._pipe_rows[ep_id] = rows
            env = os.environ.get("TFSERVE_ROUTE_LOCAL_CAP")
            cap = int(env) if env is not None else max(self._pipe_rows.values(), default=0)
        self.srv.set_router_local_cap(cap)

    def prometheus_lines(self):
        """C++ front-end and fast-path counters in Prometheus text form."""
        st = self.srv.stats()
        out = ["# TYPE tfserve_native_requests_total counter"]
        for k in ("requests", "fast_path", "slow_path", "streamed", "expired", "responses", "errors"):
            out.append(f'tfserve_native_requests_total{{kind="{k}"}} {st.get(k, 0)}')
        out.append("# TYPE tfserve_native_bytes_total counter")
        out.append(f'tfserve_native_bytes_total{{dir="in"}} {st.get("bytes_in", 0)}')
        out.append(f'tfserve_native_bytes_total{{dir="out"}} {st.get("bytes_out", 0)}')
        out.append("# TYPE tfserve_native_io_seconds_total counter")
        for k in ("recv", "h2", "dispatch", "send"):
            out.append(f'tfserve_native_io_seconds_total{{phase="{k}"}} {st.get("io_s_" + k, 0.0):.6f}')
        out.append("# TYPE tfserve_fastpath_batches_total counter")
        with self._eps_lock:
            eps = list(self._eps.items())
        for (name, ver, sig), ep in eps:
            es = self.srv.endpoint_stats(ep.id)
            lab = f'model="{name}",version="{ver}",signature="{sig}"'
            out.append(f"tfserve_fastpath_batches_total{{{lab}}} {es.get('batches', 0)}")
            out.append(f"tfserve_fastpath_rows_total{{{lab}}} {es.get('rows', 0)}")
            out.append(f"tfserve_fastpath_rejected_total{{{lab}}} {es.get('rejected', 0)}")
        return out

    def health_rows(self):
        """(model, version, signature, failed, consecutive_failed, batches,
        dead_lanes) per fast endpoint (polled by server.health.HealthMonitor)."""
        with self._eps_lock:
            eps = list(self._eps.items())
        dead = {}
        for ep_id, _b, _e, is_dead in self.srv.native_lane_stats():
            if is_dead:
                dead[ep_id] = dead.get(ep_id, 0) + 1
        for (name, ver, sig), ep in eps:
            es = self.srv.endpoint_stats(ep.id)
            yield (name, ver, sig, es.get("failed", 0), es.get("consecutive_failed", 0), es.get("batches", 0),
                   dead.get(ep.id, 0))

    def stats(self) -> dict:
        d = dict(self.srv.stats())
        rs = self.srv.router_stats()
        if rs:
            d["router"] = dict(rs)
        with self._eps_lock:
            d["endpoints"] = {f"{k[0]}/v{k[1]}/{k[2]}": self.srv.endpoint_stats(ep.id) for k, ep in self._eps.items()}
        return d
