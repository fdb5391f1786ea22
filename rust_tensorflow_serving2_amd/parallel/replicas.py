"""Data-parallel serving replicas: one server process per GPU.

Topology (MI355X-first, SURVEY.md §2.4 "DP replicas", §7.2 step 6):

* ``N`` processes, one per GPU, started by :func:`launch` (or ``torchrun``).
  Each owns its GPU's servables, HIP streams/graphs and batching lanes; none
  touches another GPU, so there is no cross-process device traffic on the
  request path at all.
* All replicas bind the SAME gRPC (and REST) port with ``SO_REUSEPORT``: the
  kernel spreads incoming connections over the replicas, i.e. the dispatcher
  is the listen-socket hash with zero hops (a client opening many
  connections, like the benchmark load generator or a pool of reference
  clients, is balanced across GPUs).
* Weights are read from disk once (leader) and broadcast over RCCL
  (:mod:`.weights`).
* ``HandleReloadConfigRequest`` arrives on whichever replica owns the
  connection.  :class:`ReplicaControl` publishes the new config to the
  group's key-value store; every replica applies configs in sequence order
  and acknowledges, and the receiving replica answers once all have (so a
  reload returns only when every GPU serves the new config, the semantics of
  ``model_service.proto:19-21`` extended to N replicas).
"""
from __future__ import annotations

import json
import logging
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Sequence

from ..schema import serving
from ..server import errors as E

log = logging.getLogger("tfserve.replicas")


class ReplicaControl:
    """Config replication across replicas through a ``torch.distributed.Store``."""

    def __init__(self, store, rank: int, world: int, prefix: str = "tfs/cfg", ack_timeout: float = 900.0):
        self.store = store
        self.rank = rank
        self.world = world
        self.prefix = prefix
        self.ack_timeout = ack_timeout
        self._manager = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.applied = 0

    def attach(self, manager) -> "ReplicaControl":
        self._manager = manager
        self._thread = threading.Thread(target=self._loop, name="tfs-cfg", daemon=True)
        self._thread.start()
        return self

    def _loop(self):
        seq = 1
        while not self._stop.is_set():
            key = f"{self.prefix}/{seq}"
            if not self.store.check([key]):
                self._stop.wait(0.02)
                continue
            cfg = serving.ModelServerConfig.FromString(self.store.get(key))
            try:
                errs = self._manager.apply_config(cfg, wait=True)
            except E.ServingError as e:
                errs = [e]
            except Exception as e:       # never leave the requester waiting
                errs = [E.internal(f"{type(e).__name__}: {e}")]
            ack = {"code": errs[0].code if errs else 0, "message": "; ".join(e.message for e in errs)}
            self.store.set(f"{self.prefix}/ack/{seq}/{self.rank}", json.dumps(ack))
            self.applied = seq
            seq += 1

    def reload(self, cfg) -> List[E.ServingError]:
        """Apply ``cfg`` on every replica; returns the errors (empty = OK everywhere)."""
        seq = int(self.store.add(f"{self.prefix}/seq", 1))
        self.store.set(f"{self.prefix}/{seq}", cfg.SerializeToString())
        keys = [f"{self.prefix}/ack/{seq}/{r}" for r in range(self.world)]
        # poll, never block in store.wait(): the store client is shared by this
        # process's threads and a blocking wait would stall our own apply loop
        deadline = time.time() + self.ack_timeout
        while not self.store.check(keys):
            if time.time() > deadline:
                return [E.ServingError(E.DEADLINE_EXCEEDED,
                                       f"config reload #{seq} was not acknowledged by every replica")]
            time.sleep(0.01)
        errs = []
        for r, k in enumerate(keys):
            ack = json.loads(self.store.get(k).decode())
            if ack["code"]:
                errs.append(E.ServingError(ack["code"], f"replica {r}: {ack['message']}"))
        return errs

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def launch(argv: Sequence[str], nproc: int, module: str = "rust_tensorflow_serving2_amd.server",
           master_addr: str = "127.0.0.1", master_port: int = 0, env: Optional[dict] = None) -> int:
    """Start ``nproc`` replica processes of ``python -m <module> <argv>`` and wait.

    Child ``i`` gets ``RANK=LOCAL_RANK=i``, ``WORLD_SIZE=nproc`` and a common
    ``MASTER_ADDR/PORT`` (the torchrun convention), so the same entry point
    also works under ``torchrun``.  SIGINT/SIGTERM are forwarded; the first
    replica to exit non-zero stops the others.  The launcher itself never
    touches the GPU (it must not: replicas are started as children, never by
    exec from a GPU-initialised process).
    """
    port = master_port or free_port(master_addr)
    procs: List[subprocess.Popen] = []
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for i in range(nproc):
        e = dict(base, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR=master_addr, MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-m", module, *argv], env=e))

    def forward(sig, _frm):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    old = {s: signal.signal(s, forward) for s in (signal.SIGINT, signal.SIGTERM)}
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    log.error("replica pid %d exited with %d; stopping the others", p.pid, r)
                    forward(signal.SIGTERM, None)
            time.sleep(0.2)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc
