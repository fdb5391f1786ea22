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
* Per-stream dispatch: SO_REUSEPORT balances connections only, and the
  reference client multiplexes everything over one or two of them
  (``src/lib.rs:132-138``), so every replica's front end also routes
  individual Predicts to the least-loaded replica through shared-memory rings
  (``csrc/router.h``; group name in ``TFSERVE_ROUTE_GROUP``).
* Fault isolation: :func:`launch` is a supervisor.  It hosts the control
  store itself (no replica's death takes the store down), restarts only a
  replica that died (a fresh child process that reads the models the group
  already holds from disk and applies the group's current config), and bumps
  the weight-broadcast generation (``tfs/gen``): the live replicas and the
  replacement form a new group at the leader's next load, so later loads are
  broadcast on every GPU again (parallel/weights.py).  Config reloads wait
  only for replicas whose heartbeat is fresh.
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

    def __init__(self, store, rank: int, world: int, prefix: str = "tfs/cfg", ack_timeout: float = 900.0,
                 restarted: bool = False, heartbeat_s: float = 0.5, dead_after_s: float = 3.0):
        self.store = store
        self.rank = rank
        self.world = world
        self.prefix = prefix
        self.ack_timeout = ack_timeout
        self.restarted = restarted
        self.heartbeat_s = heartbeat_s
        self.dead_after_s = dead_after_s
        self._manager = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._hb: Optional[threading.Thread] = None
        self.applied = 0

    def attach(self, manager) -> "ReplicaControl":
        self._manager = manager
        self._beat()
        self._hb = threading.Thread(target=self._heartbeat, name="tfs-hb", daemon=True)
        self._hb.start()
        first = 1
        if self.restarted:
            # a replacement replica: the group's newest config supersedes the
            # command-line one it started with (older ones are superseded too)
            cur = int(self.store.add(f"{self.prefix}/seq", 0))
            if cur > 0:
                self._apply(cur)
            first = cur + 1
        self._thread = threading.Thread(target=self._loop, args=(first,), name="tfs-cfg", daemon=True)
        self._thread.start()
        return self

    # ------------------------------------------------------------ liveness
    def _beat(self):
        self.store.set(f"tfs/hb/{self.rank}", repr(time.time()))

    def _heartbeat(self):
        while not self._stop.wait(self.heartbeat_s):
            try:
                self._beat()
            except Exception:            # store unreachable: the supervisor is gone
                return

    def alive(self, rank: int) -> bool:
        key = f"tfs/hb/{rank}"
        if not self.store.check([key]):
            return False
        return time.time() - float(self.store.get(key).decode()) < self.dead_after_s

    def _apply(self, seq: int):
        cfg = serving.ModelServerConfig.FromString(self.store.get(f"{self.prefix}/{seq}"))
        try:
            errs = self._manager.apply_config(cfg, wait=True)
        except E.ServingError as e:
            errs = [e]
        except Exception as e:       # never leave the requester waiting
            errs = [E.internal(f"{type(e).__name__}: {e}")]
        ack = {"code": errs[0].code if errs else 0, "message": "; ".join(e.message for e in errs)}
        self.store.set(f"{self.prefix}/ack/{seq}/{self.rank}", json.dumps(ack))
        self.applied = seq

    def _loop(self, first: int = 1):
        seq = first
        while not self._stop.is_set():
            key = f"{self.prefix}/{seq}"
            if not self.store.check([key]):
                self._stop.wait(0.02)
                continue
            self._apply(seq)
            seq += 1

    def reload(self, cfg) -> List[E.ServingError]:
        """Apply ``cfg`` on every live replica; returns the errors (empty = OK).

        A replica whose heartbeat is stale (dead, or being restarted) is not
        waited for: its replacement applies the newest config when it starts."""
        seq = int(self.store.add(f"{self.prefix}/seq", 1))
        self.store.set(f"{self.prefix}/{seq}", cfg.SerializeToString())
        keys = {r: f"{self.prefix}/ack/{seq}/{r}" for r in range(self.world)}
        # poll, never block in store.wait(): the store client is shared by this
        # process's threads and a blocking wait would stall our own apply loop
        deadline = time.time() + self.ack_timeout
        skipped = set()
        while True:
            waiting = [r for r, k in keys.items() if r not in skipped and not self.store.check([k])]
            if not waiting:
                break
            for r in waiting:
                if r != self.rank and not self.alive(r):
                    skipped.add(r)
                    log.warning("config reload #%d: replica %d is down; its replacement applies it on start",
                                seq, r)
            if time.time() > deadline:
                return [E.ServingError(E.DEADLINE_EXCEEDED,
                                       f"config reload #{seq} was not acknowledged by every live replica")]
            time.sleep(0.01)
        errs = []
        for r, k in keys.items():
            if r in skipped:
                continue
            ack = json.loads(self.store.get(k).decode())
            if ack["code"]:
                errs.append(E.ServingError(ack["code"], f"replica {r}: {ack['message']}"))
        return errs

    def close(self):
        self._stop.set()
        for t in (self._thread, self._hb):
            if t is not None:
                t.join(timeout=5)


def count_gpus() -> int:
    """GPUs visible to this process, counted without touching the HIP runtime
    (the supervisor must never initialise a device): KFD topology nodes with
    SIMDs, narrowed by ROCR/HIP/CUDA_VISIBLE_DEVICES."""
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids)) if n else len(ids)
    return n


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def shm_cleanup(group: str) -> None:
    """Remove a routing group's shared-memory rings and directory."""
    try:
        names = os.listdir("/dev/shm")
    except OSError:
        return
    for n in names:
        if n.startswith(f"tfs_{group}_"):
            try:
                os.unlink(os.path.join("/dev/shm", n))
            except OSError:
                pass


def launch(argv: Sequence[str], nproc: int, module: str = "rust_tensorflow_serving2_amd.server",
           master_addr: str = "127.0.0.1", master_port: int = 0, env: Optional[dict] = None,
           max_restarts: int = 5, restart_backoff_s: float = 1.0) -> int:
    """Supervise ``nproc`` replica processes of ``python -m <module> <argv>``.

    Child ``i`` gets ``RANK=LOCAL_RANK=i``, ``WORLD_SIZE=nproc`` and a common
    ``MASTER_ADDR/PORT`` (the torchrun convention).  The supervisor hosts the
    control store (``TFSERVE_STORE``) so it survives any replica.  A replica
    that exits non-zero (or by a signal) is restarted alone -- up to
    ``max_restarts`` times -- with ``TFSERVE_RESTARTS`` counting its
    incarnations; the others keep serving.  SIGINT/SIGTERM are forwarded and
    end the group; a replica that exits 0 is not restarted.  The supervisor
    never touches the GPU (importing torch for the TCPStore does not; replicas
    are children, never exec'd from a GPU-initialised process).
    """
    from datetime import timedelta
    from torch.distributed import TCPStore
    port = master_port or free_port(master_addr)
    store = TCPStore(master_addr, port, is_master=True, wait_for_workers=False, timeout=timedelta(seconds=60))
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    group = base.setdefault("TFSERVE_ROUTE_GROUP", f"s{os.getpid()}")
    restarts = [0] * nproc
    stopping = []

    def spawn(i: int) -> subprocess.Popen:
        e = dict(base, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR=master_addr, MASTER_PORT=str(port), TFSERVE_STORE=f"{master_addr}:{port}",
                 TFSERVE_RESTARTS=str(restarts[i]), TFSERVE_SUPERVISED="1")
        return subprocess.Popen([sys.executable, "-m", module, *argv], env=e)

    procs: List[Optional[subprocess.Popen]] = [spawn(i) for i in range(nproc)]

    def forward(sig, _frm):
        stopping.append(sig)
        for p in procs:
            if p is not None and p.poll() is None:
                p.send_signal(sig)

    old = {s: signal.signal(s, forward) for s in (signal.SIGINT, signal.SIGTERM)}
    rc = 0
    try:
        while any(p is not None for p in procs):
            for i, p in enumerate(procs):
                if p is None:
                    continue
                r = p.poll()
                if r is None:
                    continue
                procs[i] = None
                if stopping or r == 0:
                    continue
                # the weight-broadcast group lost a member: a new generation, whose
                # group (live ranks + the replacement) forms at the leader's next event
                store.add("tfs/gen", 1)
                # ... and its last heartbeat must not make it look alive for
                # dead_after_s more (the bump comes first: a rank without a
                # heartbeat key counts as alive to the weight source, which
                # gates generation >= 1 on membership instead)
                try:
                    store.delete_key(f"tfs/hb/{i}")
                except Exception:
                    pass
                if restarts[i] >= max_restarts:
                    log.error("replica %d (pid %d) exited with %d; restart budget spent", i, p.pid, r)
                    rc = rc or r
                    continue
                restarts[i] += 1
                log.error("replica %d (pid %d) exited with %d; restarting it (%d/%d), the others keep serving",
                          i, p.pid, r, restarts[i], max_restarts)
                print(f"[tfserve] supervisor: replica {i} exited with {r}; restarting", flush=True)
                time.sleep(restart_backoff_s)
                if not stopping:
                    procs[i] = spawn(i)
            time.sleep(0.2)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
        shm_cleanup(group)
        del store
    return rc
