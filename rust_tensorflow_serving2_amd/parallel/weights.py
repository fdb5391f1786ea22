"""Multi-GPU model loading: read + compile once, broadcast the device blob.

One server process per GPU (``torch.distributed``, backend ``nccl`` == RCCL on
ROCm; ``gloo`` for CPU replicas in tests).  SURVEY.md §5's design: "one
contiguous weight blob per model per GPU, which also serves as the RCCL
broadcast unit".

* **Load** (``load``): the leader reads ``saved_model.pb`` + the TensorBundle
  from disk.  Followers receive only the MetaGraphDef and each variable's
  dtype / shape (a small object broadcast) and build a *meta* bundle: float
  variables are shape-only meta tensors, so a follower never holds the
  weights on its host.
* **Compile** (``share_program``): every replica compiles the same program
  with the same fusion passes.  On the leader that folds BN, casts to bf16 and
  places the weights on its GPU; a follower compiles on shapes only (weights
  become uninitialised device tensors, graph/placement.py).  The leader then
  packs its program's device tensors into ONE contiguous device blob (D2D
  copies; the program is re-pointed at views of it) and broadcasts it
  device-to-device (a single large collective, ring/tree-pipelined by RCCL
  over xGMI: ResNet-50's ~51 MB of bf16 weights); followers bind their
  program's tensors as views into the received blob.  No host round trip, no
  per-rank re-fold.
* **Tile configs** (``publish_tuned`` / ``wait_tuned``): the leader autotunes
  each batch bucket once; its picks go through the control store and the
  followers install them before their own capture, so no rank re-tunes.

Collective ordering.  Each rank's model manager decides *when* to load on its
own (file-system polling, reload RPCs arriving on any rank), but collectives
must be issued in the same order everywhere.  So only the leader initiates:
it publishes ``(seq, kind, ...)`` events to the control store and runs the
collective; every follower has ONE event thread that consumes leader events
strictly in ``seq`` order, joins each collective and parks the result until
the local manager / compiler asks for it.  If a replica dies the supervisor
marks the group broken (``tfs/group_broken``) and every rank loads and
compiles from disk from then on.  The reference has no multi-GPU path at all
(one TF Serving container, ``serving/rundocker.sh:15``).
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from concurrent.futures import Future
from concurrent.futures import TimeoutError as FutureTimeout
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..graph import placement
from ..savedmodel import saved_model as sm
from ..schema import tf
from ..utils import tensors as T

log = logging.getLogger("tfserve.weights")


class MemoryBundle:
    """Bundle-compatible view over variables received from the leader
    (numpy arrays, or shape-only meta tensors for float weights)."""

    def __init__(self, arrays: Dict[str, object], dtypes: Dict[str, int]):
        self._a = arrays
        self._dt = dtypes

    def keys(self):
        return self._a.keys()

    def __contains__(self, k):
        return k in self._a

    def dtype(self, k):
        return self._dt[k]

    def shape(self, k):
        return tuple(self._a[k].shape)

    def __getitem__(self, k):
        return self._a[k]


class LoadError(RuntimeError):
    pass


_META_DT = {T.DT_FLOAT: torch.float32, T.DT_HALF: torch.float16, T.DT_BFLOAT16: torch.bfloat16,
            T.DT_DOUBLE: torch.float64}


def _sync(device: torch.device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def broadcast_meta(path: Optional[str], root: int, group, device: torch.device) -> sm.SavedModelBundle:
    """Collective: the root loads ``path``; followers get a meta bundle (float
    variables shape-only, small non-float ones by value).  A load failure on
    the root is broadcast as an error so followers never wait for it."""
    rank = dist.get_rank(group)
    meta = [None]
    b = None
    if rank == root:
        try:
            b = sm.load(path)
            names = sorted(b.bundle.keys()) if b.bundle is not None else []
            entries, small = [], {}
            for n in names:
                dt = b.bundle.dtype(n)
                entries.append((n, dt, list(b.bundle.shape(n))))
                if dt not in _META_DT:
                    small[n] = np.asarray(b.bundle[n])
            meta[0] = ("ok", b.meta_graph.SerializeToString(), entries, list(b.tags), small)
        except Exception as e:    # propagated to every rank
            meta[0] = ("error", f"{type(e).__name__}: {e}", None, None, None)
    dist.broadcast_object_list(meta, src=root, group=group,
                               device=device if device.type == "cuda" else None)
    status, mg_bytes, entries, tags, small = meta[0]
    if status != "ok":
        raise LoadError(mg_bytes)
    if rank == root:
        return b
    arrays, dtypes = {}, {}
    for n, dt, shape in entries:
        dtypes[n] = dt
        arrays[n] = small[n] if n in small else torch.empty(shape, dtype=_META_DT[dt], device="meta")
    mg = tf.MetaGraphDef.FromString(mg_bytes)
    return sm.SavedModelBundle(path or "", mg, MemoryBundle(arrays, dtypes), tags)


def broadcast_blob(blob: Optional[torch.Tensor], manifest, root: int, group, device: torch.device,
                   stats: Optional[dict] = None) -> Tuple[torch.Tensor, list]:
    """Collective: the root's packed program weights -> every rank's device."""
    rank = dist.get_rank(group)
    meta = [manifest if rank == root else None]
    dist.broadcast_object_list(meta, src=root, group=group, device=device if device.type == "cuda" else None)
    manifest = meta[0]
    if rank != root:
        blob = torch.empty(placement.blob_bytes(manifest), dtype=torch.uint8, device=device)
    _sync(device)
    t0 = time.perf_counter()
    if device.type == "cuda" and dist.get_backend(group) == "gloo":
        host = blob.cpu()                      # gloo rehearsal of the device path: staged through the host
        dist.broadcast(host, src=root, group=group)
        if rank != root:
            blob.copy_(host)
    else:
        dist.broadcast(blob, src=root, group=group)
    _sync(device)
    if stats is not None:
        stats["broadcast_s"] = stats.get("broadcast_s", 0.0) + time.perf_counter() - t0
        stats["broadcast_bytes"] = stats.get("broadcast_bytes", 0) + int(blob.numel())
        stats["programs"] = stats.get("programs", 0) + 1
    return blob, manifest


class ReplicatedWeightSource:
    """Leader-ordered weight replication for every replica (see module doc).

    ``store`` is a ``torch.distributed.Store`` shared by the replicas;
    ``group`` the process group the broadcasts run on (nccl/RCCL for GPUs,
    gloo for CPU replicas)."""

    def __init__(self, store, group=None, device: Optional[torch.device] = None, leader: int = 0,
                 load_timeout: float = 900.0, prefix: str = "tfs/wev", tuned_timeout: float = 600.0,
                 program_timeout: float = 120.0, share: Optional[bool] = None):
        self.store = store
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.leader = leader
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = device
        # GPU replicas share the leader's compiled device weights; CPU replicas
        # (tests, control-plane-only deployments) just read the disk each
        # unless asked to rehearse the protocol (share=True)
        if share is None:
            share = device.type == "cuda" and os.environ.get("TFSERVE_SHARE_WEIGHTS", "1") != "0"
        self.share = bool(share)
        self.load_timeout = load_timeout
        self.tuned_timeout = tuned_timeout
        self.program_timeout = program_timeout
        self.announce_wait_s = float(os.environ.get("TFSERVE_SHARE_WAIT_S", "20"))
        self.prefix = prefix
        self.stats: dict = {}
        self._lock = threading.Lock()           # leader: one collective at a time, seq order
        self._seq = 0
        self._pending: Dict[Tuple, Future] = {}
        self._parked: Dict[Tuple, Tuple[float, object]] = {}
        self._stop = threading.Event()
        self._thread = None
        self._disk: set = set()                  # (name, version) loaded from disk: compiled locally
        if self.rank != leader and self.share:
            self._thread = threading.Thread(target=self._follow, name="tfs-wev", daemon=True)
            self._thread.start()

    @property
    def is_leader(self) -> bool:
        return self.rank == self.leader

    def group_broken(self) -> bool:
        """A replica died (the supervisor says so): the collective can no
        longer complete, every rank loads from disk from now on."""
        try:
            return self.store.check(["tfs/group_broken"])
        except Exception:
            return True

    # ------------------------------------------------------------ events
    def _publish(self, event):
        self._seq += 1
        self.store.set(f"{self.prefix}/{self._seq}", json.dumps(event))

    def _follow(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        seq = 1
        while not self._stop.is_set():
            key = f"{self.prefix}/{seq}"
            if not self.store.check([key]):     # non-blocking poll (lets close() end the thread)
                self._stop.wait(0.02)
                continue
            ev = json.loads(self.store.get(key).decode())
            seq += 1
            try:
                if ev[0] == "load":
                    res = broadcast_meta(None, self.leader, self.group, self.device)
                else:
                    res = broadcast_blob(None, None, self.leader, self.group, self.device, self.stats)
                err = None
            except Exception as e:
                res, err = None, e
            k = tuple(ev[:4]) if ev[0] == "prog" else tuple(ev[:3])
            self._deliver(k, res, err)

    def _deliver(self, k, res, err):
        with self._lock:
            fut = self._pending.pop(k, None)
            if fut is None:
                self._parked[k] = (time.time(), err if err is not None else res)
                self._expire()
        if fut is not None:
            if err is not None:
                fut.set_exception(err)
            else:
                fut.set_result(res)

    def _expire(self, ttl: float = 600.0):
        now = time.time()
        for k in [k for k, (t, _) in self._parked.items() if now - t > ttl]:
            del self._parked[k]

    def _await(self, k, what: str, fallback, timeout: Optional[float] = None, fallback_on_timeout: bool = False):
        """A follower's parked / pending leader result for ``k``."""
        with self._lock:
            parked = self._parked.pop(k, None)
            if parked is None:
                fut = self._pending.get(k)
                if fut is None:
                    fut = self._pending[k] = Future()
        if parked is not None:
            if isinstance(parked[1], Exception):
                raise parked[1]
            return parked[1]
        deadline = time.time() + (self.load_timeout if timeout is None else timeout)
        while True:
            try:
                return fut.result(timeout=0.5)
            except FutureTimeout:
                if self.group_broken() or time.time() > deadline:
                    with self._lock:
                        self._pending.pop(k, None)
                    if self.group_broken() or fallback_on_timeout:   # the leader may be the replica that died
                        return fallback()
                    raise LoadError(f"timed out waiting for the leader rank to broadcast {what}")

    # ------------------------------------------------------------ API: load
    def load(self, name: str, version: int, path: str):
        if not self.share:
            self._disk.add((name, int(version)))
            return sm.load(path)
        if self.group_broken():
            self.stats["disk_loads"] = self.stats.get("disk_loads", 0) + 1
            self._disk.add((name, int(version)))
            return sm.load(path)
        self._disk.discard((name, int(version)))
        if self.is_leader:
            with self._lock:
                self._publish(["load", name, int(version), path])
                return broadcast_meta(path, self.leader, self.group, self.device)

        def disk():
            self._disk.add((name, int(version)))
            return sm.load(path)
        return self._await(("load", name, int(version)), f"{name} version {version}", disk)

    # ------------------------------------------------------------ API: compiled programs
    def share_program(self, name: str, version: int, key: str, program, recompile=None) -> None:
        """After compiling ``program`` for runner ``key`` of (name, version):
        the leader packs + broadcasts its device weights, a follower binds its
        program to the received blob (``recompile()`` builds the program from
        disk instead when the group broke meanwhile; the caller's program is
        then replaced by the return value through ``program.__dict__``)."""
        k = ("prog", name, int(version), key)
        if not self.share or (name, int(version)) in self._disk:
            return                                   # compiled from real weights: nothing to bind
        if self.is_leader:
            if self.group_broken():
                return
            with self._lock:
                self.store.set(self._announce_key(name, version, key), "1")
                self._publish(["prog", name, int(version), key])
                blob, man = placement.export_weights(program)
                broadcast_blob(blob, man, self.leader, self.group, self.device, self.stats)
            return

        def rebuild():
            if recompile is None:
                raise LoadError("the weight-broadcast group broke before this program's weights arrived")
            return ("recompiled", recompile())
        # a runner the leader does not build (one only this replica's traffic
        # asked for) is compiled from disk: wait for the leader to announce it
        # for at most announce_wait_s, then for its weights
        ak = self._announce_key(name, version, key)
        deadline = time.time() + self.announce_wait_s
        while not self.store.check([ak]):
            if time.time() > deadline or self.group_broken():
                with self._lock:
                    self._pending.pop(k, None)
                res = rebuild()
                program.__dict__.update(res[1].__dict__)
                return
            time.sleep(0.02)
        res = self._await(k, f"the compiled weights of {name} version {version}", rebuild,
                          timeout=self.program_timeout, fallback_on_timeout=True)
        if isinstance(res, tuple) and res and res[0] == "recompiled":
            program.__dict__.update(res[1].__dict__)
            return
        blob, man = res
        try:
            n = placement.bind_weights(program, blob, man)
        except ValueError as e:      # the programs differ (should not happen): compile from disk
            log.warning("cannot bind %s v%d %s to the leader's weights (%s); compiling from disk", name, version,
                        key, e)
            if recompile is None:
                raise
            program.__dict__.update(recompile().__dict__)
            return
        self.stats["bound_bytes"] = self.stats.get("bound_bytes", 0) + n

    def _announce_key(self, name: str, version: int, key: str) -> str:
        return f"{self.prefix}/progs/{name}/{int(version)}/{key}"

    def tuned_key(self, name: str, version: int, key: str, bucket: int) -> str:
        return f"{self.prefix}/tuned/{name}/{int(version)}/{key}/{int(bucket)}"

    def publish_tuned(self, name: str, version: int, key: str, bucket: int, table: Dict[str, list]) -> None:
        """Leader: the tile configs its capture of ``bucket`` settled on."""
        if self.share and self.is_leader and not self.group_broken():
            self.store.set(self.tuned_key(name, version, key, bucket), json.dumps(table))

    def wait_tuned(self, name: str, version: int, key: str, bucket: int) -> Optional[Dict[str, list]]:
        """Follower: the leader's tile configs for ``bucket`` (None after the
        timeout or when the group broke: the caller tunes for itself)."""
        if not self.share or self.is_leader or (name, int(version)) in self._disk:
            return None
        sk = self.tuned_key(name, version, key, bucket)
        deadline = time.time() + self.tuned_timeout
        while not self.store.check([sk]):
            if self.group_broken() or time.time() > deadline or self._stop.is_set():
                return None
            time.sleep(0.02)
        return json.loads(self.store.get(sk).decode())

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
