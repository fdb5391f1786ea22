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
it publishes ``(seq, kind, ..., generation)`` events to the control store and
runs the collective; every follower has ONE event thread that consumes leader
events strictly in ``seq`` order, joins each collective and parks the result
until the local manager / compiler asks for it.

Generations.  The broadcast group is re-formed after a replica restart
instead of being given up: the supervisor bumps ``tfs/gen`` when it restarts a
replica (parallel/replicas.py), and the next event the leader publishes carries
the new generation.  Every live rank -- the replacement included -- then
builds a fresh process group on the store prefix ``tfs/pg/g<gen>`` (a
standalone ``ProcessGroupNCCL`` / ``ProcessGroupGloo``: the dead process is no
member of it) before it joins that event's collective, so later loads are
broadcast again on every GPU.  A replacement skips events of older generations
(their groups ran without it) and reads the models the group loaded before it
existed from disk.

Membership.  A generation's group is used only once every rank has joined it:
each rank writes ``tfs/pg/g<gen>/member/<rank>`` -- the replacement when its
weight source starts (after it has fixed the first event it will consume),
a survivor when its event thread sees the bump.  Until all ``world`` members
are present (or while a heartbeat is stale) the leader loads from disk and
says so in the model's marker, so no rank waits for a collective that could
not complete; heartbeats alone are not enough, because a dead rank's last
heartbeat stays fresh for ``dead_after_s`` after the supervisor's bump.  A
collective that raises drops its group: the leader bumps the generation, so
the next event forms a fresh one.  The reference has no multi-GPU path at all
(one TF Serving container, ``serving/rundocker.sh:15``);
the supersede-on-reload contract this keeps fast on every GPU is
``model_service.proto:19-21``.
"""
from __future__ import annotations

import json
import logging
import os
import pickle
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


class _CommError(RuntimeError):
    """A follower's collective failed (not the leader's load): fall back to disk."""


_META_DT = {T.DT_FLOAT: torch.float32, T.DT_HALF: torch.float16, T.DT_BFLOAT16: torch.bfloat16,
            T.DT_DOUBLE: torch.float64}


def pg_backend(pg, device_type: Optional[str] = None) -> Optional[str]:
    """The backend a process group actually runs ("nccl" = RCCL on ROCm,
    "gloo"), read from the group object itself -- never inferred from the
    device the tensors live on (a gloo rehearsal on GPUs must not report
    itself as RCCL).  A multi-backend group ("cpu:gloo,cuda:nccl", e.g. one
    set up before cli.py, which then skips its own init) runs the backend
    listed for ``device_type`` (parse_backend)."""
    if pg is None:
        return None
    name = None
    try:
        name = str(dist.get_backend(pg))
    except Exception:
        try:
            name = str(pg.name())
        except Exception:
            return None
    return parse_backend(name, device_type)


def parse_backend(name: Optional[str], device_type: Optional[str] = None) -> Optional[str]:
    """"nccl" / "gloo" from a backend string: a plain name as is; a
    "device:backend,..." list -> the entry for ``device_type`` ("cuda" ->
    its entry, else "cpu"), or the only entry when there is one."""
    if name is None:
        return None
    name = name.strip().lower()
    if ":" not in name:
        return name
    pairs = {}
    for part in name.split(","):
        dev, _, be = part.partition(":")
        if be:
            pairs[dev.strip()] = be.strip()
    if device_type in pairs:
        return pairs[device_type]
    if len(set(pairs.values())) == 1:
        return next(iter(pairs.values()))
    return pairs.get("cpu") if device_type is None else None


def pg_size(pg) -> Optional[int]:
    """Ranks in the communicator (from the group object, not the launcher's env)."""
    try:
        return int(pg.size())
    except Exception:
        try:
            return int(dist.get_world_size(pg))
        except Exception:
            return None


class _StreamMark:
    """Stream-ordered completion of a collective on ``device``: an event
    recorded on the current stream (which ``Work.wait()`` has made wait for the
    process group's stream) that only THIS thread's host side waits for.  A
    device-wide ``torch.cuda.synchronize()`` here would also wait for every
    serving lane's in-flight graph replays on the GPU -- a hot reload on a busy
    replica would stall behind all of them."""

    def __init__(self, device: torch.device):
        self.device = device
        self.ev = None
        if device.type == "cuda":
            self.ev = torch.cuda.Event(enable_timing=False)
            self.ev.record(torch.cuda.current_stream(device))

    def wait(self) -> None:
        if self.ev is not None:
            self.ev.synchronize()


def broadcast_meta(path: Optional[str], root: int, comm: "_Comm") -> sm.SavedModelBundle:
    """Collective: the root loads ``path``; followers get a meta bundle (float
    variables shape-only, small non-float ones by value).  A load failure on
    the root is broadcast as an error so followers never wait for it."""
    meta = None
    b = None
    if comm.rank == root:
        try:
            b = sm.load(path)
            names = sorted(b.bundle.keys()) if b.bundle is not None else []
            entries, small = [], {}
            for n in names:
                dt = b.bundle.dtype(n)
                entries.append((n, dt, list(b.bundle.shape(n))))
                if dt not in _META_DT:
                    small[n] = np.asarray(b.bundle[n])
            meta = ("ok", b.meta_graph.SerializeToString(), entries, list(b.tags), small)
        except Exception as e:    # propagated to every rank
            meta = ("error", f"{type(e).__name__}: {e}", None, None, None)
    status, mg_bytes, entries, tags, small = comm.bcast_obj(meta, root)
    if status != "ok":
        raise LoadError(mg_bytes)
    if comm.rank == root:
        return b
    arrays, dtypes = {}, {}
    for n, dt, shape in entries:
        dtypes[n] = dt
        arrays[n] = small[n] if n in small else torch.empty(shape, dtype=_META_DT[dt], device="meta")
    mg = tf.MetaGraphDef.FromString(mg_bytes)
    return sm.SavedModelBundle(path or "", mg, MemoryBundle(arrays, dtypes), tags)


def broadcast_blob(blob: Optional[torch.Tensor], manifest, root: int, comm: "_Comm",
                   stats: Optional[dict] = None) -> Tuple[torch.Tensor, list]:
    """Collective: the root's packed program weights -> every rank's device."""
    manifest = comm.bcast_obj(manifest if comm.rank == root else None, root)
    device = comm.device
    if comm.rank != root:
        blob = torch.empty(placement.blob_bytes(manifest), dtype=torch.uint8, device=device)
    # ordering is stream-based: the root's blob was packed by copies on the
    # current stream, and ProcessGroupNCCL makes its own stream wait for the
    # current one before the collective; no device-wide synchronize
    t0 = time.perf_counter()
    if device.type == "cuda" and comm.backend == "gloo":
        host = blob.cpu()                      # gloo rehearsal of the device path: staged through the host
        comm.bcast_tensor(host, root)
        if comm.rank != root:
            blob.copy_(host)
    else:
        comm.bcast_tensor(blob, root)          # RCCL: device to device over xGMI
    _StreamMark(device).wait()                 # this collective (and the copy) only
    if stats is not None:
        stats["broadcast_s"] = stats.get("broadcast_s", 0.0) + time.perf_counter() - t0
        stats["broadcast_bytes"] = stats.get("broadcast_bytes", 0) + int(blob.numel())
        stats["programs"] = stats.get("programs", 0) + 1
    return blob, manifest


class _Comm:
    """One generation's process group: the whole world, rank numbers as in
    the replica group.  Generation 0 may be the default group
    (``init_process_group``); later ones are standalone groups on a fresh
    store prefix."""

    def __init__(self, pg, rank: int, world: int, backend: str, device: torch.device, gen: int):
        self.pg, self.rank, self.world, self.backend, self.device, self.gen = pg, rank, world, backend, device, gen

    @classmethod
    def form(cls, store, gen: int, rank: int, world: int, backend: str, device: torch.device,
             timeout_s: float) -> "_Comm":
        from datetime import timedelta
        ps = dist.PrefixStore(f"tfs/pg/g{gen}", store)
        if backend == "nccl":
            pg = dist.ProcessGroupNCCL(ps, rank, world, timedelta(seconds=timeout_s))
        else:
            pg = dist.ProcessGroupGloo(ps, rank, world, timedelta(seconds=timeout_s))
        return cls(pg, rank, world, backend, device, gen)

    def _dev(self):
        return self.device if self.backend == "nccl" else torch.device("cpu")

    def bcast_tensor(self, t: torch.Tensor, root: int) -> None:
        opts = dist.BroadcastOptions()
        opts.rootRank = root
        opts.rootTensor = 0
        self.pg.broadcast([t], opts).wait()

    def bcast_obj(self, obj, root: int):
        """Pickled object from ``root`` (our own control messages only: meta
        graphs, shapes, manifests; never a file's bytes)."""
        dev = self._dev()
        if self.rank == root:
            data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
            n = torch.tensor([len(data)], dtype=torch.int64, device=dev)
        else:
            n = torch.zeros(1, dtype=torch.int64, device=dev)
        self.bcast_tensor(n, root)
        size = int(n.item())
        if self.rank == root:
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        else:
            buf = torch.empty(size, dtype=torch.uint8, device=dev)
        self.bcast_tensor(buf, root)
        if self.rank == root:
            return obj
        return pickle.loads(buf.cpu().numpy().tobytes())


GEN_KEY = "tfs/gen"


class ReplicatedWeightSource:
    """Leader-ordered weight replication for every replica (see module doc).

    ``store`` is a ``torch.distributed.Store`` shared by the replicas.  The
    generation-0 group is ``group`` (default: the default process group when
    one is initialised); a replica started after a restart has none and forms
    the group of the current generation with the others at the next event.
    ``rank`` / ``world`` default to the default group's."""

    def __init__(self, store, group=None, device: Optional[torch.device] = None, leader: int = 0,
                 load_timeout: float = 900.0, prefix: str = "tfs/wev", tuned_timeout: float = 600.0,
                 program_timeout: float = 120.0, share: Optional[bool] = None, rank: Optional[int] = None,
                 world: Optional[int] = None, restarted: bool = False, pg_timeout_s: float = 300.0,
                 dead_after_s: float = 3.0, backend: Optional[str] = None):
        self.store = store
        if rank is None or world is None:
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        self.rank = int(rank)
        self.world = int(world)
        self.leader = leader
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = device
        # the backend of the group the collectives really run on: the default
        # group's (or ``group``'s) when one exists -- bench.py's gloo rehearsal
        # on GPUs then stages through the host (broadcast_blob) and re-forms
        # gloo groups in later generations; a restarted replica without a
        # default group uses ``backend`` / TFSERVE_WEIGHT_BACKEND / the device
        pg0 = None
        if dist.is_initialized():
            pg0 = group if group is not None else dist.distributed_c10d._get_default_group()
        self.backend = (parse_backend(backend, device.type) or pg_backend(pg0, device.type)
                        or os.environ.get("TFSERVE_WEIGHT_BACKEND")
                        or ("nccl" if device.type == "cuda" else "gloo"))
        if self.backend not in ("nccl", "gloo"):
            raise ValueError(f"weight replication needs an nccl (RCCL) or gloo group, not {self.backend!r}")
        # GPU replicas share the leader's compiled device weights; CPU replicas
        # (tests, control-plane-only deployments) read the disk each unless
        # asked to rehearse the protocol (share=True / TFSERVE_SHARE_WEIGHTS=1)
        if share is None:
            share = os.environ.get("TFSERVE_SHARE_WEIGHTS", "1" if device.type == "cuda" else "0") != "0"
        self.share = bool(share)
        self.load_timeout = load_timeout
        self.tuned_timeout = tuned_timeout
        self.program_timeout = program_timeout
        self.pg_timeout_s = pg_timeout_s
        self.dead_after_s = dead_after_s
        self.announce_wait_s = float(os.environ.get("TFSERVE_SHARE_WAIT_S", "20"))
        self.prefix = prefix
        self.stats: dict = {"gen": 0, "regroups": 0, "disk_loads": 0, "bcast_loads": 0, "broadcast_bytes": 0,
                            "broadcast_s": 0.0, "programs": 0, "comm_failures": 0}
        self._lock = threading.Lock()           # leader: one collective at a time, seq order
        self._pending: Dict[Tuple, Future] = {}
        self._parked: Dict[Tuple, Tuple[float, object]] = {}
        self._stop = threading.Event()
        self._thread = None
        self._disk: set = set()                  # (name, version) loaded from disk: compiled locally
        self._old_comms: list = []               # superseded groups (never destroyed under a peer's feet)
        # generation this process started in: events of older generations ran
        # in groups it was never part of
        self.min_gen = self._current_gen()
        self.comm: Optional[_Comm] = None
        if not restarted and self.min_gen == 0 and dist.is_initialized():
            pg = group if group is not None else dist.distributed_c10d._get_default_group()
            self.comm = _Comm(pg, self.rank, self.world, self.backend, device, 0)
        # followers consume events from the one after the newest at start-up;
        # fixed BEFORE joining the generation, so every event the leader
        # publishes once it sees this rank as a member is one it consumes
        self._first_seq = int(self.store.add(f"{prefix}/seq", 0)) + 1 if restarted else 1
        self._member_gen = -1
        self._join(self.min_gen)
        if self.rank != leader and self.share:
            self._thread = threading.Thread(target=self._follow, name="tfs-wev", daemon=True)
            self._thread.start()

    @property
    def is_leader(self) -> bool:
        return self.rank == self.leader

    @property
    def gen(self) -> int:
        return self.comm.gen if self.comm is not None else -1

    # ------------------------------------------------------------ generations / liveness
    def _current_gen(self) -> int:
        try:
            return int(self.store.add(GEN_KEY, 0))
        except Exception:
            return -1

    def _alive(self, rank: int) -> bool:
        """Heartbeat of ``rank`` (parallel/replicas.py ReplicaControl); ranks
        without one (no control plane, e.g. the benchmark) count as alive."""
        key = f"tfs/hb/{rank}"
        try:
            if not self.store.check([key]):
                return True
            return time.time() - float(self.store.get(key).decode()) < self.dead_after_s
        except Exception:
            return False

    def _all_alive(self) -> bool:
        return all(self._alive(r) for r in range(self.world) if r != self.rank)

    @staticmethod
    def _member_key(gen: int, rank: int) -> str:
        return f"tfs/pg/g{gen}/member/{rank}"

    def _join(self, gen: int) -> None:
        """Declare this rank a member of generation ``gen``'s group."""
        if gen < 0 or gen <= self._member_gen:
            return
        try:
            self.store.set(self._member_key(gen, self.rank), "1")
            self._member_gen = gen
        except Exception:
            pass

    def _group_ready(self, gen: int) -> bool:
        """Every rank joined generation ``gen`` and every heartbeat is fresh.
        Generation 0 is the group every rank started in (no restart yet)."""
        if gen < 0 or not self._all_alive():
            return False
        if gen == 0:
            return True
        self._join(gen)
        try:
            return all(self.store.check([self._member_key(gen, r)]) for r in range(self.world))
        except Exception:
            return False

    def _comm_failed(self, comm: "_Comm", e: Exception) -> None:
        """A collective on ``comm`` raised: never reuse its group.  The leader
        opens a new generation so the next event forms a fresh one."""
        self.stats["comm_failures"] = self.stats.get("comm_failures", 0) + 1
        log.warning("rank %d: collective of generation %d failed (%s); dropping the group", self.rank, comm.gen, e)
        if self.comm is comm:
            self._old_comms.append(comm)
            self.comm = None
        if self.is_leader:
            try:
                self.store.add(GEN_KEY, 1)
            except Exception:
                pass

    def _ensure_comm(self, gen: int) -> _Comm:
        """The process group of generation ``gen`` (formed on first use: every
        rank of the generation constructs it at the same event)."""
        if self.comm is not None and self.comm.gen == gen:
            return self.comm
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        comm = _Comm.form(self.store, gen, self.rank, self.world, self.backend, self.device, self.pg_timeout_s)
        if self.comm is not None:
            self._old_comms.append(self.comm)
        self.comm = comm
        self.stats["gen"] = gen
        self.stats["regroups"] = self.stats.get("regroups", 0) + 1
        log.info("rank %d: weight-broadcast group of generation %d formed", self.rank, gen)
        return comm

    def group_broken(self) -> bool:
        """(compatibility) the leader is down: waiting for its broadcast is pointless."""
        return not self._alive(self.leader)

    # ------------------------------------------------------------ events
    def _marker_key(self, name: str, version: int) -> str:
        return f"{self.prefix}/loaded/{name}/{int(version)}"

    def _marker(self, name: str, version: int) -> Optional[dict]:
        k = self._marker_key(name, version)
        try:
            if not self.store.check([k]):
                return None
            return json.loads(self.store.get(k).decode())
        except Exception:
            return None

    def _publish(self, event):
        seq = int(self.store.add(f"{self.prefix}/seq", 1))
        self.store.set(f"{self.prefix}/{seq}", json.dumps(event))

    def _follow(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        seq = self._first_seq
        idle = 0
        while not self._stop.is_set():
            key = f"{self.prefix}/{seq}"
            if not self.store.check([key]):     # non-blocking poll (lets close() end the thread)
                idle += 1
                if idle % 5 == 0:                 # a survivor joins a bumped generation
                    self._join(self._current_gen())
                self._stop.wait(0.02)
                continue
            idle = 0
            ev = json.loads(self.store.get(key).decode())
            seq += 1
            gen = int(ev[-1])
            if gen < self.min_gen:
                continue                          # a collective of a group this process never joined
            k = tuple(ev[:4]) if ev[0] == "prog" else tuple(ev[:3])
            comm = None
            try:
                self._join(gen)
                comm = self._ensure_comm(gen)
                if ev[0] == "load":
                    res = broadcast_meta(None, self.leader, comm)
                else:
                    res = broadcast_blob(None, None, self.leader, comm, self.stats)
                err = None
            except LoadError as e:                # the leader's own load failed (broadcast as an error)
                res, err = None, e
            except Exception as e:                # the collective itself: fall back to disk
                if comm is not None:
                    self._comm_failed(comm, e)
                res, err = None, _CommError(str(e))
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

    def _await(self, k, what: str, fallback, timeout: Optional[float] = None, fallback_on_timeout: bool = False,
               disk_marker: Optional[Tuple[str, int]] = None):
        """A follower's parked / pending leader result for ``k``."""
        with self._lock:
            parked = self._parked.pop(k, None)
            if parked is None:
                fut = self._pending.get(k)
                if fut is None:
                    fut = self._pending[k] = Future()
        if parked is not None:
            if isinstance(parked[1], _CommError):
                return fallback(f"the collective failed: {parked[1]}")
            if isinstance(parked[1], Exception):
                raise parked[1]
            return parked[1]
        start = time.time()
        deadline = start + (self.load_timeout if timeout is None else timeout)
        while True:
            try:
                return fut.result(timeout=0.5)
            except _CommError as e:
                return fallback(f"the collective failed: {e}")
            except FutureTimeout:
                leader_down = self.group_broken()
                m = self._marker(*disk_marker) if disk_marker else None
                skipped = m is not None and m.get("mode") == "disk"
                if leader_down or skipped or time.time() > deadline:
                    with self._lock:
                        self._pending.pop(k, None)
                    if leader_down or skipped or fallback_on_timeout:
                        return fallback("leader down" if leader_down else "leader loaded from disk" if skipped
                                        else f"no broadcast within {deadline - start:.0f} s")
                    raise LoadError(f"timed out waiting for the leader rank to broadcast {what}")

    def _disk_load(self, key, path):
        self.stats["disk_loads"] = self.stats.get("disk_loads", 0) + 1
        self._disk.add(key)
        return sm.load(path)

    # ------------------------------------------------------------ API: load
    def load(self, name: str, version: int, path: str):
        key = (name, int(version))
        if not self.share:
            self._disk.add(key)
            return sm.load(path)
        self._disk.discard(key)
        if self.is_leader:
            with self._lock:
                gen = self._current_gen()
                if not self._group_ready(gen):
                    # a replica is down or its replacement has not joined yet:
                    # no collective could complete
                    self.store.set(self._marker_key(name, version), json.dumps({"gen": gen, "mode": "disk"}))
                    return self._disk_load(key, path)
                self.store.set(self._marker_key(name, version), json.dumps({"gen": gen, "mode": "bcast"}))
                # publish first: forming a new generation's group is itself a
                # rendezvous the followers join when they see this event
                self._publish(["load", name, int(version), path, gen])
                comm = None
                try:
                    comm = self._ensure_comm(gen)
                    return broadcast_meta(path, self.leader, comm)
                except LoadError:
                    raise
                except Exception as e:
                    if comm is not None:
                        self._comm_failed(comm, e)
                    self.store.set(self._marker_key(name, version), json.dumps({"gen": gen, "mode": "disk"}))
                    return self._disk_load(key, path)
        m = self._marker(name, version)
        if m is not None and (m.get("mode") == "disk" or int(m.get("gen", 0)) < self.min_gen):
            # the leader broadcast it before this process existed, or not at all
            return self._disk_load(key, path)
        b = self._await(("load", name, int(version)), f"{name} version {version}",
                        lambda why="": self._disk_load(key, path), disk_marker=(name, int(version)))
        if key not in self._disk:
            self.stats["bcast_loads"] = self.stats.get("bcast_loads", 0) + 1
        return b

    # ------------------------------------------------------------ API: compiled programs
    def share_program(self, name: str, version: int, key: str, program, recompile=None) -> None:
        """After compiling ``program`` for runner ``key`` of (name, version):
        the leader packs + broadcasts its device weights, a follower binds its
        program to the received blob (``recompile()`` builds the program from
        disk instead when the leader does not share it; the caller's program
        is then replaced by the return value through ``program.__dict__``)."""
        k = ("prog", name, int(version), key)
        if not self.share or (name, int(version)) in self._disk:
            return                                   # compiled from real weights: nothing to bind
        if self.is_leader:
            with self._lock:
                gen = self._current_gen()
                if not self._group_ready(gen):
                    return
                self.store.set(self._announce_key(name, version, key), "1")
                self._publish(["prog", name, int(version), key, gen])
                comm = None
                try:
                    comm = self._ensure_comm(gen)
                    blob, man = placement.export_weights(program)
                    broadcast_blob(blob, man, self.leader, comm, self.stats)
                except Exception as e:          # followers recompile from disk (they got _CommError)
                    if comm is None:
                        raise
                    self._comm_failed(comm, e)
            return

        def rebuild(why="the collective failed"):
            if recompile is None:
                raise LoadError("the leader did not broadcast this program's weights")
            self._note_recompile(key, why)
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
                res = rebuild("leader down" if self.group_broken() else
                              f"not announced within {self.announce_wait_s:g} s")
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
            self._note_recompile(key, f"manifest mismatch: {e}")
            program.__dict__.update(recompile().__dict__)
            return
        self.stats["bound_bytes"] = self.stats.get("bound_bytes", 0) + n

    def _note_recompile(self, key: str, why: str) -> None:
        """A follower compiled a program from disk instead of binding the
        leader's broadcast (its weights then went host -> device)."""
        log.warning("follower compiles runner %s from disk: %s", key, why)
        with self._lock:
            self.stats["recompiles"] = self.stats.get("recompiles", 0) + 1
            self.stats.setdefault("recompile_reasons", []).append(f"{key}: {why}")

    def _announce_key(self, name: str, version: int, key: str) -> str:
        return f"{self.prefix}/progs/{name}/{int(version)}/{key}"

    def tuned_key(self, name: str, version: int, key: str, bucket: int) -> str:
        return f"{self.prefix}/tuned/{name}/{int(version)}/{key}/{int(bucket)}"

    def publish_tuned(self, name: str, version: int, key: str, bucket: int, table: Dict[str, list]) -> None:
        """Leader: the tile configs its capture of ``bucket`` settled on."""
        if self.share and self.is_leader:
            self.store.set(self.tuned_key(name, version, key, bucket), json.dumps(table))

    def wait_tuned(self, name: str, version: int, key: str, bucket: int) -> Optional[Dict[str, list]]:
        """Follower: the leader's tile configs for ``bucket`` (None after the
        timeout or when the leader is down: the caller tunes for itself)."""
        if not self.share or self.is_leader or (name, int(version)) in self._disk:
            return None
        sk = self.tuned_key(name, version, key, bucket)
        deadline = time.time() + self.tuned_timeout
        while not self.store.check([sk]):
            if self.group_broken() or time.time() > deadline or self._stop.is_set():
                return None
            time.sleep(0.02)
        return json.loads(self.store.get(sk).decode())

    def verify_collective(self) -> dict:
        """Collective (every rank of the current generation calls it at the
        same point, with no load in flight): an all-reduce of ones over the
        weight-replication group.  The sum must equal the group's size; the
        backend and size are read from the group object.  bench.py's ``rccl``
        block reports this, so a run whose "RCCL" was really gloo, or whose
        communicator is smaller than the launch, cannot pass as RCCL."""
        comm = self.comm
        if comm is None:
            comm = self._ensure_comm(max(0, self._current_gen()))
        dev = comm._dev()
        t = torch.ones(1, dtype=torch.float32, device=dev)
        t0 = time.perf_counter()
        comm.pg.allreduce([t]).wait()
        _StreamMark(comm.device if dev.type == "cuda" else torch.device("cpu")).wait()
        out = {"allreduce_sum": float(t.item()), "allreduce_s": round(time.perf_counter() - t0, 6),
               "pg_backend": pg_backend(comm.pg), "pg_size": pg_size(comm.pg),
               "allreduce_device": str(dev)}
        self.stats["verify"] = out
        return out

    def report(self) -> dict:
        """This rank's replication figures (bench.py's ``rccl`` block):
        the backend and size of the group the collectives ran on (read from
        the process-group object), generation, bytes / seconds of device-blob
        broadcast, loads received over the collective vs read from disk, the
        weight bytes this process copied host -> device itself (a follower
        that really bound the leader's blob copies none) and the last
        ``verify_collective`` result."""
        st = dict(self.stats)
        pg = self.comm.pg if self.comm is not None else None
        backend = pg_backend(pg) or self.backend
        world = pg_size(pg) or self.world
        return {"backend": backend, "world": world, "rank": self.rank, "leader": self.is_leader,
                "gen": self.gen, "broadcast_bytes": int(st.get("broadcast_bytes", 0)),
                "broadcast_s": round(float(st.get("broadcast_s", 0.0)), 6),
                "programs": int(st.get("programs", 0)), "bound_bytes": int(st.get("bound_bytes", 0)),
                "bcast_loads": int(st.get("bcast_loads", 0)), "disk_loads": int(st.get("disk_loads", 0)),
                "comm_failures": int(st.get("comm_failures", 0)),
                "recompiles": int(st.get("recompiles", 0)),
                "recompile_reasons": list(st.get("recompile_reasons", []))[:4],
                "weight_h2d_bytes": int(placement.H2D_BYTES),
                "blob_path": ("host-staged" if self.device.type == "cuda" and backend == "gloo" else
                              "device-to-device" if self.device.type == "cuda" else "host"),
                **{k: v for k, v in (st.get("verify") or {}).items()}}

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
