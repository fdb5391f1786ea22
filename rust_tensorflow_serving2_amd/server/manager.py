"""Model manager: config, version policy, lifecycle state machine, hot reload.

Implements the server side of the reference's control plane:

* ``ModelServerConfig`` / ``ModelConfig`` (``model_server_config.proto:19-84``):
  name, base_path, model_platform, ``model_version_policy`` (latest{N} default
  N=1 / all / specific, ``file_system_storage_path_source.proto:8-37``),
  ``version_labels``, ``logging_config``;
* version lifecycle START -> LOADING -> AVAILABLE -> UNLOADING -> END with a
  ``StatusProto`` per version (``get_model_status.proto:26-60``); a failed load
  ends in END + error while other versions keep serving;
* ``HandleReloadConfigRequest`` semantics: the new config *supersedes* the old
  one — omitted models are unloaded (``model_service.proto:19-21``, the reason
  ``examples/model_info.rs:41-42`` saw its model vanish);
* file-system polling for new versions (``file_system_poll_wait_seconds``),
  availability-preserving transitions (new version AVAILABLE before the old
  one UNLOADs), and refcounted servables so in-flight requests finish before
  an unload frees device memory.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from ..schema import serving
from . import errors as E

log = logging.getLogger("tfserve.manager")

START, LOADING, AVAILABLE, UNLOADING, END = 10, 20, 30, 40, 50
STATE_NAMES = {0: "UNKNOWN", START: "START", LOADING: "LOADING", AVAILABLE: "AVAILABLE",
               UNLOADING: "UNLOADING", END: "END"}


@dataclass
class VersionState:
    version: int
    state: int = START
    error_code: int = E.OK
    error_message: str = ""
    servable: object = None
    path: str = ""
    recover: bool = False               # unloading because unhealthy: load again once END
    quarantined: bool = False           # unhealthy too often: not reloaded until a config asks


@dataclass
class ModelEntry:
    config: object                      # serving.ModelConfig
    versions: Dict[int, VersionState] = field(default_factory=dict)
    error: Optional[E.ServingError] = None
    removed: bool = False


def list_versions(base_path: str) -> Dict[int, str]:
    out = {}
    try:
        names = os.listdir(base_path)
    except OSError:
        return out
    for n in names:
        if n.isdigit():
            p = os.path.join(base_path, n)
            if os.path.isdir(p):
                out[int(n)] = p
    return out


def aspired_versions(cfg, available: Dict[int, str]) -> List[int]:
    pol = cfg.model_version_policy
    kind = pol.WhichOneof("policy_choice")
    vs = sorted(available)
    if kind == "all":
        return vs
    if kind == "specific":
        return sorted(v for v in pol.specific.versions if v in available)
    n = pol.latest.num_versions if kind == "latest" and pol.latest.num_versions > 0 else 1
    return vs[-n:]


Loader = Callable[[str, int, str, object], object]   # (name, version, path, ModelConfig) -> servable


class ModelManager:
    def __init__(self, loader: Loader, load_threads: int = 4, poll_wait_seconds: float = 1.0,
                 unload_timeout: float = 30.0):
        self._loader = loader
        self._models: Dict[str, ModelEntry] = {}
        self._lock = threading.RLock()
        self._cv = threading.Condition(self._lock)
        self._pool = cf.ThreadPoolExecutor(max_workers=load_threads, thread_name_prefix="tfs-load")
        self.poll_wait_seconds = poll_wait_seconds
        self.unload_timeout = unload_timeout
        self._poller: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.listeners: List[Callable[[str, int, int], None]] = []   # (model, version, state)
        # called with each model name an explicit config (apply_config) lists
        self.config_listeners: List[Callable[[str], None]] = []

    # ------------------------------------------------------------ config
    def config(self):
        cfg = serving.ModelServerConfig()
        with self._lock:
            for e in self._models.values():
                if not e.removed:
                    cfg.model_config_list.config.add().CopyFrom(e.config)
        return cfg

    def model_config(self, name: str):
        with self._lock:
            e = self._models.get(name)
            return None if e is None or e.removed else e.config

    @staticmethod
    def validate_config(server_config) -> Dict[str, object]:
        """Check a ModelServerConfig; returns {name: ModelConfig} (raises INVALID_ARGUMENT)."""
        kind = server_config.WhichOneof("config")
        if kind != "model_config_list":
            raise E.invalid("ModelServerConfig: only model_config_list is supported "
                            f"(got {kind or 'empty config'})")
        new = {}
        for mc in server_config.model_config_list.config:
            if not mc.name:
                raise E.invalid("ModelConfig.name must be set")
            if mc.name in new:
                raise E.invalid(f"Illegal to list model {mc.name} multiple times in config list")
            if not mc.base_path:
                raise E.invalid(f"ModelConfig {mc.name}: base_path must be set")
            if mc.model_platform and mc.model_platform not in ("tensorflow", "tf", "savedmodel"):
                raise E.invalid(f"ModelConfig {mc.name}: unsupported model_platform {mc.model_platform!r}")
            new[mc.name] = mc
        return new

    def apply_config(self, server_config, wait: bool = True, timeout: float = 600.0) -> List[E.ServingError]:
        """Make the running set match ``server_config`` (supersedes previous config)."""
        new = self.validate_config(server_config)
        with self._lock:
            for name, entry in self._models.items():
                if name not in new and not entry.removed:
                    entry.removed = True
                    for vs in entry.versions.values():
                        self._begin_unload(name, vs)
            for name, mc in new.items():
                entry = self._models.get(name)
                if entry is None or entry.removed:
                    entry = ModelEntry(config=mc)
                    self._models[name] = entry
                else:
                    if entry.config.base_path != mc.base_path:
                        # different model location: unload everything loaded from the old path
                        for vs in entry.versions.values():
                            self._begin_unload(name, vs)
                        entry.versions = {v: s for v, s in entry.versions.items() if s.state != END}
                    entry.config = mc
                    for vs in entry.versions.values():     # an explicit config lifts quarantine
                        vs.quarantined = False
                self._reconcile(name, entry)
        for name in new:
            for cb in list(self.config_listeners):
                try:
                    cb(name)
                except Exception:
                    log.exception("config listener failed")
        if wait:
            return self.wait_until_settled(list(new), timeout)
        return []

    # ------------------------------------------------------------ reconciliation
    def _reconcile(self, name: str, entry: ModelEntry) -> None:
        cfg = entry.config
        avail = list_versions(cfg.base_path)
        if not avail:
            if not os.path.isdir(cfg.base_path):
                entry.error = E.not_found(f"Could not find base path {cfg.base_path} for servable {name}")
            else:
                entry.error = E.not_found(f"No versions of servable {name} found under base path {cfg.base_path}")
        else:
            entry.error = None
        aspired = set(aspired_versions(cfg, avail))
        for v in sorted(aspired):
            vs = entry.versions.get(v)
            if vs is None or (vs.state == END and not vs.quarantined):
                vs = VersionState(version=v, state=START, path=avail[v])
                entry.versions[v] = vs
                self._notify(name, v, START)
                self._pool.submit(self._load, name, vs)
        # availability preserving: unload non-aspired versions only once an
        # aspired version is serving (or nothing aspired can ever serve)
        aspired_up = any(entry.versions[v].state == AVAILABLE for v in aspired if v in entry.versions)
        aspired_pending = any(entry.versions[v].state in (START, LOADING) for v in aspired if v in entry.versions)
        for v, vs in list(entry.versions.items()):
            if v in aspired or vs.state in (UNLOADING, END):
                continue
            if aspired_up or not aspired_pending:
                self._begin_unload(name, vs)

    def _load(self, name: str, vs: VersionState) -> None:
        with self._lock:
            entry = self._models.get(name)
            if entry is None or vs.state != START:
                return
            vs.state = LOADING
            cfg = entry.config
        self._notify(name, vs.version, LOADING)
        try:
            servable = self._loader(name, vs.version, vs.path, cfg)
        except Exception as e:  # load failure -> END with error, others keep serving
            code = e.code if isinstance(e, E.ServingError) else E.UNKNOWN
            log.error("failed to load %s version %d: %s", name, vs.version, e)
            with self._cv:
                vs.state = END
                vs.error_code = code
                vs.error_message = str(e)
                self._cv.notify_all()
            self._notify(name, vs.version, END)
            return
        with self._cv:
            entry = self._models.get(name)
            if entry is None or entry.removed or vs.state != LOADING:
                unload_now = True
            else:
                unload_now = False
                vs.servable = servable
                vs.state = AVAILABLE
            self._cv.notify_all()
        if unload_now:
            _safe_unload(servable)
            return
        log.info("model %s version %d AVAILABLE", name, vs.version)
        self._notify(name, vs.version, AVAILABLE)
        with self._lock:
            entry = self._models.get(name)
            if entry is not None and not entry.removed:
                self._reconcile_unloads_only(name, entry)

    def _reconcile_unloads_only(self, name: str, entry: ModelEntry) -> None:
        avail = list_versions(entry.config.base_path)
        aspired = set(aspired_versions(entry.config, avail))
        if any(entry.versions[v].state == AVAILABLE for v in aspired if v in entry.versions):
            for v, vs in list(entry.versions.items()):
                if v not in aspired and vs.state == AVAILABLE:
                    self._begin_unload(name, vs)

    def _begin_unload(self, name: str, vs: VersionState) -> None:
        if vs.state in (START, LOADING):
            vs.state = END       # loader sees the change and drops the result
            self._cv.notify_all()
            return
        if vs.state != AVAILABLE:
            return
        vs.state = UNLOADING
        servable = vs.servable
        self._notify(name, vs.version, UNLOADING)

        def work():
            if servable is not None and hasattr(servable, "drain"):
                servable.drain(self.unload_timeout)
            _safe_unload(servable)
            with self._cv:
                vs.servable = None
                vs.state = END
                self._cv.notify_all()
            self._notify(name, vs.version, END)
            log.info("model %s version %d unloaded", name, vs.version)
            if vs.recover:
                with self._lock:
                    entry = self._models.get(name)
                    if entry is not None and not entry.removed:
                        self._reconcile(name, entry)     # still aspired -> loaded again
        self._pool.submit(work)

    # ------------------------------------------------------------ health
    def recover(self, name: str, version: int, why: str, quarantine: bool = False) -> bool:
        """Take an AVAILABLE version that keeps failing down and (unless
        ``quarantine``) load it again from disk (server/health.py).  Other
        versions keep serving; returns False if the version was not AVAILABLE."""
        with self._cv:
            entry = self._models.get(name)
            vs = entry.versions.get(version) if entry is not None else None
            if vs is None or entry.removed or vs.state != AVAILABLE:
                return False
            vs.recover = not quarantine
            vs.quarantined = quarantine
            vs.error_code = E.UNAVAILABLE
            vs.error_message = ("quarantined after repeated device failures: " if quarantine else
                                "unhealthy, reloading: ") + why
            self._begin_unload(name, vs)
            return True

    def _notify(self, name, version, state):
        for cb in list(self.listeners):
            try:
                cb(name, version, state)
            except Exception:  # listeners must never break the state machine
                log.exception("state listener failed")

    def wait_until_settled(self, names: List[str], timeout: float) -> List[E.ServingError]:
        deadline = time.time() + timeout
        with self._cv:
            while True:
                busy = False
                for n in names:
                    e = self._models.get(n)
                    if e is None:
                        continue
                    if any(vs.state in (START, LOADING) for vs in e.versions.values()):
                        busy = True
                if not busy:
                    break
                left = deadline - time.time()
                if left <= 0:
                    return [E.ServingError(E.DEADLINE_EXCEEDED, "timed out waiting for models to load")]
                self._cv.wait(min(left, 0.5))
            errs = []
            for n in names:
                e = self._models.get(n)
                if e is None:
                    continue
                if e.error is not None:
                    errs.append(e.error)
                for vs in e.versions.values():
                    if vs.state == END and vs.error_code != E.OK:
                        errs.append(E.ServingError(vs.error_code, vs.error_message))
            return errs

    # ------------------------------------------------------------ polling
    def poll_once(self) -> None:
        with self._lock:
            for name, entry in list(self._models.items()):
                if not entry.removed:
                    self._reconcile(name, entry)

    def start_polling(self) -> None:
        if self._poller is not None or self.poll_wait_seconds <= 0:
            return

        def loop():
            while not self._stop.wait(self.poll_wait_seconds):
                try:
                    self.poll_once()
                except Exception:
                    log.exception("file system poll failed")
        self._poller = threading.Thread(target=loop, name="tfs-fs-poll", daemon=True)
        self._poller.start()

    def stop(self) -> None:
        self._stop.set()
        with self._lock:
            for name, entry in self._models.items():
                entry.removed = True
                for vs in entry.versions.values():
                    self._begin_unload(name, vs)
        self._pool.shutdown(wait=True)

    # ------------------------------------------------------------ queries
    def resolve(self, name: str, version: Optional[int] = None, label: Optional[str] = None):
        """-> AVAILABLE servable for the request's ModelSpec (acquired: caller must release)."""
        if not name:
            raise E.invalid("Missing ModelSpec name")
        with self._lock:
            entry = self._models.get(name)
            if entry is None or entry.removed:
                raise E.not_found(f"Servable not found for request: Latest({name})" if version is None and
                                  label is None else f"Servable not found for request: "
                                  f"Specific({name}, {version if version is not None else label})")
            if label is not None:
                labels = dict(entry.config.version_labels)
                if label not in labels:
                    raise E.invalid(f"Unrecognized servable version label: {label}")
                version = labels[label]
            if version is not None:
                vs = entry.versions.get(version)
                if vs is None or vs.state != AVAILABLE:
                    if vs is not None and vs.state in (START, LOADING):
                        raise E.unavailable(f"Servable {name} version {version} is still loading")
                    raise E.not_found(f"Servable not found for request: Specific({name}, {version})")
            else:
                live = [v for v, vs in entry.versions.items() if vs.state == AVAILABLE]
                if not live:
                    if any(vs.state in (START, LOADING) for vs in entry.versions.values()):
                        raise E.unavailable(f"Servable {name} is still loading")
                    raise E.not_found(f"Servable not found for request: Latest({name})")
                vs = entry.versions[max(live)]
            s = vs.servable
            if hasattr(s, "acquire"):
                s.acquire()
            return s

    def status(self, name: str, version: Optional[int] = None) -> List[VersionState]:
        if not name:
            raise E.invalid("Missing model name in ModelSpec")
        with self._lock:
            entry = self._models.get(name)
            if entry is None or (entry.removed and not entry.versions):
                raise E.not_found(f"Could not find any versions of model {name}")
            if version is not None:
                vs = entry.versions.get(version)
                if vs is None:
                    raise E.not_found(f"Could not find version {version} of model {name}")
                return [VersionState(vs.version, vs.state, vs.error_code, vs.error_message)]
            if not entry.versions:
                raise E.not_found(f"Could not find any versions of model {name}")
            return [VersionState(v.version, v.state, v.error_code, v.error_message)
                    for _k, v in sorted(entry.versions.items())]

    def available(self) -> List[Tuple[str, int, object]]:
        with self._lock:
            return [(n, v, vs.servable) for n, e in self._models.items() if not e.removed
                    for v, vs in e.versions.items() if vs.state == AVAILABLE]


def _safe_unload(servable):
    try:
        if servable is not None and hasattr(servable, "unload"):
            servable.unload()
    except Exception:
        log.exception("unload failed")
