"""Host topology for one-process-per-GPU serving: which CPUs sit next to which GPU.

Every replica's data plane (HTTP/2 IO threads, the batcher, the native lanes
and -- in the benchmark -- the load generator) moves ~602 KB per request
through host memory (socket buffer -> pinned batch slot -> SDMA).  On a
two-socket 8-GPU node a replica whose threads and pinned slots land on the far
socket pays every one of those bytes across the socket link, so each rank is
pinned to CPUs of its own GPU's NUMA node ("the data plane next
to its GPU"; the reference runs one container, ``serving/rundocker.sh:15``).

Nothing here touches the HIP runtime (the launcher and the supervisor must
never initialise a device).  Sources, all sysfs:

* ``/sys/class/kfd/kfd/topology/nodes/*/properties``: GPU agents in HIP device
  order (nodes with ``simd_count > 0`` sorted by node id, narrowed by
  ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES``), their PCI
  ``location_id`` (bus << 8 | dev << 3 | fn) and ``domain``;
* ``/sys/bus/pci/devices/<bdf>/numa_node`` (falls back to the KFD io-link to a
  CPU node when the firmware reports -1);
* ``/sys/devices/system/node/node*/cpulist``;
* ``/sys/bus/pci/devices/<bdf>/gpu_busy_percent`` for the busy sampler.

``root`` re-bases every path (tests build a fake sysfs tree).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass
class GpuInfo:
    index: int                 # HIP device index in this process
    kfd_node: int
    bdf: str                   # PCI address "dddd:bb:dd.f" ("" if unknown)
    numa_node: int             # -1 if unknown


@dataclass
class Placement:
    rank: int
    gpu: int
    numa_node: int
    cpus: List[int] = field(default_factory=list)

    def as_dict(self) -> dict:
        return {"rank": self.rank, "gpu": self.gpu, "numa_node": self.numa_node, "cpus": compress(self.cpus)}


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str) -> List[int]:
    """"0-3,8,10-11" -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def compress(cpus: Sequence[int]) -> str:
    """[0, 1, 2, 3, 8] -> "0-3,8"."""
    cpus = sorted(set(cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def _props(path: str) -> Dict[str, str]:
    txt = _read(path)
    if txt is None:
        return {}
    out = {}
    for line in txt.splitlines():
        f = line.split()
        if len(f) >= 2:
            out[f[0]] = f[1]
    return out


def _visible(n: int) -> List[int]:
    """Indices (into the KFD GPU list) this process sees, in HIP order."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if not v or not v.strip():      # unset or empty: no narrowing
            continue
        try:
            sel = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:          # UUID form: keep the order we have
            continue
        idx = [idx[i] for i in sel if 0 <= i < len(idx)]
    return idx


def gpus(root: str = "/") -> List[GpuInfo]:
    """Visible GPUs in HIP device order (empty when there is no KFD)."""
    base = os.path.join(root, "sys/class/kfd/kfd/topology/nodes")
    try:
        nodes = sorted(int(x) for x in os.listdir(base) if x.isdigit())
    except OSError:
        return []
    gpu_nodes, cpu_nodes = [], []
    for nd in nodes:
        p = _props(os.path.join(base, str(nd), "properties"))
        if int(p.get("simd_count", "0")) > 0:
            gpu_nodes.append((nd, p))
        elif int(p.get("cpu_cores_count", "0")) > 0:
            cpu_nodes.append(nd)
    out = []
    for i, k in enumerate(_visible(len(gpu_nodes))):
        nd, p = gpu_nodes[k]
        loc = int(p.get("location_id", "0"))
        dom = int(p.get("domain", "0"))
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7:x}" if loc else ""
        numa = -1
        if bdf:
            v = _read(os.path.join(root, "sys/bus/pci/devices", bdf, "numa_node"))
            if v is not None and v.lstrip("-").isdigit():
                numa = int(v)
        if numa < 0:
            # KFD io-link from the GPU to its CPU node (CPU KFD nodes are the
            # NUMA nodes, in order)
            lbase = os.path.join(base, str(nd), "io_links")
            try:
                for ln in sorted(os.listdir(lbase)):
                    to = int(_props(os.path.join(lbase, ln, "properties")).get("node_to", "-1"))
                    if to in cpu_nodes:
                        numa = cpu_nodes.index(to)
                        break
            except OSError:
                pass
        out.append(GpuInfo(index=i, kfd_node=nd, bdf=bdf, numa_node=numa))
    return out


def numa_cpus(root: str = "/") -> Dict[int, List[int]]:
    base = os.path.join(root, "sys/devices/system/node")
    out: Dict[int, List[int]] = {}
    try:
        names = os.listdir(base)
    except OSError:
        return out
    for n in names:
        if n.startswith("node") and n[4:].isdigit():
            c = _read(os.path.join(base, n, "cpulist"))
            if c:
                out[int(n[4:])] = parse_cpulist(c)
    return out


def _core_order(cpus: List[int], root: str) -> List[int]:
    first = {}
    for c in cpus:
        sib = _read(os.path.join(root, f"sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list"))
        first[c] = min(parse_cpulist(sib)) if sib else c
    return sorted(cpus, key=lambda c: (first[c], c))


def plan(nranks: int, allowed: Optional[Sequence[int]] = None, root: str = "/",
         gpu_of_rank: Optional[Sequence[int]] = None) -> List[Placement]:
    """Disjoint CPU sets for ``nranks`` replicas, each from its GPU's NUMA node.

    The CPUs this process may use (``allowed``, default its affinity mask) are
    grouped by NUMA node; each node's CPUs are split evenly over the ranks whose
    GPU hangs off it.  Ranks with an unknown node (or more ranks than GPUs, the
    shared-GPU rehearsal) draw from what is left, so every rank gets a
    non-empty set whenever ``len(allowed) >= nranks``."""
    allowed = sorted(set(allowed if allowed is not None else os.sched_getaffinity(0)))
    info = gpus(root)
    if gpu_of_rank is None:
        gpu_of_rank = [r % len(info) if info else r for r in range(nranks)]
    nodes = numa_cpus(root)
    node_of_cpu = {c: n for n, cs in nodes.items() for c in cs}
    free_by_node: Dict[int, List[int]] = {}
    for c in allowed:
        free_by_node.setdefault(node_of_cpu.get(c, -1), []).append(c)
    # SMT siblings adjacent, so an even split hands out whole physical cores
    # (Linux numbers a core's second thread cpu+ncores: a plain slice of the
    # node's list would put two ranks on the two threads of one core)
    for nd in free_by_node:
        free_by_node[nd] = _core_order(free_by_node[nd], root)
    out = [Placement(rank=r, gpu=int(g), numa_node=(info[g].numa_node if g < len(info) else -1))
           for r, g in enumerate(gpu_of_rank)]
    # ranks per node (known node and that node has allowed CPUs)
    by_node: Dict[int, List[Placement]] = {}
    for p in out:
        if p.numa_node in free_by_node:
            by_node.setdefault(p.numa_node, []).append(p)
    for nd, ps in by_node.items():
        cs = free_by_node[nd]
        share = len(cs) // len(ps)
        if share == 0:
            continue
        for i, p in enumerate(ps):
            p.cpus = cs[i * share:(i + 1) * share]
        free_by_node[nd] = cs[len(ps) * share:]
    rest = [p for p in out if not p.cpus]
    if rest:
        pool = [c for cs in free_by_node.values() for c in cs]
        if len(pool) < len(rest):          # too few left over: share the whole allowed set
            pool = allowed
        share = max(1, len(pool) // len(rest))
        for i, p in enumerate(rest):
            p.cpus = pool[(i * share) % len(pool):(i * share) % len(pool) + share] or list(pool)
            if p.numa_node < 0 and p.cpus:
                p.numa_node = node_of_cpu.get(p.cpus[0], -1)
    return out


def pin(cpus: Sequence[int]) -> bool:
    """Restrict this process (threads created afterwards inherit it)."""
    if not cpus:
        return False
    try:
        os.sched_setaffinity(0, set(cpus))
        return True
    except (OSError, ValueError):
        return False


def busy_path(bdf: str, root: str = "/") -> Optional[str]:
    if not bdf:
        return None
    p = os.path.join(root, "sys/bus/pci/devices", bdf, "gpu_busy_percent")
    return p if os.path.exists(p) else None


class BusySampler:
    """Samples a GPU's ``gpu_busy_percent`` (the amdgpu driver's activity
    counter, the same source rocm-smi reads) on a background thread."""

    def __init__(self, bdf: str, period_s: float = 0.01, root: str = "/"):
        self.path = busy_path(bdf, root)
        self.period_s = period_s
        self.samples: List[float] = []
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None

    def start(self) -> "BusySampler":
        if self.path is not None:
            self._th = threading.Thread(target=self._run, name="tfs-busy", daemon=True)
            self._th.start()
        return self

    def _run(self):
        while not self._stop.wait(self.period_s):
            v = _read(self.path)
            if v is not None and v.isdigit():
                self.samples.append(float(v))

    def stop(self) -> Optional[dict]:
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=2)
        if not self.samples:
            return None
        s = self.samples
        return {"mean": round(sum(s) / len(s), 1), "max": max(s), "samples": len(s)}


def cpu_quota() -> Optional[float]:
    """cgroup-v2 CPU quota in cores (None when unlimited / unknown)."""
    v = _read("/sys/fs/cgroup/cpu.max")
    if not v:
        return None
    q, _, per = v.partition(" ")
    if q == "max":
        return None
    try:
        return int(q) / int(per or 100000)
    except ValueError:
        return None


def thread_cpu_by_tid(pid: Optional[int] = None) -> Dict[int, Tuple[str, float]]:
    """{tid: (thread name, CPU seconds)} (schedstat ns, like thread_cpu)."""
    out: Dict[int, Tuple[str, float]] = {}
    base = f"/proc/{pid or os.getpid()}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"{base}/{tid}/schedstat") as f:
                out[int(tid)] = (name, int(f.read().split()[0]) / 1e9)
        except (OSError, ValueError, IndexError):
            continue
    return out


def runq_wait_by_tid(pid: Optional[int] = None) -> Dict[int, Tuple[str, float]]:
    """{tid: (thread name, seconds spent runnable but waiting for a CPU)}:
    schedstat's second field.  Time a busy thread waits on a run queue is CPU
    contention (other tenants on its CPUs, or the cgroup quota throttling it)."""
    out: Dict[int, Tuple[str, float]] = {}
    base = f"/proc/{pid or os.getpid()}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/comm") as f:
                name = f.read().strip()
            with open(f"{base}/{tid}/schedstat") as f:
                out[int(tid)] = (name, int(f.read().split()[1]) / 1e9)
        except (OSError, ValueError, IndexError):
            continue
    return out


def runq_wait_by_group(before: Dict[int, Tuple[str, float]], after: Dict[int, Tuple[str, float]],
                       elapsed: float) -> Dict[str, float]:
    """Run-queue wait per thread group over a window, as a fraction of the
    window summed over the group's threads (1.0 = one thread waited the whole
    window)."""
    groups: Dict[str, float] = {}
    for tid, (name, v) in after.items():
        g = name.rstrip("0123456789")
        groups[g] = groups.get(g, 0.0) + v - before.get(tid, (name, 0.0))[1]
    return {k: round(v / max(elapsed, 1e-9), 3) for k, v in sorted(groups.items(), key=lambda x: -x[1])
            if v / max(elapsed, 1e-9) >= 0.001}


def cpu_times(root: str = "/") -> Dict[int, Tuple[int, int]]:
    """{cpu: (busy jiffies, total jiffies)} of every CPU of the host, from
    /proc/stat (it shows the whole machine, other tenants included)."""
    out: Dict[int, Tuple[int, int]] = {}
    try:
        with open(os.path.join(root, "proc/stat")) as f:
            lines = f.readlines()
    except OSError:
        return out
    for ln in lines:
        if not ln.startswith("cpu") or ln.startswith("cpu "):
            continue
        parts = ln.split()
        try:
            cpu = int(parts[0][3:])
            v = [int(x) for x in parts[1:]]
        except ValueError:
            continue
        idle = v[3] + (v[4] if len(v) > 4 else 0)           # idle + iowait
        total = sum(v[:8])                                     # guest time is already inside user
        out[cpu] = (total - idle, total)
    return out


def busy_fraction(before: Dict[int, Tuple[int, int]], after: Dict[int, Tuple[int, int]],
                  cpus: Optional[Sequence[int]] = None) -> Optional[float]:
    """Busy share of ``cpus`` (default: all) between two cpu_times() snapshots."""
    keys = [c for c in (cpus if cpus is not None else after.keys()) if c in before and c in after]
    busy = sum(after[c][0] - before[c][0] for c in keys)
    total = sum(after[c][1] - before[c][1] for c in keys)
    return round(busy / total, 3) if total > 0 else None


def cgroup_throttling() -> Dict[str, int]:
    """cgroup-v2 ``cpu.stat`` counters (nr_periods, nr_throttled, throttled_usec)."""
    out: Dict[str, int] = {}
    v = _read("/sys/fs/cgroup/cpu.stat")
    for ln in (v or "").splitlines():
        k, _, n = ln.partition(" ")
        if k in ("nr_periods", "nr_throttled", "throttled_usec") and n.strip().isdigit():
            out[k] = int(n)
    return out


class HostContention:
    """What the rest of the machine did to a window: busy share of this
    process's NUMA-node CPUs and of the whole host (other tenants included),
    run-queue wait of this process's threads, and cgroup quota throttling."""

    def __init__(self, cpus: Optional[Sequence[int]] = None):
        self.cpus = list(cpus) if cpus else None

    def start(self) -> "HostContention":
        self.t0 = time.perf_counter()
        self.ct0, self.rq0, self.th0 = cpu_times(), runq_wait_by_tid(), cgroup_throttling()
        return self

    def stop(self) -> dict:
        secs = time.perf_counter() - self.t0
        ct1, rq1, th1 = cpu_times(), runq_wait_by_tid(), cgroup_throttling()
        d = {"host_busy": busy_fraction(self.ct0, ct1),
             "node_busy": busy_fraction(self.ct0, ct1, self.cpus) if self.cpus else None,
             "runq_wait": runq_wait_by_group(self.rq0, rq1, secs)}
        if th1 and self.th0:
            d["throttled_periods"] = th1.get("nr_throttled", 0) - self.th0.get("nr_throttled", 0)
            d["throttled_ms"] = round((th1.get("throttled_usec", 0) - self.th0.get("throttled_usec", 0)) / 1e3, 1)
        return d


def llc_groups(cpus: Sequence[int], root: str = "/") -> List[List[int]]:
    """``cpus`` grouped by last-level cache (``cache/index3/shared_cpu_list``:
    one group per CCD on EPYC), groups in order of their lowest CPU."""
    groups: Dict[int, List[int]] = {}
    for c in cpus:
        s = _read(os.path.join(root, f"sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list"))
        key = min(parse_cpulist(s)) if s else -1
        groups.setdefault(key, []).append(c)
    return [sorted(v) for _k, v in sorted(groups.items())]


def pick_llcs(cpus: Sequence[int], n: int, sample_s: float = 0.2, root: str = "/") -> List[int]:
    """The CPUs of the ``n`` least-busy last-level-cache groups among ``cpus``
    (busy share over a ``sample_s`` look at /proc/stat, other tenants included).
    A loopback benchmark moves every 602 KB request from the load generator's
    core to an IO thread's core: inside one L3 that copy stays on-die, across
    CCDs it goes through the fabric."""
    groups = llc_groups(cpus, root)
    if n <= 0 or n >= len(groups):
        return sorted(cpus)
    a = cpu_times(root)
    time.sleep(sample_s)
    b = cpu_times(root)
    groups.sort(key=lambda g: (busy_fraction(a, b, g) or 0.0, g[0]))
    return sorted(c for g in groups[:n] for c in g)


def thread_llcs(prefixes: Sequence[str], root: str = "/") -> Dict[str, object]:
    """Where this process's hot threads last ran: {"cpus": {name: cpu},
    "llcs": distinct last-level caches among them}."""
    where: Dict[str, int] = {}
    base = f"/proc/{os.getpid()}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        tids = []
    for tid in tids:
        try:
            with open(f"{base}/{tid}/comm") as f:
                name = f.read().strip()
            if not any(name.startswith(p) for p in prefixes):
                continue
            with open(f"{base}/{tid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            where[f"{name}/{tid}"] = int(fields[36])       # field 39: CPU last run on
        except (OSError, ValueError, IndexError):
            continue
    llcs = set()
    for c in where.values():
        s = _read(os.path.join(root, f"sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list"))
        llcs.add(min(parse_cpulist(s)) if s else c)
    return {"cpus": dict(sorted(where.items())), "llcs": len(llcs)}


def confine_threads(cpus: Sequence[int]) -> Dict[int, List[int]]:
    """Move every thread of this process (and threads it creates later: they
    inherit the calling thread's mask) onto ``cpus``.  Returns the previous
    masks by thread id, for ``restore_threads``."""
    old: Dict[int, List[int]] = {}
    want = set(int(c) for c in cpus)
    if not want:
        return old
    try:
        tids = [int(t) for t in os.listdir(f"/proc/{os.getpid()}/task")]
    except OSError:
        tids = []
    for tid in tids:
        try:
            old[tid] = sorted(os.sched_getaffinity(tid))
            os.sched_setaffinity(tid, want)
        except (OSError, ValueError):
            continue
    return old


def restore_threads(old: Dict[int, List[int]]) -> None:
    for tid, mask in old.items():
        try:
            os.sched_setaffinity(tid, set(mask))
        except (OSError, ValueError):
            continue


def pin_hot_threads(prefixes: Sequence[str], cpus: Sequence[int], sample_s: float = 0.2,
                    root: str = "/") -> Dict[str, int]:
    """Give each thread of this process whose name starts with one of
    ``prefixes`` a physical core of its own, from ``cpus``: cores whose
    hardware threads were least busy over a ``sample_s`` look at /proc/stat
    first (other tenants included), one hardware thread per hot thread.
    Returns {"tid name": cpu}."""
    a = cpu_times(root)
    time.sleep(sample_s)
    b = cpu_times(root)
    cores: Dict[int, List[int]] = {}
    for c in cpus:
        sib = _read(os.path.join(root, f"sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list"))
        sibs = parse_cpulist(sib) if sib else [c]
        cores.setdefault(min(sibs), []).append(c)

    def load(core):
        sib = _read(os.path.join(root, f"sys/devices/system/cpu/cpu{core}/topology/thread_siblings_list"))
        sibs = parse_cpulist(sib) if sib else [core]
        return busy_fraction(a, b, sibs) or 0.0

    order = sorted(cores, key=lambda k: (load(k), k))
    hot = [(tid, name) for tid, (name, _v) in sorted(thread_cpu_by_tid().items())
           if any(name.startswith(p) for p in prefixes)]
    out: Dict[str, int] = {}
    for i, (tid, name) in enumerate(hot):
        if not order:
            break
        cpu = cores[order[i % len(order)]][0]
        try:
            os.sched_setaffinity(tid, {cpu})
            out[f"{tid} {name}"] = cpu
        except (OSError, ValueError):
            continue
    return out


def top_threads(before: Dict[int, Tuple[str, float]], after: Dict[int, Tuple[str, float]], elapsed: float,
                n: int = 6) -> List[list]:
    """The ``n`` busiest threads of a window: [name, tid, cores, is_main_thread]."""
    rows = []
    for tid, (name, v) in after.items():
        d = v - before.get(tid, (name, 0.0))[1]
        if d > 0:
            rows.append([name, tid, round(d / max(elapsed, 1e-9), 2), tid == os.getpid()])
    rows.sort(key=lambda r: -r[2])
    rows = rows[:n]
    who = python_thread_sites()
    for r in rows:
        # a busy thread the kernel only knows by the process name: say which
        # Python thread (and where it is) or which kernel wait it sits in
        if r[1] in who:
            r.append(who[r[1]])
        else:
            r.append(_kernel_state(r[1]))
    return rows


def python_thread_sites() -> Dict[int, str]:
    """{native thread id: "name @ file:line in function"} of this process's
    Python threads (innermost frame)."""
    import sys
    import threading
    frames = sys._current_frames()
    out: Dict[int, str] = {}
    for t in threading.enumerate():
        nid = getattr(t, "native_id", None)
        f = frames.get(t.ident)
        if nid is None:
            continue
        where = ""
        if f is not None:
            where = f" @ {os.path.basename(f.f_code.co_filename)}:{f.f_lineno} in {f.f_code.co_name}"
        out[nid] = f"py:{t.name}{where}"
    return out


def _kernel_state(tid: int) -> str:
    """A native (non-Python) thread's scheduler state and wait channel."""
    base = f"/proc/{os.getpid()}/task/{tid}"
    state = wchan = ""
    try:
        with open(f"{base}/stat") as f:
            state = f.read().rsplit(")", 1)[1].split()[0]
    except (OSError, IndexError):
        pass
    try:
        with open(f"{base}/wchan") as f:
            wchan = f.read().strip()
    except OSError:
        pass
    return f"native:{state}:{wchan or '-'}"


def thread_cpu(pid: Optional[int] = None) -> Dict[str, float]:
    """{thread name: CPU seconds} of a process: on-CPU nanoseconds from
    ``schedstat`` (tick-based utime+stime from ``stat`` when schedstats are
    off; ticks are 10 ms, too coarse for a few-ms window)."""
    tick = os.sysconf("SC_CLK_TCK")
    out: Dict[str, float] = {}
    base = f"/proc/{pid or os.getpid()}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/comm") as f:
                name = f.read().strip()
            v = None
            try:
                with open(f"{base}/{tid}/schedstat") as f:
                    v = int(f.read().split()[0]) / 1e9
            except (OSError, ValueError, IndexError):
                pass
            if v is None:
                with open(f"{base}/{tid}/stat") as f:
                    fields = f.read().rsplit(")", 1)[1].split()
                v = (int(fields[11]) + int(fields[12])) / tick
            out[name] = out.get(name, 0.0) + v
        except (FileNotFoundError, ProcessLookupError, IndexError, ValueError):
            continue
    return out


def cpu_by_group(before: Dict[str, float], after: Dict[str, float], elapsed: float) -> Dict[str, float]:
    """Cores used per thread group (thread names without trailing digits)."""
    groups: Dict[str, float] = {}
    for k, v in after.items():
        g = k.rstrip("0123456789")
        groups[g] = groups.get(g, 0.0) + v - before.get(k, 0.0)
    return {k: round(v / max(elapsed, 1e-9), 2) for k, v in sorted(groups.items(), key=lambda x: -x[1])
            if v > 0.01}

