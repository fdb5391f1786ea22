"""bench.py as the driver invokes it: ``--gpus N`` launches N ranks by itself,
pins each to its GPU's NUMA-node CPUs and reports per-rank diagnostics.

CPU mode (``--device cpu``: CPU servables + gloo) so it runs without a GPU;
the GPU path differs only in the device and the nccl backend."""
import json
import os
import subprocess
import sys

import pytest

from rust_tensorflow_serving2_amd.parallel import topology

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_gpus2_self_launch_cpu(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["TMPDIR"] = str(tmp_path)
    cmd = [sys.executable, BENCH, "--gpus", "2", "--device", "cpu", "--model", "tiny", "--image-size", "32",
           "--steps", "4", "--warmup", "1", "--prewarm-s", "0.2", "--ref-client-requests", "64",
           "--c1-requests", "10", "--io-threads", "2", "--client-threads", "1", "--connections", "2",
           "--lanes", "2"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    out = _json_line(p.stdout)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["errors"] == 0 and out["value"] > 0
    diags = out["diagnostics"]
    assert [d["placement"]["rank"] for d in diags] == [0, 1]
    # both ranks served their own load generator's traffic in the timed window
    assert all(d["timed"]["requests"] > 0 for d in diags), diags
    assert all(d["prewarm"]["window_s"] > 0 for d in diags)
    # disjoint CPU sets when there are enough CPUs for both
    if len(os.sched_getaffinity(0)) >= 2:
        a, b = (set(topology.parse_cpulist(d["placement"]["cpus"])) for d in diags)
        assert a and b and not (a & b)
        assert all(d["placement"]["pinned"] for d in diags)
    assert out["ref_client_errors"] == 0
    # the weight replication the driver's scaling run depends on: the follower
    # received the leader's compiled weights over the collective (gloo here,
    # RCCL on the GPUs), read nothing from disk, copied no weight to a device
    # the replication protocol passed, but over gloo: a rehearsal, never "RCCL ok"
    assert out["replication_ok"] is True and "rccl_problems" not in out, out.get("rccl_problems")
    assert out["rehearsal"] is True and out["rccl_ok"] is False and out["rccl_backend"] == "gloo"
    lead, fol = out["rccl"]
    assert lead["leader"] and lead["backend"] == "gloo" and lead["world"] == 2
    # backend / size read from the group object, and an all-reduce of ones over it
    for x in (lead, fol):
        assert x["pg_backend"] == "gloo" and x["pg_size"] == 2 and x["allreduce_sum"] == 2.0, x
        assert x["blob_path"] == "host"
    assert lead["broadcast_bytes"] > 0 and lead["programs"] >= 1
    assert not fol["leader"] and fol["disk_loads"] == 0 and fol["weight_h2d_bytes"] == 0
    assert fol["bcast_loads"] >= 1 and fol["bound_bytes"] > 0
    assert fol["recompiles"] == 0, fol["recompile_reasons"]
    # every runner the follower built was bound to a broadcast blob
    assert fol["bound_bytes"] * lead["programs"] >= lead["broadcast_bytes"] * fol["programs"] * 0.9
    assert fol["broadcast_bytes"] == lead["broadcast_bytes"] and fol["broadcast_s"] >= 0
    pr = out["per_rank"]
    assert [x["rank"] for x in pr] == [0, 1] and all(x["ok"] > 0 and x["elapsed_s"] > 0 for x in pr)
    assert all("start_sync_ms" in x and "end_sync_ms" in x for x in pr)
    # the timed region ends at the last counted completion, inside the bracket
    assert all(x["bracket_s"] >= x["elapsed_s"] for x in pr)


@pytest.mark.timeout(900)
def test_bench_gpus8_self_launch_cpu(tmp_path):
    """The driver's N = 8 scaling run, rehearsed on the CPU (gloo, tiny
    model): 8 ranks launched by bench.py itself, every follower bound the
    broadcast weights, the all-reduce over the group sums to 8, and the
    reference-client phase (one client on rank 0's port, 1024 calls in flight)
    spills past rank 0 once its pipeline is full.  This rehearsal found a
    router leak at 8 ranks: a forwarded call whose cell was freed under it hung
    its client for the phase's 300-s timeout (ref_client_rps 1.7); see
    csrc/router.cpp respond_remote / reap."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["TMPDIR"] = str(tmp_path)
    cmd = [sys.executable, BENCH, "--gpus", "8", "--device", "cpu", "--model", "tiny", "--image-size", "32",
           "--steps", "4", "--warmup", "1", "--prewarm-s", "0.2", "--ref-client-requests", "512",
           "--c1-requests", "10", "--io-threads", "1", "--client-threads", "1", "--connections", "2",
           "--lanes", "2"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=880, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    out = _json_line(p.stdout)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["errors"] == 0 and out["value"] > 0 and out["value_bracket"] > 0
    pr = out["per_rank"]
    assert [x["rank"] for x in pr] == list(range(8))
    assert all(x["ok"] > 0 and 0 < x["interval_s"] <= x["elapsed_s"] for x in pr), pr
    assert out["rehearsal"] is True and out["replication_ok"] is True and "rccl_problems" not in out
    assert [x["allreduce_sum"] for x in out["rccl"]] == [8.0] * 8
    assert sum(1 for x in out["rccl"] if x["leader"]) == 1
    assert all(x["disk_loads"] == 0 and x["bcast_loads"] >= 1 for x in out["rccl"] if not x["leader"])
    # the reference client: no errors, no hung call (the leak made this 1.7 RPC/s)
    assert out["ref_client_errors"] == 0 and out["ref_client_rps"] > 100, out["ref_client_rps"]
    share = out["ref_client_gpu_share"]
    assert len(share) == 8 and abs(sum(share) - 1) < 0.01
    assert sum(share[1:]) > 0.5, share            # spilled past rank 0
    for d in out["diagnostics"]:
        for phase in (d["timed"], d["ref_client"]):
            r = phase.get("router") or {}
            assert r.get("orphaned", 0) == 0 and r.get("lost", 0) == 0, r


def test_rccl_problems_flags_silent_fallbacks():
    """bench.py exits non-zero (after printing its line) when a follower did
    not really receive the broadcast."""
    sys.path.insert(0, ROOT)
    import bench
    lead = {"rank": 0, "leader": True, "world": 2, "broadcast_bytes": 10, "disk_loads": 0, "weight_h2d_bytes": 5,
            "bcast_loads": 0, "bound_bytes": 0}
    good = {"rank": 1, "leader": False, "world": 2, "broadcast_bytes": 10, "disk_loads": 0, "weight_h2d_bytes": 0,
            "bcast_loads": 1, "bound_bytes": 10}
    assert bench.rccl_problems([lead, good], 2) == []
    assert bench.rccl_problems([lead, dict(good, disk_loads=1)], 2)
    assert bench.rccl_problems([lead, dict(good, weight_h2d_bytes=8)], 2)
    assert bench.rccl_problems([lead, dict(good, bound_bytes=0)], 2)
    assert bench.rccl_problems([dict(lead, broadcast_bytes=0), good], 2)
    assert bench.rccl_problems([lead, None], 2)
    # the all-reduce of ones over the group must sum to the launch's world size
    assert bench.rccl_problems([dict(lead, allreduce_sum=2.0), dict(good, allreduce_sum=2.0)], 2) == []
    assert bench.rccl_problems([dict(lead, allreduce_sum=1.0), good], 2)


@pytest.mark.timeout(200)
def test_bench_launcher_forwards_sigterm(tmp_path):
    """A driver timeout (SIGTERM to the launcher) ends the ranks too, although
    each runs in its own session."""
    import signal
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["TMPDIR"] = str(tmp_path)
    cmd = [sys.executable, BENCH, "--gpus", "2", "--device", "cpu", "--model", "tiny", "--image-size", "32",
           "--steps", "100000000", "--warmup", "1", "--prewarm-s", "0.2", "--io-threads", "1",
           "--client-threads", "1", "--connections", "1", "--lanes", "1"]
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, cwd=str(tmp_path))
    ranks = []
    deadline = time.time() + 120
    while time.time() < deadline and len(ranks) < 2:
        out = subprocess.run(["pgrep", "-P", str(p.pid)], capture_output=True, text=True).stdout.split()
        ranks = [int(x) for x in out]
        time.sleep(0.2)
    assert len(ranks) == 2
    time.sleep(3.0)
    p.send_signal(signal.SIGTERM)
    p.wait(timeout=60)
    assert p.returncode != 0
    deadline = time.time() + 30
    while time.time() < deadline and any(os.path.exists(f"/proc/{r}") and
                                         open(f"/proc/{r}/stat").read().split()[2] != "Z" for r in ranks):
        time.sleep(0.2)
    alive = [r for r in ranks if os.path.exists(f"/proc/{r}")]
    for r in alive:
        os.kill(r, signal.SIGKILL)
    assert not alive, alive


def test_bench_rejects_gpus_world_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--device", "cpu"], env=env, capture_output=True,
                       text=True, timeout=120, cwd=str(tmp_path))
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def _fake_sysfs(root, gpus_numa, cpus_per_node=8, smt=True):
    """KFD topology with CPU nodes then GPU nodes, PCI numa_node, NUMA cpulists
    and SMT siblings (cpu c and c + ncores)."""
    nnodes = max(gpus_numa) + 1
    ncores = nnodes * cpus_per_node
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    for n in range(nnodes):
        d = kfd / str(n)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {cpus_per_node}\nsimd_count 0\n")
    for i, numa in enumerate(gpus_numa):
        d = kfd / str(nnodes + i)
        d.mkdir(parents=True)
        bus = 0x10 * (i + 1)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        pci = root / f"sys/bus/pci/devices/0000:{bus:02x}:00.0"
        pci.mkdir(parents=True)
        (pci / "numa_node").write_text(f"{numa}\n")
        (pci / "gpu_busy_percent").write_text("42\n")
    for n in range(nnodes):
        d = root / f"sys/devices/system/node/node{n}"
        d.mkdir(parents=True)
        lo = n * cpus_per_node
        lst = f"{lo}-{lo + cpus_per_node - 1}"
        if smt:
            lst += f",{ncores + lo}-{ncores + lo + cpus_per_node - 1}"
        (d / "cpulist").write_text(lst + "\n")
    for c in range(ncores):
        for t in ([c, c + ncores] if smt else [c]):
            d = root / f"sys/devices/system/cpu/cpu{t}/topology"
            d.mkdir(parents=True, exist_ok=True)
            (d / "thread_siblings_list").write_text(f"{c},{c + ncores}\n" if smt else f"{c}\n")
    return list(range(2 * ncores if smt else ncores))


def test_topology_plan_numa_local_whole_cores(tmp_path, monkeypatch):
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    # 8 GPUs, 4 per socket, 2 sockets x 8 cores x 2 threads
    allowed = _fake_sysfs(tmp_path, [0, 0, 0, 0, 1, 1, 1, 1])
    info = topology.gpus(str(tmp_path))
    assert [g.numa_node for g in info] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert info[0].bdf == "0000:10:00.0"
    pl = topology.plan(8, allowed=allowed, root=str(tmp_path))
    node_cpus = topology.numa_cpus(str(tmp_path))
    seen = set()
    for p in pl:
        assert len(p.cpus) == 4
        assert set(p.cpus) <= set(node_cpus[p.numa_node])        # local socket
        cores = {c % 16 for c in p.cpus}
        assert len(cores) == 2                                     # two whole cores (both SMT threads)
        assert not (seen & set(p.cpus))
        seen |= set(p.cpus)
    # a restricted affinity mask (the 1-GPU box share) is respected
    pl = topology.plan(2, allowed=[0, 1, 16, 17], root=str(tmp_path))
    assert sorted(c for p in pl for c in p.cpus) == [0, 1, 16, 17]
    assert pl[0].cpus == [0, 16] and pl[1].cpus == [1, 17]


def test_topology_visible_devices_and_rehearsal(tmp_path, monkeypatch):
    allowed = _fake_sysfs(tmp_path, [0, 1], cpus_per_node=4, smt=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    info = topology.gpus(str(tmp_path))
    assert len(info) == 1 and info[0].numa_node == 1 and info[0].index == 0
    # 4 ranks sharing the one visible GPU (gloo rehearsal): disjoint slices of its node
    pl = topology.plan(4, allowed=allowed, root=str(tmp_path))
    assert all(p.gpu == 0 and p.numa_node == 1 for p in pl)
    assert sorted(c for p in pl for c in p.cpus) == [4, 5, 6, 7]
    s = topology.BusySampler(info[0].bdf, period_s=0.005, root=str(tmp_path)).start()
    import time
    time.sleep(0.05)
    r = s.stop()
    assert r and r["mean"] == 42.0


def test_host_contention_probes(tmp_path):
    """/proc/stat busy shares, run-queue wait and the per-thread core pinning
    bench.py reports / applies (``--pin-threads``)."""
    proc = tmp_path / "proc"
    proc.mkdir()
    (proc / "stat").write_text("cpu  10 0 10 80 0 0 0 0 0 0\n"
                               "cpu0 10 0 0 30 0 0 0 0 0 0\n"
                               "cpu1 0 0 10 50 0 0 0 0 0 0\nintr 1 2\n")
    a = topology.cpu_times(str(tmp_path))
    assert a == {0: (10, 40), 1: (10, 60)}
    b = {0: (30, 60), 1: (10, 80)}                       # cpu0 fully busy since, cpu1 idle
    assert topology.busy_fraction(a, b) == 0.5
    assert topology.busy_fraction(a, b, [0]) == 1.0 and topology.busy_fraction(a, b, [1]) == 0.0
    hc = topology.HostContention(sorted(os.sched_getaffinity(0))).start()
    sum(i * i for i in range(200000))
    d = hc.stop()
    assert d["host_busy"] is None or 0.0 <= d["host_busy"] <= 1.0
    assert isinstance(d["runq_wait"], dict)
    before = os.sched_getaffinity(0)
    try:
        with open("/proc/self/comm") as f:
            me = f.read().strip()
        pins = topology.pin_hot_threads((me,), sorted(before), sample_s=0.02)
        mine = [cpu for k, cpu in pins.items() if k.startswith(f"{os.getpid()} ")]
        assert mine and mine[0] in before and os.sched_getaffinity(0) == {mine[0]}
    finally:
        os.sched_setaffinity(0, before)


def test_llc_groups_and_pick(tmp_path):
    """L3 groups from cache/index3/shared_cpu_list; pick_llcs keeps the
    least-busy groups (per /proc/stat) and returns everything when asked for
    as many groups as exist."""
    cpus = list(range(8))
    for c in cpus:
        d = tmp_path / f"sys/devices/system/cpu/cpu{c}/cache/index3"
        d.mkdir(parents=True)
        lo = (c // 4) * 4
        (d / "shared_cpu_list").write_text(f"{lo}-{lo + 3}\n")
    assert topology.llc_groups(cpus, str(tmp_path)) == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert topology.pick_llcs(cpus, 2, root=str(tmp_path)) == cpus
    assert topology.pick_llcs(cpus, 0, root=str(tmp_path)) == cpus
    (tmp_path / "proc").mkdir()
    (tmp_path / "proc/stat").write_text("".join(f"cpu{c} 0 0 0 100 0 0 0 0\n" for c in cpus))
    # a static /proc/stat reads as idle everywhere: ties go to the lowest group
    assert topology.pick_llcs(cpus, 1, sample_s=0.0, root=str(tmp_path)) == [0, 1, 2, 3]
    on = topology.thread_llcs(("no-such-thread",), root=str(tmp_path))
    assert on == {"cpus": {}, "llcs": 0}


def test_cpulist_roundtrip():
    assert topology.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert topology.compress([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"


@pytest.mark.timeout(300)
def test_bench_multi_model_reload_cpu(tmp_path):
    """--model multi (BASELINE config 5) in CPU mode: ResNet traffic keeps
    flowing with zero errors while BERT is dropped and re-added by
    HandleReloadConfigRequest; reload-to-AVAILABLE times are reported."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["TMPDIR"] = str(tmp_path)
    cmd = [sys.executable, BENCH, "--model", "multi", "--device", "cpu", "--image-size", "32", "--seq-len", "16",
           "--batch", "8", "--reload-cycles", "2", "--bert-requests", "32", "--prewarm-s", "0.2",
           "--io-threads", "2", "--client-threads", "1", "--connections", "2", "--lanes", "2", "--concurrency", "16"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    out = _json_line(p.stdout)
    assert out["errors"] == 0 and out["value"] > 0 and out["bert_rps"] > 0
    assert len(out["reload_to_available_s"]) == 2 and all(t > 0 for t in out["reload_to_available_s"])
    r0 = out["per_rank"][0]
    assert r0["resnet_calls_during_reload"] > 0          # ResNet served while BERT reloaded
    # after the drop BERT was gone or on its way out (UNLOADING 40 / END 50), never AVAILABLE (30)
    assert all(30 not in c["bert_states_after_drop"] for c in r0["cycles"])
