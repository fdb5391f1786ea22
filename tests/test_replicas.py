"""Data-parallel replicas on CPU (gloo, world_size 2): leader-ordered weight
broadcast (parallel/weights.py), config replication (parallel/replicas.py) and
the multi-replica server binary sharing one port via SO_REUSEPORT."""
import asyncio
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _weights_worker(rank, world, port, model_dir, out_q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from rust_tensorflow_serving2_amd.graph import placement
    from rust_tensorflow_serving2_amd.parallel.weights import LoadError, ReplicatedWeightSource
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    store = dist.distributed_c10d._get_default_store()
    ws = ReplicatedWeightSource(store, device=torch.device("cpu"), load_timeout=60, share=True)
    res = {}
    if rank == 0:
        time.sleep(0.5)                         # followers ask first: they must wait for the leader
    path = os.path.join(model_dir, "1")
    b = ws.load("m", 1, path)
    res["keys"] = sorted(b.bundle.keys())
    # followers hold no weight values: float variables are shape-only
    res["meta"] = sum(1 for k in res["keys"] if isinstance(b.bundle[k], torch.Tensor) and b.bundle[k].is_meta)
    res["sigs"] = sorted(b.signatures)
    # compile on every rank; the followers' program binds the leader's packed weights
    s = Servable("m", 1, path, ServableOptions(device="cpu", fuse=True), b, weight_source=ws)
    x = np.random.default_rng(0).random((2, 32, 32, 3), dtype=np.float32)
    out = s.run("serving_default", {"input": x}, ["classes", "probabilities"])
    res["probs"] = out["probabilities"].tolist()
    res["bound"] = ws.stats.get("bound_bytes", 0)
    try:
        ws.load("m", 2, os.path.join(model_dir, "does_not_exist"))
        res["err"] = None
    except LoadError as e:
        res["err"] = str(e)
    ws.close()
    dist.barrier()
    dist.destroy_process_group()
    out_q.put((rank, res))


def test_replicated_weight_source_gloo(tiny_resnet_path):
    """Leader reads + compiles, followers get a shape-only bundle and bind
    their compiled program to the leader's broadcast weight blob; outputs are
    identical on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_weights_worker, args=(r, 2, port, tiny_resnet_path, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0]["keys"] == out[1]["keys"] and len(out[0]["keys"]) > 10
    assert out[0]["meta"] == 0 and out[1]["meta"] > 10
    assert out[0]["sigs"] == out[1]["sigs"]
    np.testing.assert_array_equal(np.asarray(out[0]["probs"]), np.asarray(out[1]["probs"]))
    assert out[1]["bound"] > 0 and out[0]["bound"] == 0
    assert out[0]["err"] and out[1]["err"] and out[0]["err"] == out[1]["err"]


async def _predict(port, model, x):
    from rust_tensorflow_serving2_amd.client import TensorflowServing
    c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
    return await c.predict_tensors(model, {"x": x})


def test_cli_two_replicas_shared_port_and_reload(hpt_path, tmp_path):
    """`--num_gpus 2` on CPU: two replica processes on one port; a reload sent to
    whichever replica owns the connection is applied on both."""
    from rust_tensorflow_serving2_amd.client import TensorflowServing
    from rust_tensorflow_serving2_amd.schema import serving
    port = _free_port()
    logf = str(tmp_path / "replicas.log")
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    proc = subprocess.Popen([sys.executable, "-m", "rust_tensorflow_serving2_amd.server", f"--port={port}",
                             "--model_name=a", f"--model_base_path={hpt_path}", "--num_gpus=2", "--device=cpu",
                             "--host=127.0.0.1", "--file_system_poll_wait_seconds=0", "--log_level=WARNING"],
                            env=env, stdout=open(logf, "w"), stderr=subprocess.STDOUT, text=True,
                            start_new_session=True)
    try:
        deadline = time.time() + 180
        while time.time() < deadline and proc.poll() is None:
            if open(logf).read().count("ready:") >= 2:
                break
            time.sleep(0.2)
        assert open(logf).read().count("ready:") == 2, open(logf).read()[-3000:]
        x = np.array([[2.0]], np.float32)
        for _ in range(8):          # fresh connections spread over both replicas
            assert asyncio.run(_predict(port, "a", x))["y"].reshape(-1).tolist() == [3.0]

        async def reload():
            c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
            cfg = serving.ModelConfig(name="b", base_path=hpt_path, model_platform="tensorflow")
            return await c.reload([cfg])
        resp = asyncio.run(reload())
        assert resp.status.error_code == 0, resp.status.error_message
        for _ in range(16):         # both replicas now serve "b" and no longer "a"
            assert asyncio.run(_predict(port, "b", x))["y"].reshape(-1).tolist() == [3.0]
        from rust_tensorflow_serving2_amd.client import TFServingError
        with pytest.raises(TFServingError):
            asyncio.run(_predict(port, "a", x))
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)
            proc.wait()


def _stats(d):
    import json
    out = {}
    for f in sorted(os.listdir(d)):
        if f.endswith(".json"):
            with open(os.path.join(d, f)) as fh:
                s = json.load(fh)
            out[(s["rank"], s["pid"])] = s
    return out


def test_four_replicas_one_connection_and_replica_restart(hpt_path, tmp_path):
    """Four CPU replicas (gloo), ONE client connection (the reference client's
    pattern): the front end that owns the connection routes Predicts to the
    least-loaded replica over shared memory, so every replica serves >= 15%
    of 400 calls.  Then `kill -9` of one replica: the others keep serving,
    a config reload issued during the outage completes, the supervisor
    restarts only the dead replica, which rejoins (applies the new config,
    takes routed calls)."""
    import json
    import signal as sig
    from rust_tensorflow_serving2_amd.client import TensorflowServing, TFServingError
    from rust_tensorflow_serving2_amd.schema import serving
    port = _free_port()
    logf = str(tmp_path / "replicas.log")
    stats_dir = str(tmp_path / "stats")
    # the CPU replicas stand in for GPU replicas whose calls take real service
    # time: the per-request Python path (not the batched CPU fast path, which
    # answers half_plus_two in ~0.2 ms and so keeps almost everything local)
    # gives the load-based router the queueing it reacts to
    env = dict(os.environ, PYTHONPATH=ROOT, TFSERVE_STATS_DIR=stats_dir, TFSERVE_ROUTE_CELLS="16",
               TFSERVE_ROUTE_MARGIN="2", TFSERVE_SHARE_WAIT_S="2", TFSERVE_CPU_FAST_PATH="0")
    env.pop("WORLD_SIZE", None)
    proc = subprocess.Popen([sys.executable, "-m", "rust_tensorflow_serving2_amd.server", f"--port={port}",
                             "--model_name=a", f"--model_base_path={hpt_path}", "--num_gpus=4", "--device=cpu",
                             "--host=127.0.0.1", "--file_system_poll_wait_seconds=0", "--log_level=WARNING",
                             "--io_threads=1"],
                            env=env, stdout=open(logf, "w"), stderr=subprocess.STDOUT, text=True,
                            start_new_session=True)

    def ready_count():
        return open(logf).read().count("ready:")

    async def burst(model, n, conc=32):
        c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()   # one channel
        x = {"x": np.array([[2.0]], np.float32)}
        sem = asyncio.Semaphore(conc)

        async def one():
            async with sem:
                return (await c.clone().predict_tensors(model, x))["y"].reshape(-1).tolist()
        return await asyncio.gather(*[one() for _ in range(n)])

    try:
        deadline = time.time() + 240
        while time.time() < deadline and proc.poll() is None and ready_count() < 4:
            time.sleep(0.2)
        assert ready_count() == 4, open(logf).read()[-3000:]
        time.sleep(1.0)                                  # routers see their peers
        out = asyncio.run(burst("a", 400))
        assert all(v == [3.0] for v in out)
        time.sleep(1.0)                                  # stats files refresh every 0.5 s
        st = _stats(stats_dir)
        served = {r: s["served"] for (r, _p), s in st.items()}
        assert len(served) == 4 and sum(served.values()) >= 400, st
        for r, n in served.items():
            assert n >= 0.15 * 400, (served, st)

        # ---- kill -9 one replica: the rest keep serving on fresh connections
        victim = 2
        vpid = next(p for (r, p) in st if r == victim)
        os.kill(vpid, sig.SIGKILL)
        time.sleep(0.5)
        for _ in range(6):
            assert asyncio.run(burst("a", 10, conc=4)) == [[3.0]] * 10

        # ---- a reload during the outage completes (the dead replica is not waited for)
        async def reload():
            c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
            return await c.reload([serving.ModelConfig(name="b", base_path=hpt_path, model_platform="tensorflow")])
        t0 = time.time()
        resp = asyncio.run(reload())
        assert resp.status.error_code == 0, resp.status.error_message
        assert time.time() - t0 < 60

        # ---- the supervisor restarted only the victim; it rejoins with the new config
        deadline = time.time() + 240
        while time.time() < deadline and ready_count() < 5:
            time.sleep(0.2)
        log_text = open(logf).read()
        assert ready_count() == 5 and "replica 2 exited" in log_text, log_text[-3000:]
        time.sleep(1.5)
        out = asyncio.run(burst("b", 400))
        assert all(v == [3.0] for v in out)
        with pytest.raises(TFServingError):
            asyncio.run(burst("a", 1, conc=1))
        time.sleep(1.0)
        st2 = _stats(stats_dir)
        new = [s for (r, p), s in st2.items() if r == victim and p != vpid]
        assert new and new[0]["restarts"] == 1 and new[0]["served"] > 0, st2
        assert proc.poll() is None                       # the group is still up
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)
            proc.wait()


def test_restart_reforms_weight_broadcast_group(tiny_resnet_path, tmp_path):
    """Three CPU replicas sharing weights through the leader's broadcast
    (gloo; TFSERVE_SHARE_WEIGHTS=1 rehearses the GPU path).  `kill -9` of a
    follower: the supervisor restarts it and bumps the group's generation.
    A reload to a new version is then broadcast again -- every follower, the
    replacement included, forms the generation-1 group and receives the new
    version from the leader (no disk read on the survivor) -- instead of every
    later load on every rank going to disk (model_service.proto:19-21)."""
    import json
    import shutil
    import signal as sig
    from rust_tensorflow_serving2_amd.client import TensorflowServing
    from rust_tensorflow_serving2_amd.schema import serving
    base = str(tmp_path / "r")
    shutil.copytree(os.path.join(tiny_resnet_path, "1"), os.path.join(base, "1"))
    port = _free_port()
    logf = str(tmp_path / "replicas.log")
    stats_dir = str(tmp_path / "stats")
    env = dict(os.environ, PYTHONPATH=ROOT, TFSERVE_STATS_DIR=stats_dir, TFSERVE_SHARE_WEIGHTS="1",
               TFSERVE_SHARE_WAIT_S="5")
    env.pop("WORLD_SIZE", None)
    proc = subprocess.Popen([sys.executable, "-m", "rust_tensorflow_serving2_amd.server", f"--port={port}",
                             "--model_name=r", f"--model_base_path={base}", "--num_gpus=3", "--device=cpu",
                             "--host=127.0.0.1", "--file_system_poll_wait_seconds=0", "--log_level=WARNING",
                             "--io_threads=1"],
                            env=env, stdout=open(logf, "w"), stderr=subprocess.STDOUT, text=True,
                            start_new_session=True)

    def ready_count():
        return open(logf).read().count("ready:")

    x = np.random.default_rng(0).random((1, 32, 32, 3), dtype=np.float32)

    async def predict(version=None):
        c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
        from rust_tensorflow_serving2_amd.client import ModelDescription
        return await c.predict_tensors(ModelDescription("r", version) if version else "r", {"input": x})

    try:
        deadline = time.time() + 240
        while time.time() < deadline and proc.poll() is None and ready_count() < 3:
            time.sleep(0.2)
        assert ready_count() == 3, open(logf).read()[-3000:]
        p1 = asyncio.run(predict())["probabilities"]
        time.sleep(1.0)
        st = _stats(stats_dir)
        gen0 = {r: s["weights"] for (r, _p), s in st.items()}
        assert gen0[1]["gen"] == 0 and gen0[2]["gen"] == 0 and gen0[2]["disk_loads"] == 0, gen0

        victim = 1
        vpid = next(p for (r, p) in st if r == victim)
        os.kill(vpid, sig.SIGKILL)
        deadline = time.time() + 240
        while time.time() < deadline and ready_count() < 4:
            time.sleep(0.2)
        assert ready_count() == 4, open(logf).read()[-3000:]
        time.sleep(1.5)                                   # the replacement's heartbeat is fresh

        # a new version, loaded by a reload (supersedes the config)
        shutil.copytree(os.path.join(base, "1"), os.path.join(base, "2"))

        async def reload():
            c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
            return await c.reload([serving.ModelConfig(name="r", base_path=base, model_platform="tensorflow")])
        resp = asyncio.run(reload())
        assert resp.status.error_code == 0, resp.status.error_message
        for _ in range(6):
            np.testing.assert_allclose(asyncio.run(predict(2))["probabilities"], p1, rtol=1e-5, atol=1e-6)
        time.sleep(1.0)
        st2 = _stats(stats_dir)
        now = {r: s for (r, p), s in st2.items() if p != vpid}
        surv, repl = now[2]["weights"], now[victim]["weights"]
        assert now[victim]["restarts"] == 1
        # the survivor: regrouped at generation 1 and got version 2 over the broadcast
        assert surv["gen"] == 1 and surv["disk_loads"] == 0 and surv["bcast_loads"] >= 2, surv
        # the replacement: version 1 from disk (before it existed), version 2 over the broadcast
        assert repl["gen"] == 1 and repl["disk_loads"] == 1 and repl["bcast_loads"] >= 1, repl
        assert now[0]["weights"]["gen"] == 1
        assert proc.poll() is None
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)
            proc.wait()


def test_reload_right_after_replica_kill_does_not_hang(tiny_resnet_path, tmp_path):
    """A reload issued while a killed follower is still being replaced (its
    last heartbeat fresh, the generation already bumped) must not block in a
    broadcast the dead rank -- or its replacement, which starts after the
    event -- can never join: the leader gates the new generation on
    membership and loads from disk until every rank has joined.  Once the
    replacement is up, the next reload is broadcast again."""
    import json
    import shutil
    import signal as sig
    from rust_tensorflow_serving2_amd.client import ModelDescription, TensorflowServing
    from rust_tensorflow_serving2_amd.schema import serving
    base = str(tmp_path / "r")
    shutil.copytree(os.path.join(tiny_resnet_path, "1"), os.path.join(base, "1"))
    port = _free_port()
    logf = str(tmp_path / "replicas.log")
    stats_dir = str(tmp_path / "stats")
    env = dict(os.environ, PYTHONPATH=ROOT, TFSERVE_STATS_DIR=stats_dir, TFSERVE_SHARE_WEIGHTS="1",
               TFSERVE_SHARE_WAIT_S="5")
    env.pop("WORLD_SIZE", None)
    proc = subprocess.Popen([sys.executable, "-m", "rust_tensorflow_serving2_amd.server", f"--port={port}",
                             "--model_name=r", f"--model_base_path={base}", "--num_gpus=3", "--device=cpu",
                             "--host=127.0.0.1", "--file_system_poll_wait_seconds=0", "--log_level=WARNING",
                             "--io_threads=1"],
                            env=env, stdout=open(logf, "w"), stderr=subprocess.STDOUT, text=True,
                            start_new_session=True)

    def ready_count():
        return open(logf).read().count("ready:")

    x = np.random.default_rng(0).random((1, 32, 32, 3), dtype=np.float32)

    async def predict(version=None):
        c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
        return await c.predict_tensors(ModelDescription("r", version) if version else "r", {"input": x})

    async def reload():
        c = await TensorflowServing.new().hostname("127.0.0.1").port(port).build()
        return await c.reload([serving.ModelConfig(name="r", base_path=base, model_platform="tensorflow")])

    try:
        deadline = time.time() + 240
        while time.time() < deadline and proc.poll() is None and ready_count() < 3:
            time.sleep(0.2)
        assert ready_count() == 3, open(logf).read()[-3000:]
        p1 = asyncio.run(predict())["probabilities"]
        time.sleep(1.0)
        st = _stats(stats_dir)
        victim = 1
        vpid = next(p for (r, p) in st if r == victim)
        shutil.copytree(os.path.join(base, "1"), os.path.join(base, "2"))
        os.kill(vpid, sig.SIGKILL)
        time.sleep(0.5)                                   # the supervisor has bumped the generation
        t0 = time.time()
        resp = asyncio.run(reload())
        took = time.time() - t0
        assert resp.status.error_code == 0, resp.status.error_message
        assert took < 60, took                            # not a collective waiting for the dead rank
        np.testing.assert_allclose(asyncio.run(predict(2))["probabilities"], p1, rtol=1e-5, atol=1e-6)

        deadline = time.time() + 240
        while time.time() < deadline and ready_count() < 4:
            time.sleep(0.2)
        assert ready_count() == 4, open(logf).read()[-3000:]
        time.sleep(1.5)
        shutil.copytree(os.path.join(base, "1"), os.path.join(base, "3"))
        resp = asyncio.run(reload())
        assert resp.status.error_code == 0, resp.status.error_message
        np.testing.assert_allclose(asyncio.run(predict(3))["probabilities"], p1, rtol=1e-5, atol=1e-6)
        time.sleep(1.0)
        now = {r: s for (r, p), s in _stats(stats_dir).items() if p != vpid}
        surv = now[2]["weights"]
        # version 2 went to disk (the group was not complete); version 3 over the broadcast
        assert surv["gen"] >= 1 and surv["disk_loads"] >= 1 and surv["bcast_loads"] >= 2, surv
        assert now[victim]["weights"]["bcast_loads"] >= 1, now[victim]
        assert proc.poll() is None
    finally:
        os.killpg(proc.pid, 15)
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, 9)
            proc.wait()


def test_backend_strings_pick_the_device_backend():
    """Round-5 ADVICE: a group set up before cli.py may report a multi-backend
    string; the replica runs the backend listed for its device type."""
    from rust_tensorflow_serving2_amd.parallel.weights import parse_backend
    assert parse_backend("nccl", "cuda") == "nccl"
    assert parse_backend("GLOO", "cpu") == "gloo"
    assert parse_backend("cpu:gloo,cuda:nccl", "cuda") == "nccl"
    assert parse_backend("cpu:gloo,cuda:nccl", "cpu") == "gloo"
    assert parse_backend("cpu:gloo, cuda:gloo", "cuda") == "gloo"
    assert parse_backend("cuda:nccl", "cpu") == "nccl"       # the only entry
    assert parse_backend(None, "cuda") is None
