"""Device-resident weight replication on the MI355X (parallel/weights.py).

* nccl (RCCL) at world size 1: the leader's load / compile / pack / broadcast
  path runs on the hardware.
* gloo at world size 2 on ONE GPU (two replicas sharing the device; RCCL
  refuses two ranks per GPU): the follower compiles ResNet-50 on shapes only,
  binds its program to the leader's packed bf16 device blob, installs the
  leader's tile picks -- zero host->device weight copies, no autotuning of
  its own -- and returns bit-identical outputs."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, backend, port, path, out_q, regroup=False, own_gpu=False, concurrent=False):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from rust_tensorflow_serving2_amd import ops
    from rust_tensorflow_serving2_amd.graph import placement
    from rust_tensorflow_serving2_amd.parallel.weights import ReplicatedWeightSource
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    try:
        dev = torch.device("cuda", rank if own_gpu else 0)
        torch.cuda.set_device(dev)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        ws = ReplicatedWeightSource(dist.distributed_c10d._get_default_store(), device=dev, load_timeout=300)
        h2d0 = placement.H2D_BYTES
        b = ws.load("resnet", 1, path)
        s = Servable("resnet", 1, path, ServableOptions(device=str(dev), max_batch_size=4,
                                                         allowed_batch_sizes=(4,)), b, weight_source=ws)
        x = np.random.default_rng(7).random((4, 224, 224, 3), dtype=np.float32)
        out = s.run("serving_default", {"input": x}, ["classes", "probabilities"])
        res = {"probs": out["probabilities"], "classes": out["classes"], "h2d": placement.H2D_BYTES - h2d0,
               "bound": ws.stats.get("bound_bytes", 0), "bcast": ws.stats.get("broadcast_bytes", 0),
               "tuned_here": len(ops._TUNE_TIMES), "remote": len(ops._REMOTE)}
        if regroup:
            # a replica restart bumps the generation: the next load forms a
            # standalone ProcessGroupNCCL on a fresh store prefix and broadcasts
            # through it (parallel/weights.py _Comm.form)
            store = dist.distributed_c10d._get_default_store()
            store.add("tfs/gen", 1)
            b0 = res["bcast"]
            b2 = ws.load("resnet", 2, path)
            s2 = Servable("resnet", 2, path, ServableOptions(device=str(dev), max_batch_size=4,
                                                              allowed_batch_sizes=(4,)), b2, weight_source=ws)
            out2 = s2.run("serving_default", {"input": x}, ["classes", "probabilities"])
            res.update(gen=ws.gen, regroups=ws.stats.get("regroups", 0),
                       bcast2=ws.stats.get("broadcast_bytes", 0) - b0, probs2=out2["probabilities"],
                       pg=type(ws.comm.pg).__name__)
        if concurrent:
            # a hot reload broadcast while version 1's lanes keep replaying:
            # the broadcast is ordered on its own stream (weights.py
            # _StreamMark), not behind a device-wide synchronize, and the live
            # replays stay bit-exact while it runs
            import threading
            stop, seen = threading.Event(), {"runs": 0, "bad": 0}

            def serve():
                while not stop.is_set():
                    o = s.run("serving_default", {"input": x}, ["classes", "probabilities"])
                    seen["runs"] += 1
                    seen["bad"] += int(not np.array_equal(o["probabilities"], res["probs"]))
            t = threading.Thread(target=serve)
            t.start()
            b0 = ws.stats.get("broadcast_bytes", 0)
            b3 = ws.load("resnet", 3, path)
            s3 = Servable("resnet", 3, path, ServableOptions(device=str(dev), max_batch_size=4,
                                                              allowed_batch_sizes=(4,)), b3, weight_source=ws)
            out3 = s3.run("serving_default", {"input": x}, ["classes", "probabilities"])
            runs_at_v3 = seen["runs"]
            stop.set()
            t.join(60)
            res.update(bcast3=ws.stats.get("broadcast_bytes", 0) - b0, probs3=out3["probabilities"],
                       runs_during=runs_at_v3, bad_during=seen["bad"], runs_total=seen["runs"])
        ws.close()
        dist.barrier()
        dist.destroy_process_group()
        out_q.put((rank, res))
    except Exception as e:  # pragma: no cover - reported to the test
        import traceback
        out_q.put((rank, {"error": f"{e}\n{traceback.format_exc()}"}))


def _run(world, backend, path, regroup=False, own_gpu=False, concurrent=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, backend, port, path, q, regroup, own_gpu, concurrent)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r, v in out.items():
        assert "error" not in v, v["error"]
    return out


@pytest.fixture(scope="module")
def r50(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("r50w"))
    resnet.export(os.path.join(base, "1"), seed=5)
    return os.path.join(base, "1")


def test_rccl_world1_leader_path(r50):
    out = _run(1, "nccl", r50)
    r = out[0]
    assert r["bcast"] > 20e6                       # ResNet-50's packed bf16 program weights went through RCCL
    np.testing.assert_allclose(r["probs"].sum(1), 1.0, atol=1e-4)


def test_rccl_regroup_after_restart_world1(r50):
    """Single-device stand-in for the post-restart regroup (RCCL refuses two
    ranks on one GPU): after the generation bump the next load runs through a
    freshly formed standalone ProcessGroupNCCL -- the device-side broadcast
    call a live replica and its replacement make on a real 8-GPU node."""
    out = _run(1, "nccl", r50, regroup=True)
    r = out[0]
    assert r["gen"] == 1 and r["regroups"] >= 1 and r["pg"] == "ProcessGroupNCCL"
    assert r["bcast2"] > 20e6                     # version 2's weights went through the generation-1 group
    np.testing.assert_array_equal(r["probs"], r["probs2"])


def test_rccl_reload_broadcast_while_lanes_replay_world1(r50):
    """Collective ordering against live lanes on the device: version 1 keeps
    serving (graph replays on its lanes' streams, in a thread) while version
    3 loads through RCCL -- its weights broadcast, compile and capture.  The
    replays during the reload stay bit-identical to before it, and version
    3's outputs match version 1's (same weights)."""
    out = _run(1, "nccl", r50, concurrent=True)
    r = out[0]
    assert r["bcast3"] > 20e6                     # version 3 went through RCCL
    assert r["runs_during"] >= 1                   # version 1 was replaying while it loaded
    assert r["bad_during"] == 0, r
    np.testing.assert_allclose(r["probs3"], r["probs"], atol=2e-4, rtol=0)   # tile picks may differ


def test_follower_binds_leader_blob_without_host_copies(r50):
    out = _run(2, "gloo", r50)
    lead, fol = out[0], out[1]
    np.testing.assert_array_equal(lead["probs"], fol["probs"])
    np.testing.assert_array_equal(lead["classes"], fol["classes"])
    assert lead["h2d"] > 20e6                      # the leader uploaded the folded weights once
    assert fol["h2d"] == 0                         # the follower: not one weight byte host -> device
    assert fol["bound"] >= 0.9 * lead["bcast"] and fol["bound"] > 20e6
    assert fol["tuned_here"] == 0 and fol["remote"] > 0     # the leader's tile picks, no own autotune


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL refuses two ranks on one GPU)")
def test_rccl_world2_device_broadcast_two_gpus(r50):
    """Two replicas on two GPUs over RCCL/xGMI, then a replica restart: the
    follower binds the leader's blob from a device-to-device broadcast (no
    host copy), both generations, bit-identical outputs."""
    out = _run(2, "nccl", r50, regroup=True, own_gpu=True)
    lead, fol = out[0], out[1]
    np.testing.assert_array_equal(lead["probs"], fol["probs"])
    np.testing.assert_array_equal(lead["probs2"], fol["probs2"])
    assert fol["h2d"] == 0 and fol["bound"] > 20e6
    assert lead["bcast2"] > 20e6 and fol["regroups"] >= 1 and fol["pg"] == "ProcessGroupNCCL"
