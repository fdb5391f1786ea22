"""ResNet-50 v1.5 (random init) end to end on the GPU runtime vs the fp32 CPU
reference interpreter of the same SavedModel (BASELINE config 2 shape)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


@pytest.fixture(scope="module")
def resnet50(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("r50"))
    resnet.export(os.path.join(base, "1"), seed=0)
    return os.path.join(base, "1")


def _check_logits_and_classes(g, c):
    """bf16 GPU vs fp32 CPU: logits (recovered as centred log-probabilities)
    within 5 % of their spread, and the same top-1 class wherever the fp32
    top-1 / top-2 margin exceeds 3x the observed logit error."""
    lg = np.log(np.maximum(g["probabilities"], 1e-30)).astype(np.float64)
    lc = np.log(np.maximum(c["probabilities"], 1e-30)).astype(np.float64)
    lg -= lg.mean(1, keepdims=True)
    lc -= lc.mean(1, keepdims=True)
    err = np.abs(lg - lc).max(1)
    rel = err / lc.std(1)
    assert rel.max() < 5e-2, rel
    top2 = np.sort(lc, 1)[:, -2:]
    decided = (top2[:, 1] - top2[:, 0]) > 3 * err
    assert decided.any()
    np.testing.assert_array_equal(g["classes"][decided], c["classes"][decided])
    return rel.max()


def test_resnet50_gpu_matches_cpu(resnet50):
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    gpu = Servable("resnet", 1, resnet50, ServableOptions(device="cuda:0", max_batch_size=8))
    cpu = Servable("resnet", 1, resnet50, ServableOptions(device="cpu"))
    x = np.random.default_rng(1).random((5, 224, 224, 3), dtype=np.float32)
    g = gpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    c = cpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    assert g["probabilities"].shape == (5, 1001)
    np.testing.assert_allclose(g["probabilities"].sum(1), 1.0, atol=1e-4)
    err = np.abs(g["probabilities"] - c["probabilities"]).max()
    assert err < 5e-3, err
    _check_logits_and_classes(g, c)
    # run again (HIP-graph replay path, different batch inside the same bucket)
    g2 = gpu.run("serving_default", {"input": x[:3]}, ["classes", "probabilities"])
    # bucket 4 vs bucket 8 may pick different tile/split-K configs -> fp32 summation order differs
    np.testing.assert_allclose(g2["probabilities"], g["probabilities"][:3], atol=2e-4)
    runner = next(iter(gpu._runners.values()))
    hist = runner.program.op_histogram(flat=True)
    # 53 convs: 4 stage-entry (expand conv + projection shortcut) pairs run as
    # one K-concatenated dual-source GEMM each
    # the stem conv runs inside the fused stem + max-pool kernel
    assert hist.get("_FusedDualConv") == 4 and "Conv2D" not in hist
    assert hist.get("_StemPool") == 1 and "_MaxPool" not in hist
    # the 2 stage-1 and 3 stage-2 expand -> next-reduce pairs are chained ops
    # (each bucket then times the chain kernel against the two convs)
    assert hist.get("_ChainConv") == 5
    assert hist.get("_FusedConv2D") + 2 * hist["_FusedDualConv"] + 2 * hist["_ChainConv"] + hist["_StemPool"] == 53


@pytest.fixture(scope="module")
def resnet50_v2(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("r50v2"))
    resnet.export(os.path.join(base, "1"), version="v2", seed=2)
    return os.path.join(base, "1")


def test_resnet50_v2_gpu_fully_fused_matches_cpu(resnet50_v2):
    """ResNet-50 v2 -- the model the reference serves (serving/fetch.sh:7,
    resnet_v2_fp32_savedmodel_NHWC): pre-activation BN+ReLU ride on the
    producing conv / pool epilogues, so the GPU program has no BN, ReLU or Mul
    node left; logits and classes match the fp32 CPU interpreter."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    gpu = Servable("resnet", 1, resnet50_v2, ServableOptions(device="cuda:0", max_batch_size=8))
    cpu = Servable("resnet", 1, resnet50_v2, ServableOptions(device="cpu"))
    x = np.random.default_rng(3).random((6, 224, 224, 3), dtype=np.float32)
    g = gpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    c = cpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(g["probabilities"].sum(1), 1.0, atol=1e-4)
    _check_logits_and_classes(g, c)
    runner = next(iter(gpu._runners.values()))
    hist = runner.program.op_histogram(flat=True)
    for op in ("FusedBatchNormV3", "Relu", "Mul", "Conv2D", "AddV2"):
        assert op not in hist, hist
    assert hist.get("_StemPool") == 1 and "_MaxPool" not in hist
    assert hist.get("_FusedConv2D") + 2 * hist.get("_FusedDualConv", 0) + 2 * hist.get("_ChainConv", 0) + \
        hist["_StemPool"] == 53


def test_smoke():
    from rust_tensorflow_serving2_amd.smoke import run_smoke
    run_smoke()


def _pool_bytes(pool_ids):
    """Device bytes reserved by the given graph memory pools (allocator snapshot)."""
    snap = torch.cuda.memory._snapshot()
    return sum(seg["total_size"] for seg in snap["segments"] if tuple(seg.get("segment_pool_id", ())) in pool_ids)


def test_lane_buckets_share_one_graph_pool(resnet50, monkeypatch):
    """Every bucket graph of a lane captures into one memory pool (the lane
    replays one bucket at a time): far less device memory than a private pool
    per bucket, and replays in any bucket order give the same outputs."""
    import gc
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    x = torch.from_numpy(np.random.default_rng(5).random((32, 224, 224, 3), dtype=np.float32))
    used = {}
    for share in ("0", "1"):
        monkeypatch.setenv("TFSERVE_SHARED_GRAPH_POOL", share)
        s = Servable("resnet", 1, resnet50, ServableOptions(
            device="cuda:0", max_batch_size=32, allowed_batch_sizes=(1, 2, 4, 8, 16, 32), lanes=1))
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        r.lane_host_pointers(0)
        lane = r.lanes[0]
        torch.cuda.synchronize()
        pools = {tuple(g.pool()) for g in lane.graphs.values()}
        assert len(pools) == (1 if share == "1" else len(lane.graphs))
        used[share] = _pool_bytes(pools)
        lane.dev_in[0].copy_(x.to(lane.dev_in[0].device))
        # buckets of <= 4 rows copy their rows from the pinned host rows inside
        # the graph (GpuRunner._graph_h2d): give them the same rows
        lane.host_in[0].copy_(x.to(lane.host_in[0].dtype))
        probs = {}
        for b in (32, 1, 16, 2, 32, 8, 4, 1, 16):
            with torch.cuda.stream(lane.stream):
                lane.graphs[b].replay()
            lane.stream.synchronize()
            probs.setdefault(b, []).append(lane.static_out[b][1][:b].float().cpu().clone())
        for b, ps in probs.items():
            for p in ps[1:]:
                assert torch.equal(p, ps[0]), b
            # buckets may pick different tiles / split-K -> fp32 summation order differs
            torch.testing.assert_close(ps[0], probs[32][0][:b], atol=2e-4, rtol=0)
        del s, r, lane
        gc.collect()
        torch.cuda.empty_cache()
    assert used["1"] > 0 and used["1"] < 0.7 * used["0"], used


def test_bf16_ingest_is_bit_identical_to_fp32_feed(resnet50, monkeypatch):
    """The stem rounds its fp32 input to bf16 itself, so the runner stages the
    request as bf16 (half the pinned / PCIe / device bytes) and the outputs are
    the same bits as feeding fp32 (same tile picks: autotuning off)."""
    from rust_tensorflow_serving2_amd import ops
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    from rust_tensorflow_serving2_amd.utils import tensors as T
    monkeypatch.setattr(ops, "AUTOTUNE", False)
    x = np.random.default_rng(9).random((4, 224, 224, 3), dtype=np.float32) * 255.0
    # denormal pixels too: the host rounds them to bf16 denormals, as the
    # stem's device conversion does (csrc/ingest.h)
    x[0, :8, :8, :] = np.float32(3e-39)
    x[1, 100:104, 50:60, 1] = np.float32(-1.1e-38)
    outs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("TFSERVE_BF16_INGEST", mode)
        s = Servable("resnet", 1, resnet50, ServableOptions(device="cuda:0", max_batch_size=4,
                                                              allowed_batch_sizes=(4,), graph_autotune=False))
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        assert r.slot_dtypes == [T.DT_BFLOAT16 if mode == "1" else T.DT_FLOAT]
        assert r.lanes[0].host_in[0].dtype == (torch.bfloat16 if mode == "1" else torch.float32)
        outs[mode] = r.run([x])
    np.testing.assert_array_equal(outs["0"][0], outs["1"][0])
    np.testing.assert_array_equal(outs["0"][1], outs["1"][1])


def test_small_buckets_write_their_rows_to_the_host(resnet50, monkeypatch):
    """Buckets of <= 4 rows: the one-launch classifier head stores the
    probabilities and classes straight into the lane's pinned output rows
    inside the graph, so the lane skips their D2H copies (two ~4.5-us blit
    kernels at batch 1); runner outputs match TFSERVE_HEAD_HOST=0, and the
    b32 bucket keeps its copies."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    x = np.random.default_rng(11).random((4, 224, 224, 3), dtype=np.float32)
    got, written = {}, {}
    for mode in ("0", "1"):
        monkeypatch.setenv("TFSERVE_HEAD_HOST", mode)
        s = Servable("resnet", 1, resnet50, ServableOptions(
            device="cuda:0", max_batch_size=32, allowed_batch_sizes=(1, 4, 32), lanes=1))
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        got[mode] = [r.run([x[:n]]) for n in (1, 3, 4, 1)]
        r.run([np.concatenate([x] * 8)])                     # the b32 bucket
        written[mode] = dict(r.lanes[0].host_written)
        s.unload() if hasattr(s, "unload") else None
    assert written["1"][1] == [True, True] and written["1"][4] == [True, True], written
    assert written["1"][32] == [False, False] and not any(any(v) for v in written["0"].values()), written
    for a, b in zip(got["0"], got["1"]):
        np.testing.assert_allclose(a[1], b[1], atol=2e-4, rtol=0)
        assert a[1].shape == b[1].shape and a[0].shape == b[0].shape
        top2 = np.sort(a[1], -1)[:, -2:]
        clear = (top2[:, 1] - top2[:, 0]) > 1e-3
        np.testing.assert_array_equal(a[0][clear], b[0][clear])


def test_small_buckets_copy_their_inputs_inside_the_graph(resnet50, monkeypatch):
    """Buckets of <= 4 rows: the graph's first node copies the lane's pinned
    input rows (``h2d_rows``), so the lane issues no SDMA copy ahead of the
    replay.  Distinct inputs through the same rows, bucket after bucket, give
    the outputs of the lane-side copy (TFSERVE_GRAPH_H2D_MAX=0); b32 keeps
    the lane-side copy."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    rng = np.random.default_rng(12)
    xs = [rng.random((4, 224, 224, 3), dtype=np.float32) for _ in range(4)]
    got, captured = {}, {}
    for mode in ("0", "4"):
        monkeypatch.setenv("TFSERVE_GRAPH_H2D_MAX", mode)
        s = Servable("resnet", 1, resnet50, ServableOptions(
            device="cuda:0", max_batch_size=32, allowed_batch_sizes=(1, 4, 32), lanes=1))
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        got[mode] = [r.run([x[:n]]) for x in xs for n in (1, 3, 4, 1)]
        got[mode].append(r.run([np.concatenate([xs[0]] * 8)]))
        captured[mode] = dict(r.lanes[0].in_captured)
    assert captured["4"] == {1: True, 4: True, 32: False} and not any(captured["0"].values()), captured
    for a, b in zip(got["0"], got["4"]):
        np.testing.assert_allclose(a[1], b[1], atol=2e-4, rtol=0)
        top2 = np.sort(a[1], -1)[:, -2:]
        clear = (top2[:, 1] - top2[:, 0]) > 1e-3
        np.testing.assert_array_equal(a[0][clear], b[0][clear])
    # the four inputs differ, so a stale row would show: their outputs must too
    assert not np.allclose(got["4"][0][1], got["4"][4][1], atol=1e-3)
