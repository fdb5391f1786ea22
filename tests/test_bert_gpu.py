"""BERT-base (random init) on the GPU runtime vs the fp32 CPU reference
(BASELINE config 3 shape: seq 128, bf16 fused kernels)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


@pytest.fixture(scope="module")
def bert_base(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import bert
    path = os.path.join(str(tmp_path_factory.mktemp("bert")), "1")
    bert.export(path, seed=0)
    return path


def test_bert_matmul_ln_opt_in_matches_cpu(bert_base, monkeypatch):
    """TFSERVE_MATMUL_LN=1: the 12 attention-output LayerNorms ride on their
    GEMM (_FusedMatMulLN; each bucket still times it against the two launches)
    and the program matches the CPU one."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    monkeypatch.setenv("TFSERVE_MATMUL_LN", "1")
    gpu = Servable("bert", 1, bert_base, ServableOptions(device="cuda:0", max_batch_size=8))
    cpu = Servable("bert", 1, bert_base, ServableOptions(device="cpu"))
    rng = np.random.default_rng(1)
    feeds = {"input_ids": rng.integers(0, 30522, (2, 128)).astype(np.int32),
             "input_mask": np.ones((2, 128), np.int32), "segment_ids": np.zeros((2, 128), np.int32)}
    outs = ["pooled_output", "probabilities"]
    g = gpu.run("serving_default", feeds, outs)
    c = cpu.run("serving_default", feeds, outs)
    assert np.abs(g["pooled_output"] - c["pooled_output"]).max() < 5e-2
    hist = next(iter(gpu._runners.values())).program.op_histogram()
    assert hist["_FusedMatMulLN"] == 12 and hist["_LayerNorm"] == 12


@pytest.mark.parametrize("defer_ln", [True, False])
def test_bert_base_gpu_matches_cpu(bert_base, defer_ln, monkeypatch):
    """defer_ln: the encoder LayerNorms folded into their GEMMs
    (graph/fused.py defer_layernorm, opt-in) or run as kernels (default)."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    monkeypatch.setenv("TFSERVE_DEFER_LN", "1" if defer_ln else "0")
    gpu = Servable("bert", 1, bert_base, ServableOptions(device="cuda:0", max_batch_size=8))
    cpu = Servable("bert", 1, bert_base, ServableOptions(device="cpu"))
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 30522, (4, 128)).astype(np.int32)
    mask = np.ones((4, 128), np.int32)
    mask[2, 77:] = 0
    seg = np.zeros((4, 128), np.int32)
    seg[:, 64:] = 1
    feeds = {"input_ids": ids, "input_mask": mask, "segment_ids": seg}
    outs = ["pooled_output", "probabilities"]
    g = gpu.run("serving_default", feeds, outs)
    c = cpu.run("serving_default", feeds, outs)
    err = np.abs(g["pooled_output"] - c["pooled_output"]).max()
    assert err < 5e-2, err
    assert np.abs(g["probabilities"] - c["probabilities"]).max() < 1e-2
    runner = next(iter(gpu._runners.values()))
    hist = runner.program.op_histogram()
    assert hist["_Attention"] == 12 and hist["_FusedQKV"] == 12
    # deferred: only the last one stays (the pooler reads its output as a strided view)
    assert hist["_LayerNorm"] == (1 if defer_ln else 24)
    assert "_FusedMatMulLN" not in hist        # fuse_matmul_layernorm is opt-in (measured slower)
    assert hist["_EmbeddingLN"] == 1 and hist["_KeyMaskAdder"] == 1 and "GatherV2" not in hist


@pytest.mark.parametrize("seq", [384, 512])
def test_bert_long_sequence_uses_hip_attention(tmp_path, seq):
    """BERT-QA's seq 384 and the full 512 positions: the fused attention runs
    the KV-block kernel (no fp32 torch fallback) and matches the CPU program."""
    from rust_tensorflow_serving2_amd.models import bert
    from rust_tensorflow_serving2_amd.ops import hip
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    cfg = bert.BertConfig(vocab_size=2000, layers=2, seq_len=seq)
    path = os.path.join(str(tmp_path), "1")
    bert.export(path, cfg, seed=1)
    mod = hip()
    orig = mod.attention
    seqs = []

    def spy(qkv, *a):
        seqs.append(qkv.shape[1])
        return orig(qkv, *a)
    mod.attention = spy
    try:
        gpu = Servable("bert", 1, path, ServableOptions(device="cuda:0", max_batch_size=4))
        rng = np.random.default_rng(1)
        ids = rng.integers(0, 2000, (2, seq)).astype(np.int32)
        mask = np.ones((2, seq), np.int32)
        mask[1, seq - 100:] = 0
        feeds = {"input_ids": ids, "input_mask": mask, "segment_ids": np.zeros((2, seq), np.int32)}
        outs = ["pooled_output", "probabilities"]
        g = gpu.run("serving_default", feeds, outs)
    finally:
        mod.attention = orig
    assert seqs and set(seqs) == {seq}, seqs          # the HIP kernel ran (not the torch fallback)
    c = Servable("bert", 1, path, ServableOptions(device="cpu")).run("serving_default", feeds, outs)
    assert np.abs(g["pooled_output"] - c["pooled_output"]).max() < 5e-2
    assert np.abs(g["probabilities"] - c["probabilities"]).max() < 1e-2
