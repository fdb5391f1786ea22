"""HIP kernel numerics vs plain PyTorch fp32 references of the same op (MI355X).

Inputs are bf16-rounded first so the only differences are accumulation order
and the final bf16 rounding of outputs."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402

DEV = torch.device("cuda:0")
BF = torch.bfloat16


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale)


def pack_w(w_hwio):
    kh, kw, cin, cout = w_hwio.shape
    k = kh * kw * cin
    kp = -(-k // 64) * 64
    w = w_hwio.permute(3, 0, 1, 2).reshape(cout, k)
    w = torch.cat([w, torch.zeros(cout, kp - k)], 1)
    return w.to(BF).contiguous().to(DEV)


def ref_conv(x, w_hwio, bias, stride, pads, res=None, act="none"):
    pt, pb, pl, pr = pads
    y = F.conv2d(F.pad(x.float().permute(0, 3, 1, 2), [pl, pr, pt, pb]), w_hwio.float().permute(3, 2, 0, 1),
                 stride=stride).permute(0, 2, 3, 1) + bias
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if act == "relu" else y


CONV_SHAPES = [
    # N, H, W, Cin, Cout, k, stride, pads            (ResNet-50 layers, small batch)
    (2, 56, 56, 64, 64, 1, 1, (0, 0, 0, 0)),
    (2, 56, 56, 64, 64, 3, 1, (1, 1, 1, 1)),
    (2, 56, 56, 64, 256, 1, 1, (0, 0, 0, 0)),
    (2, 56, 56, 256, 128, 1, 1, (0, 0, 0, 0)),
    (2, 56, 56, 128, 128, 3, 2, (1, 1, 1, 1)),
    (2, 56, 56, 256, 512, 1, 2, (0, 0, 0, 0)),
    (3, 14, 14, 256, 256, 3, 1, (1, 1, 1, 1)),
    (1, 7, 7, 512, 2048, 1, 1, (0, 0, 0, 0)),
    (1, 9, 9, 24, 40, 3, 2, (0, 1, 0, 1)),   # odd channels (C % 64 != 0), asymmetric SAME pads
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
@pytest.mark.parametrize("cfg,splits", [(0, 1), (1, 1), (2, 1), (3, 1), (3, 3), (1, 4), (4, 1), (5, 2), (6, 1), (12, 1), (13, 1), (14, 2), (15, 1), (16, 1),
                                        (7, 1), (8, 1), (9, 1), (10, 1), (11, 2)])
def test_conv_matches_fp32(shape, cfg, splits):
    n, h, w, cin, cout, k, s, pads = shape
    x = rnd(n, h, w, cin, seed=1).to(BF)
    wt = rnd(k, k, cin, cout, scale=1 / math.sqrt(k * k * cin), seed=2).to(BF).float()
    b = rnd(cout, scale=0.1, seed=3)
    ho = (h + pads[0] + pads[1] - k) // s + 1
    wo = (w + pads[2] + pads[3] - k) // s + 1
    res = rnd(n, ho, wo, cout, seed=4).to(BF)
    y = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV), k, k, s, s, *pads, act=ACT["relu"], cfg=cfg,
                     splits=splits)
    ref = ref_conv(x, wt, b, s, pads, res, "relu")
    torch.cuda.synchronize()
    err = (y.float().cpu() - ref).abs().max().item()
    assert y.shape == (n, ho, wo, cout)
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err


CGEMM_CFGS = list(range(32, 48)) + list(range(64, 76)) + list(range(96, 107)) + list(range(112, 124))
CGEMM_CONV_SHAPES = [s for s in CONV_SHAPES if s[3] % 64 == 0] + [
    (2, 7, 7, 512, 512, 3, 1, (1, 1, 1, 1)),   # tiny image: most taps hit padding at the border rows
    (1, 15, 13, 64, 192, 3, 2, (0, 1, 1, 1)),  # odd sizes, asymmetric pads, N tail
]


@pytest.mark.parametrize("shape", CGEMM_CONV_SHAPES)
@pytest.mark.parametrize("cfg", CGEMM_CFGS)
def test_cgemm_conv_matches_fp32(shape, cfg):
    """Pipelined cgemm kernel (im2col with C % 64 == 0 and 1x1 dense) vs fp32 conv."""
    n, h, w, cin, cout, k, s, pads = shape
    x = rnd(n, h, w, cin, seed=1).to(BF)
    wt = rnd(k, k, cin, cout, scale=1 / math.sqrt(k * k * cin), seed=2).to(BF).float()
    b = rnd(cout, scale=0.1, seed=3)
    ho = (h + pads[0] + pads[1] - k) // s + 1
    wo = (w + pads[2] + pads[3] - k) // s + 1
    res = rnd(n, ho, wo, cout, seed=4).to(BF)
    ref = ref_conv(x, wt, b, s, pads, res, "relu")
    for splits in (1, 3):
        y = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV), k, k, s, s, *pads, act=ACT["relu"],
                         cfg=cfg, splits=splits)
        torch.cuda.synchronize()
        err = (y.float().cpu() - ref).abs().max().item()
        assert y.shape == (n, ho, wo, cout)
        assert err < 3e-2 * max(1.0, ref.abs().max().item()), (splits, err)


HALO_CFGS = list(range(48, 59)) + [80, 81, 82, 83, 85, 86, 87, 88, 89, 90]
HALO_SHAPES = [
    # N, H, W, Cin, Cout, pads            (3x3 stride 1; ResNet-50 stages + edge cases)
    (2, 56, 56, 64, 64, (1, 1, 1, 1)),
    (2, 28, 28, 128, 128, (1, 1, 1, 1)),
    (3, 14, 14, 256, 256, (1, 1, 1, 1)),
    (2, 7, 7, 512, 512, (1, 1, 1, 1)),
    (1, 13, 17, 192, 72, (1, 1, 1, 1)),    # odd image, 3 chunks, N tail (72 % BN != 0)
    (2, 9, 11, 64, 136, (0, 0, 0, 0)),     # VALID (no padding)
    (1, 5, 6, 128, 64, (2, 0, 1, 1)),      # asymmetric top pad
    (5, 7, 7, 128, 64, (1, 1, 1, 1)),      # whole-image tiles: up to 3 images per tile, last tile partial
    (4, 6, 5, 64, 72, (0, 2, 1, 1)),       # whole-image tiles with asymmetric pads
]


@pytest.mark.parametrize("shape", HALO_SHAPES)
@pytest.mark.parametrize("cfg", HALO_CFGS)
def test_halo_conv_matches_fp32(shape, cfg):
    """Halo-tiled 3x3 stride-1 conv (one input halo per 64-channel chunk, nine
    shifted taps from LDS) vs fp32 conv, with bias + residual + ReLU and split-K."""
    n, h, w, cin, cout, pads = shape
    x = rnd(n, h, w, cin, seed=11).to(BF)
    wt = rnd(3, 3, cin, cout, scale=1 / math.sqrt(9 * cin), seed=12).to(BF).float()
    b = rnd(cout, scale=0.1, seed=13)
    ho = h + pads[0] + pads[1] - 2
    wo = w + pads[2] + pads[3] - 2
    res = rnd(n, ho, wo, cout, seed=14).to(BF)
    ref = ref_conv(x, wt, b, 1, pads, res, "relu")
    for splits in (1, 2, 3):
        y = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV), 3, 3, 1, 1, *pads, act=ACT["relu"],
                         cfg=cfg, splits=splits)
        torch.cuda.synchronize()
        err = (y.float().cpu() - ref).abs().max().item()
        assert y.shape == (n, ho, wo, cout)
        assert err < 3e-2 * max(1.0, ref.abs().max().item()), (splits, err)


@pytest.mark.parametrize("shape", [
    (32, 56, 56, (1, 1, 1, 1)),      # ResNet-50 stage 1 at b32: 896 tiles, 3-4 per workgroup
    (3, 56, 56, (1, 1, 1, 1)),       # fewer tiles than CUs
    (5, 7, 7, (1, 1, 1, 1)),         # whole-image tiles (several images per tile, last tile partial)
    (2, 13, 17, (0, 2, 1, 1)),       # odd image, asymmetric pads
])
@pytest.mark.parametrize("act", ["relu", "none"])
def test_halo_persist_matches_fp32(shape, act):
    """Persistent halo conv (config 146: the 64 x 64 x 3 x 3 filter resident in
    LDS, each workgroup walking several tiles with double-buffered halos and its
    stores draining under the next tile) vs fp32; it takes the plain bf16
    output only and rejects residual / other channel counts."""
    n, h, w, pads = shape
    x = rnd(n, h, w, 64, seed=21).to(BF)
    wt = rnd(3, 3, 64, 64, scale=1 / math.sqrt(9 * 64), seed=22).to(BF).float()
    b = rnd(64, scale=0.1, seed=23)
    ho, wo = h + pads[0] + pads[1] - 2, w + pads[2] + pads[3] - 2
    ref = ref_conv(x, wt, b, 1, pads, None, act)
    y = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), None, 3, 3, 1, 1, *pads, act=ACT[act], cfg=146)
    y2 = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), None, 3, 3, 1, 1, *pads, act=ACT[act], cfg=146)
    torch.cuda.synchronize()
    assert y.shape == (n, ho, wo, 64)
    assert (y.float().cpu() - ref).abs().max().item() < 3e-2 * max(1.0, ref.abs().max().item())
    assert torch.equal(y, y2)
    res = rnd(n, ho, wo, 64, seed=24).to(BF)
    with pytest.raises(RuntimeError):
        hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV), 3, 3, 1, 1, *pads, act=ACT[act], cfg=146)
    # a split request over the single 64-channel chunk runs unsplit (the binding clamps it)
    y3 = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), None, 3, 3, 1, 1, *pads, act=ACT[act], cfg=146, splits=2)
    torch.cuda.synchronize()
    assert torch.equal(y, y3)
    x2 = rnd(1, 8, 8, 128, seed=25).to(BF)
    w2 = rnd(3, 3, 128, 64, scale=0.03, seed=26).to(BF).float()
    with pytest.raises(RuntimeError):
        hip().conv2d(x2.to(DEV), pack_w(w2), b.to(DEV), None, 3, 3, 1, 1, 1, 1, 1, 1, act=ACT[act], cfg=146)


def test_halo_exact_identity_taps():
    """Integer-valued operands (exact in bf16 and fp32): every output pixel of
    every tile position, tap and channel chunk must match bit for bit — catches
    a mis-shifted halo row or a wrong swizzle that tolerances could hide."""
    n, h, w, cin, cout = 2, 19, 23, 128, 64
    g = torch.Generator().manual_seed(5)
    x = torch.randint(-3, 4, (n, h, w, cin), generator=g).float()
    wt = torch.randint(-2, 3, (3, 3, cin, cout), generator=g).float()
    ref = ref_conv(x, wt, torch.zeros(cout), 1, (1, 1, 1, 1))
    for cfg in HALO_CFGS:
        y = hip().conv2d(x.to(BF).to(DEV), pack_w(wt), None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=cfg,
                         out_f32=True)
        assert torch.equal(y.cpu(), ref), cfg


def test_halo_rejects_non_3x3():
    x = torch.zeros(1, 8, 8, 64, device=DEV, dtype=BF)
    w = torch.zeros(64, 64 * 9, device=DEV, dtype=BF)
    with pytest.raises(RuntimeError, match="halo config"):
        hip().conv2d(x, w, None, None, 3, 3, 2, 2, 1, 1, 1, 1, act=0, cfg=48)


@pytest.mark.parametrize("m,n,k", [(32, 1000, 2048), (256, 2304, 768), (1000, 768, 3072), (8, 72, 64)])
@pytest.mark.parametrize("cfg", CGEMM_CFGS)
def test_cgemm_linear_matches_fp32(m, n, k, cfg):
    x = rnd(m, k, seed=7).to(BF)
    w = rnd(n, k, scale=1 / math.sqrt(k), seed=8).to(BF)
    b = rnd(n, scale=0.1, seed=9)
    res = rnd(m, n, seed=10).to(BF)
    ref = x.float() @ w.float().t() + b + res.float()
    for act, fn, out_f32 in (("none", lambda t: t, False), ("relu", torch.relu, True),
                             ("gelu_tanh", lambda t: F.gelu(t, approximate="tanh"), False),
                             ("gelu_erf", F.gelu, True), ("tanh", torch.tanh, False)):
        y = hip().linear(x.to(DEV), w.to(DEV), b.to(DEV), res.to(DEV), ACT[act], cfg, out_f32)
        err = (y.float().cpu() - fn(ref)).abs().max().item()
        assert err < 3e-2 * max(1.0, ref.abs().max().item()), (act, err)


@pytest.mark.parametrize("cfg", CGEMM_CFGS + [140, 141, 142])
def test_cgemm_asymmetric_identity(cfg):
    """A = I, asymmetric B (exact in bf16 / fp32): catches a transposed or
    swizzle-permuted C tile in every cgemm config."""
    m, n, k = 256, 256, 128
    a = torch.eye(m, k).to(BF)
    bmat = (torch.arange(n * k, dtype=torch.float32).reshape(n, k) % 17 - 8)
    y = hip().linear(a.to(DEV), bmat.to(BF).to(DEV), None, None, 0, cfg, True)
    assert torch.equal(y.cpu(), a.float() @ bmat.t())


@pytest.mark.parametrize("n,ho,c1,h,c2,s,cout", [(2, 56, 64, 56, 64, 1, 256), (2, 28, 128, 56, 256, 2, 512),
                                                 (1, 7, 512, 14, 1024, 2, 2048), (1, 5, 64, 9, 128, 2, 72)])
@pytest.mark.parametrize("cfg", [32, 36, 42, 43, 44, 45, 47, 112, 114, 117, 121])
def test_conv2d_dual_matches_fp32(n, ho, c1, h, c2, s, cout, cfg):
    """One GEMM for a bottleneck tail: relu(conv1x1(h) + conv1x1_stride(x) + b)."""
    hh = rnd(n, ho, ho, c1, seed=21).to(BF)
    x = rnd(n, h, h, c2, seed=22).to(BF)
    w1 = rnd(cout, c1, scale=1 / math.sqrt(c1), seed=23).to(BF)
    w2 = rnd(cout, c2, scale=1 / math.sqrt(c2), seed=24).to(BF)
    b = rnd(cout, scale=0.1, seed=25)
    w = torch.cat([w1, w2], 1).contiguous()
    ref = torch.relu(hh.float() @ w1.float().t() + x.float()[:, ::s, ::s, :] @ w2.float().t() + b)
    for splits in (1, 2):
        y = hip().conv2d_dual(hh.to(DEV), x.to(DEV), w.to(DEV), b.to(DEV), s, s, ACT["relu"], cfg, None, splits)
        err = (y.float().cpu() - ref).abs().max().item()
        assert y.shape == (n, ho, ho, cout)
        assert err < 3e-2 * max(1.0, ref.abs().max().item()), (splits, err)


def test_cgemm_rejects_unaligned():
    """cgemm configs refuse (loudly) operands that are not 64-aligned (K) or
    whose output rows are not 16-B chunks (N % 8)."""
    x = torch.zeros(4, 40, device=DEV, dtype=BF)
    w = torch.zeros(8, 40, device=DEV, dtype=BF)
    with pytest.raises(RuntimeError, match="64-aligned"):
        hip().linear(x, w, None, None, 0, 32, False)
    x = torch.zeros(4, 64, device=DEV, dtype=BF)
    w = torch.zeros(12, 64, device=DEV, dtype=BF)
    with pytest.raises(RuntimeError, match="64-aligned"):
        hip().linear(x, w, None, None, 0, 32, True)


@pytest.mark.parametrize("k,c,cfg", [(7, 3, 1), (7, 3, 0), (3, 3, 3), (5, 4, 1)])
def test_stem_conv_fp32_input(k, c, cfg):
    """fp32 request tensor with few channels: the ingest cast is fused into the
    operand gather (7x7x3 = specialised ResNet stem loader; others generic)."""
    x = torch.rand(2, 33, 31, c)
    wt = rnd(k, k, c, 64, scale=0.1, seed=5).to(BF).float()
    b = rnd(64, scale=0.1, seed=6)
    pads = (k // 2 - 1, k // 2, k // 2 - 1, k // 2)
    y = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), None, k, k, 2, 2, *pads, act=ACT["relu"], cfg=cfg)
    ref = ref_conv(x.to(BF).float(), wt, b, 2, pads, None, "relu")
    assert y.shape == ref.shape
    assert (y.float().cpu() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("k,c", [(7, 3), (3, 3), (5, 4), (7, 1)])
def test_rgba_stem_path(k, c):
    """ingest_c4 (fp32 RGB -> bf16 RGBA) + kAC4 gather with [Cout][kh][8][4] weights."""
    x = torch.rand(3, 37, 29, c)
    wt = rnd(k, k, c, 64, scale=0.1, seed=7).to(BF).float()
    b = rnd(64, scale=0.1, seed=8)
    w4 = torch.zeros(k, 8, 4, 64)
    w4[:, :k, :c, :] = wt
    wp = w4.permute(3, 0, 1, 2).reshape(64, k * 32)
    kp = -(-k * 32 // 64) * 64
    wp = torch.cat([wp, torch.zeros(64, kp - k * 32)], 1).to(BF).contiguous().to(DEV)
    x4 = hip().ingest_c4(x.to(DEV))
    assert x4.shape == (3, 37, 29, 4) and torch.equal(x4[..., :c].float().cpu(), x.to(BF).float())
    pads = (k // 2 - 1, k // 2, k // 2 - 1, k // 2) if k > 1 else (0, 0, 0, 0)
    for cfg in (1, 3):
        y = hip().conv2d(x4, wp, b.to(DEV), None, k, k, 2, 2, *pads, act=ACT["relu"], cfg=cfg)
        ref = ref_conv(x.to(BF).float(), wt, b, 2, pads, None, "relu")
        assert (y.float().cpu() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("k,c,s", [(7, 3, 2), (3, 3, 1), (5, 4, 2), (1, 3, 1)])
@pytest.mark.parametrize("cfg", [36, 42, 43, 44, 32, 112, 114])
def test_cgemm_padded_rgba_stem(k, c, s, cfg):
    """ingest_c4_padded (zero-bordered bf16 RGBA) + cgemm stem mode (even kh,
    8 taps: every operand chunk is two in-bounds pixels) vs the fp32 conv."""
    n, h, w = 3, 37, 29
    x = torch.rand(n, h, w, c)
    wt = rnd(k, k, c, 64, scale=0.1, seed=17).to(BF).float()
    b = rnd(64, scale=0.1, seed=18)
    pt, pb, pl, pr = k // 2, (k - 1) // 2, k // 2, (k - 1) // 2
    ho, wo = (h + pt + pb - k) // s + 1, (w + pl + pr - k) // s + 1
    khp = k + k % 2
    w4 = torch.zeros(khp, 8, 4, 64)
    w4[:k, :k, :c, :] = wt
    wp = w4.permute(3, 0, 1, 2).reshape(64, khp * 32).to(BF).contiguous().to(DEV)
    xp = hip().ingest_c4_padded(x.to(DEV), (ho - 1) * s + khp, (wo - 1) * s + 8, pt, pl)
    y = hip().conv2d(xp, wp, b.to(DEV), None, khp, 8, s, s, 0, 0, 0, 0, act=ACT["relu"], cfg=cfg)
    ref = ref_conv(x.to(BF).float(), wt, b, s, (pt, pb, pl, pr), None, "relu")
    assert y.shape == ref.shape
    assert (y.float().cpu() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("n,h,w,c,hp,wp,pt,pl", [(3, 37, 29, 3, 44, 40, 3, 3), (2, 5, 300, 4, 7, 310, 1, 2),
                                                  (32, 224, 224, 3, 230, 232, 3, 3), (1, 3, 3, 1, 3, 3, 0, 0)])
def test_ingest_c4_padded_exact(n, h, w, c, hp, wp, pt, pl):
    x = torch.rand(n, h, w, c) * 4 - 2
    y = hip().ingest_c4_padded(x.to(DEV), hp, wp, pt, pl).cpu()
    ref = torch.zeros(n, hp, wp, 4, dtype=BF)
    ref[:, pt:pt + h, pl:pl + w, :c] = x.to(BF)
    assert y.shape == ref.shape and torch.equal(y.view(torch.int16), ref.view(torch.int16))


def test_asymmetric_identity_gemm():
    """A = I, asymmetric B: catches a transposed C write (guide §3)."""
    m = n = 64
    a = torch.eye(m, 128)[:, :128].to(BF)
    bmat = torch.arange(n * 128, dtype=torch.float32).reshape(n, 128) % 17 - 8
    y = hip().linear(a.to(DEV), bmat.to(BF).to(DEV), None, None, 0, 3, True)
    ref = a.float() @ bmat.t()
    assert torch.equal(y.cpu(), ref)


@pytest.mark.parametrize("m,n,k,act", [(32, 1001, 2048, "none"), (256, 2304, 768, "none"),
                                       (256, 3072, 768, "gelu_tanh"), (256, 768, 3072, "none"),
                                       (8, 768, 768, "tanh"), (100, 72, 40, "gelu_erf")])
@pytest.mark.parametrize("cfg,splits", [(0, 1), (3, 1), (3, 8), (1, 3), (5, 1), (8, 1), (9, 2), (10, 1), (11, 1), (12, 1), (13, 3), (16, 1)])
def test_linear_matches_fp32(m, n, k, act, cfg, splits):
    x = rnd(m, k, seed=7).to(BF)
    w = rnd(n, k, scale=1 / math.sqrt(k), seed=8).to(BF)
    b = rnd(n, scale=0.1, seed=9)
    res = rnd(m, n, seed=10).to(BF) if act == "none" else None
    out_f32 = n % 8 != 0
    y = hip().linear(x.to(DEV), w.to(DEV), b.to(DEV), None if res is None else res.to(DEV), ACT[act], cfg, out_f32,
                     splits=splits)
    ref = x.float() @ w.float().t() + b
    if res is not None:
        ref = ref + res.float()
    ref = {"none": ref, "gelu_tanh": F.gelu(ref, approximate="tanh"), "gelu_erf": F.gelu(ref),
           "tanh": torch.tanh(ref)}[act]
    err = (y.float().cpu() - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("cfg", [140, 141, 142])
@pytest.mark.parametrize("m,n,k,act,splits,mode", [
    (4096, 2304, 768, "none", 1, "bf16"),          # BERT QKV (256 x 256: 16 x 9 tiles)
    (4096, 3072, 768, "gelu_tanh", 1, "bf16"),     # FFN1
    (4096, 768, 3072, "none", 1, "residual"),      # FFN2 + residual, the two-pass fp32 epilogue
    (4096, 768, 3072, "none", 4, "bf16"),          # split-K slabs + reduce launch
    (300, 264, 64, "relu", 1, "bf16"),             # one k-tile; partial tiles in M and N
    (520, 136, 192, "tanh", 1, "f32"),             # odd k-tile count, fp32 output
    (777, 1000, 640, "none", 3, "residual"),       # ragged everything, split-K with residual
])
def test_bgemm_matches_fp32(m, n, k, act, splits, mode, cfg):
    """The big-tile ping-pong GEMM (kernels/bgemm.hip) against an fp32 matmul:
    every epilogue path (one-pass bf16, two-pass fp32 with residual / fp32
    output, split-K slabs), ragged M / N edges and k-tile counts of 1..48."""
    x = rnd(m, k, seed=m + k).to(BF)
    w = rnd(n, k, scale=1 / math.sqrt(k), seed=n + 1).to(BF)
    b = rnd(n, scale=0.1, seed=n + 2)
    res = rnd(m, n, seed=m + 3).to(BF) if mode == "residual" else None
    y = hip().linear(x.to(DEV), w.to(DEV), b.to(DEV), None if res is None else res.to(DEV), ACT[act], cfg,
                     mode == "f32", splits=splits)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t() + b
    if res is not None:
        ref = ref + res.float()
    ref = {"none": ref, "relu": F.relu(ref), "gelu_tanh": F.gelu(ref, approximate="tanh"),
           "tanh": torch.tanh(ref)}[act]
    err = (y.float().cpu() - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err


def test_bgemm_rejects_non_dense_and_is_deterministic():
    """bgemm takes dense operands only (a conv operand mode is a host-side
    rejection the tuner skips), and repeated launches are bit-identical (no
    read of a half-tile before its DMA landed)."""
    x = rnd(1024, 512, seed=5).to(BF).to(DEV)
    w = rnd(768, 512, scale=0.05, seed=6).to(BF).to(DEV)
    ys = [hip().linear(x, w, None, None, 0, 140, False) for _ in range(8)]
    torch.cuda.synchronize()
    for y in ys[1:]:
        assert torch.equal(y, ys[0])
    xc = rnd(2, 8, 8, 64, seed=7).to(BF).to(DEV)
    wc = pack_w(rnd(3, 3, 64, 64, scale=0.05, seed=8).to(BF).float())
    with pytest.raises(RuntimeError):
        hip().conv2d(xc, wc, None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=140)


@pytest.mark.parametrize("n,h,w,c,k,st,pt,pb", [(2, 9, 13, 8, 3, 2, 1, 1), (3, 17, 5, 520, 2, 2, 0, 1),
                                                 (1, 30, 30, 2048, 3, 1, 1, 1), (32, 112, 112, 64, 3, 2, 0, 1)])
def test_maxpool_shapes(n, h, w, c, k, st, pt, pb):
    x = rnd(n, h, w, c, seed=h * w + c).to(BF)
    y = hip().maxpool(x.to(DEV), k, k, st, st, pt, pb, pt, pb)
    ref = F.max_pool2d(F.pad(x.float().permute(0, 3, 1, 2), [pt, pb, pt, pb], value=-1e30), k, st)
    assert torch.equal(y.float().cpu(), ref.permute(0, 2, 3, 1))


def test_pools_and_head():
    x = rnd(4, 112, 112, 64, seed=11).to(BF)
    y = hip().maxpool(x.to(DEV), 3, 3, 2, 2, 0, 1, 0, 1)
    ref = F.max_pool2d(F.pad(x.float().permute(0, 3, 1, 2), [0, 1, 0, 1], value=-1e30), 3, 2).permute(0, 2, 3, 1)
    assert torch.equal(y.float().cpu(), ref)
    g = rnd(4, 7, 7, 2048, seed=12).to(BF)
    gy = hip().global_avgpool(g.to(DEV))
    assert (gy.float().cpu() - g.float().mean((1, 2))).abs().max() < 1e-2
    logits = rnd(37, 1001, scale=3, seed=13)
    logits[5, 7] = logits[5, 9] = 100.0          # tie -> smallest index (TF ArgMax)
    p, c = hip().softmax_argmax(logits.to(DEV))
    assert torch.allclose(p.cpu(), torch.softmax(logits, -1), atol=1e-6)
    assert torch.equal(c.cpu(), torch.argmax(logits, -1)) and c[5].item() == 7


@pytest.mark.parametrize("rows,cols", [(3, 5000), (2, 10), (1, 4096)])
def test_softmax_argmax_shapes(rows, cols):
    logits = rnd(rows, cols, scale=4, seed=rows + cols)
    p, c = hip().softmax_argmax(logits.to(DEV))
    assert torch.allclose(p.cpu(), torch.softmax(logits, -1), atol=1e-6)
    assert torch.equal(c.cpu(), torch.argmax(logits, -1))


@pytest.mark.parametrize("cols", [1001, 5000])
def test_softmax_argmax_row_strided(cols):
    """Logits as the first `cols` columns of a padded [rows, ceil8(cols)] GEMM
    output (the ResNet FC with N padded to a multiple of 8)."""
    ld = -(-cols // 8) * 8 + 8
    full = rnd(7, ld, scale=4, seed=cols)
    full[:, cols:] = 1e4                     # padding columns must never be read
    view = full.to(DEV)[:, :cols]
    p, c = hip().softmax_argmax(view)
    logits = full[:, :cols]
    assert torch.allclose(p.cpu(), torch.softmax(logits, -1), atol=1e-6)
    assert torch.equal(c.cpu(), torch.argmax(logits, -1))


def test_linear_padded_n_feeds_softmax():
    """FusedMatMul with N = 1001 padded to 1008 (cgemm) == fp32 reference."""
    from rust_tensorflow_serving2_amd.graph.fused import FusedMatMul
    w = rnd(2048, 1001, scale=0.03, seed=51)
    b = rnd(1001, scale=0.1, seed=52)
    x = rnd(32, 2048, seed=53).to(BF)
    mm = FusedMatMul(w, b, "none", True, torch.device(DEV), True, "fc", pad_n=True)
    assert mm.np == 1008
    y = mm(None, None, [x.to(DEV)])[0]
    assert y.shape == (32, 1001) and y.stride(0) == 1008
    ref = x.float() @ w.to(BF).float() + b
    assert (y.cpu() - ref).abs().max() < 3e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("n,hw,c", [(3, 1, 72), (2, 9, 520), (1, 49, 4096)])
def test_global_avgpool_shapes(n, hw, c):
    g = rnd(n, hw, 1, c, seed=hw + c).to(BF)
    gy = hip().global_avgpool(g.to(DEV))
    assert (gy.float().cpu() - g.float().mean((1, 2))).abs().max() < 1e-2


def test_layernorm_and_embedding():
    x = rnd(300, 768, seed=14).to(BF)
    r = rnd(300, 768, seed=15).to(BF)
    gm, bt = rnd(768, seed=16), rnd(768, seed=17)
    y = hip().layernorm(x.to(DEV), r.to(DEV), gm.to(DEV), bt.to(DEV), 1e-12)
    ref = F.layer_norm(x.float() + r.float(), (768,), gm, bt, 1e-12)
    assert (y.float().cpu() - ref).abs().max() < 5e-2
    ids = torch.randint(0, 1000, (3, 128), dtype=torch.int32)
    tt = torch.randint(0, 2, (3, 128), dtype=torch.int32)
    word, pos, typ = rnd(1000, 768, seed=18).to(BF), rnd(512, 768, seed=19).to(BF), rnd(2, 768, seed=20).to(BF)
    e = hip().embed_ln(ids.to(DEV), tt.to(DEV), word.to(DEV), pos.to(DEV), typ.to(DEV), gm.to(DEV), bt.to(DEV),
                       1e-12, 128)
    ref = F.layer_norm(word.float()[ids.long()] + pos.float()[:128] + typ.float()[tt.long()], (768,), gm, bt, 1e-12)
    assert e.shape == (3, 128, 768)
    assert (e.float().cpu() - ref).abs().max() < 5e-2


@pytest.mark.parametrize("m,n,k", [(4096, 768, 768), (100, 768, 768), (33, 512, 1024), (70, 1024, 256),
                                   (17, 768, 3072)])
@pytest.mark.parametrize("bm", [16, 32, 64])
@pytest.mark.parametrize("res,bias", [(True, True), (False, False)])
def test_linear_ln_matches_fp32(m, n, k, bm, res, bias):
    """GEMM + residual + LayerNorm in one launch (kernels/lngemm.hip): whole
    rows per workgroup (bm rows), partial last workgroups, offset rows (the
    two-pass variance), against LN(x w^T + b + r) in fp32."""
    if not hip().linear_ln_supported(m, n, k, bm):
        with pytest.raises(RuntimeError):
            hip().linear_ln(torch.zeros(m, k, dtype=BF, device=DEV), torch.zeros(n, k, dtype=BF, device=DEV),
                            None, None, torch.ones(n, device=DEV), torch.zeros(n, device=DEV), 1e-12, bm)
        return
    x = rnd(m, k, seed=61).to(BF)
    w = (rnd(n, k, seed=62) / math.sqrt(k)).to(BF)
    b = rnd(n, seed=63) if bias else None
    r = (rnd(m, n, seed=64) * 2 + 3).to(BF) if res else None
    gm, bt = rnd(n, seed=65), rnd(n, seed=66)
    from rust_tensorflow_serving2_amd.graph.fused import ln_weight_frags
    y = hip().linear_ln(x.to(DEV), ln_weight_frags(w).to(DEV), None if b is None else b.to(DEV),
                        None if r is None else r.to(DEV), gm.to(DEV), bt.to(DEV), 1e-12, bm)
    z = x.float() @ w.float().t()
    if b is not None:
        z = z + b
    if r is not None:
        z = z + r.float()
    ref = F.layer_norm(z, (n,), gm, bt, 1e-12)
    assert y.shape == (m, n) and y.dtype == BF
    assert (y.float().cpu() - ref).abs().max() < 6e-2


@pytest.mark.parametrize("cols", [64, 520, 2048, 4104, 128, 256, 384, 512, 768, 1024])
def test_layernorm_register_and_streaming_paths(cols):
    """Rows up to 2048 columns stay in registers; longer ones stream twice;
    exact-fit widths (128 .. 2048) take the lanes-per-row kernel (37 rows: a
    partial last workgroup)."""
    x = (rnd(37, cols, seed=41) * 3 + 5).to(BF)      # offset mean: the two-pass variance matters
    r = rnd(37, cols, seed=42).to(BF)
    gm, bt = rnd(cols, seed=43), rnd(cols, seed=44)
    y = hip().layernorm(x.to(DEV), r.to(DEV), gm.to(DEV), bt.to(DEV), 1e-5)
    ref = F.layer_norm(x.float() + r.float(), (cols,), gm, bt, 1e-5)
    assert (y.float().cpu() - ref).abs().max() < 6e-2
    y2 = hip().layernorm(x.to(DEV), None, gm.to(DEV), bt.to(DEV), 1e-5)
    assert (y2.float().cpu() - F.layer_norm(x.float(), (cols,), gm, bt, 1e-5)).abs().max() < 6e-2


@pytest.mark.parametrize("hd", [64, 520, 1024, 2048])
def test_embedding_out_of_range_rows_are_zero(hd):
    """Ids outside a table add a zero row (TF's GPU GatherV2); type ids and
    positions are optional; hidden sizes up to 2048 in 8-wide chunks."""
    S = 16
    ids = torch.randint(0, 50, (2 * S,), dtype=torch.int32)
    ids[3], ids[7] = -1, 50
    tt = torch.randint(0, 3, (2 * S,), dtype=torch.int32)
    tt[5] = 9
    word, typ, pos = rnd(50, hd, seed=31).to(BF), rnd(3, hd, seed=32).to(BF), rnd(S, hd, seed=33).to(BF)
    gm, bt = rnd(hd, seed=34), rnd(hd, seed=35)
    wz = torch.cat([word.float(), torch.zeros(1, hd)])
    tz = torch.cat([typ.float(), torch.zeros(1, hd)])
    wi = torch.where((ids >= 0) & (ids < 50), ids, 50).long()
    ti = torch.where((tt >= 0) & (tt < 3), tt, 3).long()
    full = wz[wi] + tz[ti] + pos.float().repeat(2, 1)
    e = hip().embed_ln(ids.to(DEV), tt.to(DEV), word.to(DEV), pos.to(DEV), typ.to(DEV), gm.to(DEV), bt.to(DEV),
                       1e-6, S)
    assert (e.float().cpu() - F.layer_norm(full, (hd,), gm, bt, 1e-6)).abs().max() < 5e-2
    e2 = hip().embed_ln(ids.to(DEV), None, word.to(DEV), None, None, gm.to(DEV), bt.to(DEV), 1e-6, S)
    assert (e2.float().cpu() - F.layer_norm(wz[wi], (hd,), gm, bt, 1e-6)).abs().max() < 5e-2
    with pytest.raises(RuntimeError):
        hip().embed_ln(ids.to(DEV), None, word.to(DEV), None, None, gm.to(DEV), bt.to(DEV), 1e-6, 5)   # 32 % 5


@pytest.mark.parametrize("m,hw,k,np_,n", [(32, 49, 2048, 1001, 1001), (32, 49, 2048, 1008, 1001), (1, 49, 2048, 1001, 1001),
                                         (3, 4, 512, 10, 10), (70, 9, 1024, 300, 257), (5, 1, 4096, 33, 33),
                                         (3, 4, 512, 2000, 1500)])   # > 1024 classes: the 16-per-thread softmax tile
@pytest.mark.parametrize("head_ks", ["4", "8"])
def test_classifier_head_matches_fp32(monkeypatch, head_ks, m, hw, k, np_, n):
    """mean_hw -> dense -> softmax/argmax in two launches (split-K partial rows,
    then bias + partial sums + softmax) vs fp32; rows in several 32-row chunks,
    a weight matrix padded past the n classes read.  TFSERVE_HEAD_KS=8 splits K
    eight ways where K is a multiple of 1024 (four elsewhere)."""
    monkeypatch.setenv("TFSERVE_HEAD_KS", head_ks)
    monkeypatch.setenv("TFSERVE_HEAD_FUSED", "0")            # the three-launch path at every m
    x = rnd(m, hw, 1, k, seed=41).to(BF)
    w = rnd(np_, k, scale=0.05, seed=42).to(BF)
    b = rnd(np_, scale=0.1, seed=43)
    probs, cls = hip().classifier_head(x.to(DEV), w.to(DEV), b.to(DEV), n)
    pooled = x.float().mean(dim=(1, 2)).to(BF).float()        # the kernel pools into bf16 (MFMA operand)
    logits = (pooled @ w.float().t() + b)[:, :n]
    ref = torch.softmax(logits, -1)
    assert probs.shape == (m, n) and cls.shape == (m,)
    assert (probs.cpu() - ref).abs().max() < 1e-4
    top2 = logits.topk(2, -1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3                 # rows whose argmax is not a near-tie
    assert torch.equal(cls.cpu()[clear], logits.argmax(-1)[clear])


@pytest.mark.parametrize("m,hw,k,np_,n", [(1, 49, 2048, 1001, 1001), (2, 49, 2048, 1008, 1001), (4, 64, 1024, 300, 257),
                                         (7, 3, 512, 10, 10), (16, 49, 2048, 1001, 1001),
                                         (2, 9, 512, 2000, 2000)])   # > 1024 classes: the 16-per-thread tile
def test_classifier_head_one_launch_matches_three(monkeypatch, m, hw, k, np_, n):
    """The small-batch head (pool + dense + arrival-counter hand-off + softmax
    in ONE launch, misc.hip head_small_kernel) vs the three-launch head and
    fp32: eager calls back to back (the kernel re-zeroes its counter) and
    replays of a captured graph."""
    x = rnd(m, hw, 1, k, seed=44).to(BF).to(DEV)
    w = rnd(np_, k, scale=0.05, seed=45).to(BF).to(DEV)
    b = rnd(np_, scale=0.1, seed=46).to(DEV)
    monkeypatch.setenv("TFSERVE_HEAD_FUSED", "0")
    p3, c3 = hip().classifier_head(x, w, b, n)
    monkeypatch.setenv("TFSERVE_HEAD_FUSED", "16")
    for _ in range(3):
        p1, c1 = hip().classifier_head(x, w, b, n)
        assert (p1 - p3).abs().max().item() < 1e-6
        assert torch.equal(c1, c3)
    pooled = x.float().cpu().mean(dim=(1, 2)).to(BF).float()
    ref = torch.softmax((pooled @ w.float().cpu().t() + b.cpu())[:, :n], -1)
    assert (p1.cpu() - ref).abs().max() < 1e-4
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hip().classifier_head(x, w, b, n)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        pg, cg = hip().classifier_head(x, w, b, n)
    for _ in range(3):
        pg.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert (pg - p3).abs().max().item() < 1e-6
        assert torch.equal(cg, c3)


@pytest.mark.parametrize("s", [64, 128, 192, 256,
                               32, 100, 320, 384, 512])     # KV-block (online softmax) kernel, partial blocks
@pytest.mark.parametrize("plds", [0, 1])                    # P in registers (default) / through LDS (previous)
def test_attention_matches_fp32(s, plds):
    if plds and s not in (64, 128, 192, 256):
        pytest.skip("the P-through-LDS layout is a fixed-S kernel")
    prev = hip().set_attention_plds(plds)
    try:
        _check_attention(s)
    finally:
        hip().set_attention_plds(prev)


def test_attention_one_workgroup_per_head_at_large_batch():
    """S = 128 with batch x heads >= 256 takes the 128-query-row workgroup
    (8 waves, K / V staged once per (batch, head))."""
    _check_attention(128, b=22)


def _check_attention(s, b=3):
    h, d = 12, 64
    qkv = rnd(b, s, 3 * h * d, seed=21).to(BF)
    mask = torch.zeros(b, s)
    mask[1, s // 2:] = -10000.0
    y = hip().attention(qkv.to(DEV), mask.to(DEV), h, 1 / math.sqrt(d), None, s, 0)   # [B, S] key mask
    q, k, v = qkv.float().reshape(b, s, 3, h, d).permute(2, 0, 3, 1, 4)
    att = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d) + mask[:, None, None, :], -1)
    ref = (att @ v).permute(0, 2, 1, 3).reshape(b, s, h * d)
    assert (y.float().cpu() - ref).abs().max() < 3e-2
    # full per-query mask [B, 1, S, S] (BERT adder layout), causal-style pattern
    full = torch.triu(torch.full((s, s), -10000.0), 1).expand(b, 1, s, s).contiguous()
    y2 = hip().attention(qkv.to(DEV), full.to(DEV), h, 1 / math.sqrt(d), None, s * s, s)
    att2 = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d) + full, -1)
    ref2 = (att2 @ v).permute(0, 2, 1, 3).reshape(b, s, h * d)
    assert (y2.float().cpu() - ref2).abs().max() < 3e-2
    # no mask
    y3 = hip().attention(qkv.to(DEV), None, h, 1 / math.sqrt(d), None, 0, 0)
    att3 = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), -1)
    ref3 = (att3 @ v).permute(0, 2, 1, 3).reshape(b, s, h * d)
    assert (y3.float().cpu() - ref3).abs().max() < 3e-2


@pytest.mark.parametrize("cfg,splits,shape", [
    (42, 1, (2, 14, 14, 256, 256, 1, 1, (0, 0, 0, 0))),
    (36, 3, (2, 14, 14, 256, 256, 1, 1, (0, 0, 0, 0))),     # split-K: the reduce kernel writes both
    (44, 1, (2, 28, 28, 128, 128, 3, 2, (1, 1, 1, 1))),     # im2col, strided
    (48, 1, (2, 28, 28, 128, 128, 3, 1, (1, 1, 1, 1))),     # halo 3x3
    (51, 2, (1, 7, 7, 512, 512, 3, 1, (1, 1, 1, 1))),       # halo, split over channel chunks
    (117, 1, (2, 14, 14, 256, 256, 1, 1, (0, 0, 0, 0))),    # 32x32 MFMA build
    (113, 2, (2, 28, 28, 128, 128, 3, 2, (1, 1, 1, 1))),    # 32x32 MFMA build, im2col, split-K
])
def test_conv_post_activation_outputs(cfg, splits, shape):
    """ResNet v2 epilogue: one conv writes the block sum y (+bias +residual)
    AND relu(y * s + t) (the next block's pre-activation), or only the latter."""
    n, h, w, cin, cout, k, s, pads = shape
    x = rnd(n, h, w, cin, seed=31).to(BF)
    wt = rnd(k, k, cin, cout, scale=1 / math.sqrt(k * k * cin), seed=32).to(BF).float()
    b = rnd(cout, scale=0.1, seed=33)
    ho = (h + pads[0] + pads[1] - k) // s + 1
    wo = (w + pads[2] + pads[3] - k) // s + 1
    res = rnd(n, ho, wo, cout, seed=34).to(BF)
    sc, sh = rnd(cout, seed=35) * 0.5 + 1.0, rnd(cout, seed=36) * 0.2
    ref = ref_conv(x, wt, b, s, pads, res, "none")
    ref2 = torch.relu(ref * sc + sh)
    out2 = torch.empty(n, ho, wo, cout, device=DEV, dtype=BF)
    y = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV), k, k, s, s, *pads, act=0, cfg=cfg, splits=splits,
                     post_scale=sc.to(DEV), post_shift=sh.to(DEV), post_act=ACT["relu"], out2=out2)
    torch.cuda.synchronize()
    tol = 3e-2 * max(1.0, ref.abs().max().item())
    assert (y.float().cpu() - ref).abs().max().item() < tol
    assert (out2.float().cpu() - ref2).abs().max().item() < tol
    only = hip().conv2d(x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV), k, k, s, s, *pads, act=0, cfg=cfg,
                        splits=splits, post_scale=sc.to(DEV), post_shift=sh.to(DEV), post_act=ACT["relu"],
                        post_only=True)
    torch.cuda.synchronize()
    assert (only.float().cpu() - ref2).abs().max().item() < tol


def test_conv_post_rejects_igemm():
    x = torch.zeros(1, 8, 8, 64, device=DEV, dtype=BF)
    w = torch.zeros(64, 64, device=DEV, dtype=BF)
    sc = torch.ones(64, device=DEV)
    with pytest.raises(RuntimeError, match="post-activation output needs"):
        hip().conv2d(x, w, None, None, 1, 1, 1, 1, 0, 0, 0, 0, act=0, cfg=3, post_scale=sc, post_shift=sc,
                     post_only=True)


def test_conv2d_dual_post_output():
    n, ho, c1, hh, c2, s, cout = 2, 14, 256, 28, 512, 2, 1024
    h = rnd(n, ho, ho, c1, seed=41).to(BF)
    x = rnd(n, hh, hh, c2, seed=42).to(BF)
    w1 = rnd(cout, c1, scale=1 / math.sqrt(c1), seed=43).to(BF)
    w2 = rnd(cout, c2, scale=1 / math.sqrt(c2), seed=44).to(BF)
    b = rnd(cout, scale=0.1, seed=45)
    sc, sh = rnd(cout, seed=46) * 0.5 + 1.0, rnd(cout, seed=47) * 0.2
    ref = h.float() @ w1.float().t() + x.float()[:, ::s, ::s, :] @ w2.float().t() + b
    w = torch.cat([w1, w2], 1).contiguous().to(DEV)
    out2 = torch.empty(n, ho, ho, cout, device=DEV, dtype=BF)
    y = hip().conv2d_dual(h.to(DEV), x.to(DEV), w, b.to(DEV), s, s, 0, 43, None, 1, post_scale=sc.to(DEV),
                          post_shift=sh.to(DEV), post_act=ACT["relu"], out2=out2)
    torch.cuda.synchronize()
    tol = 3e-2 * max(1.0, ref.abs().max().item())
    assert (y.float().cpu() - ref).abs().max().item() < tol
    assert (out2.float().cpu() - torch.relu(ref * sc + sh)).abs().max().item() < tol


def test_maxpool_post_affine():
    x = rnd(2, 112, 112, 64, seed=51).to(BF)
    sc, sh = rnd(64, seed=52) * 0.5, rnd(64, seed=53) * 0.2     # negative scales included
    y = hip().maxpool(x.to(DEV), 3, 3, 2, 2, 0, 1, 0, 1, post_scale=sc.to(DEV), post_shift=sh.to(DEV),
                      post_act=ACT["relu"])
    xp = F.pad(x.float().permute(0, 3, 1, 2), [0, 1, 0, 1], value=float("-inf"))
    ref = F.max_pool2d(xp, 3, 2).permute(0, 2, 3, 1)
    ref = torch.relu(ref * sc + sh)
    torch.cuda.synchronize()
    assert (y.float().cpu() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("cfg,splits,shape,post", [
    (36, 4, (2, 7, 7, 512, 512, 3, 2, (1, 1, 1, 1)), False),      # cgemm im2col, strided
    (42, 3, (2, 14, 14, 256, 256, 1, 1, (0, 0, 0, 0)), True),     # cgemm dense 1x1, post output
    (51, 4, (2, 7, 7, 512, 512, 3, 1, (1, 1, 1, 1)), False),      # halo, split over channel chunks
    (54, 2, (3, 14, 14, 256, 256, 3, 1, (1, 1, 1, 1)), True),     # 9-slot halo, post output
    (114, 2, (2, 14, 14, 256, 256, 1, 1, (0, 0, 0, 0)), True),    # 32x32 MFMA build, post output
])
def test_splitk_in_kernel_fixup_inside_graph(cfg, splits, shape, post, monkeypatch):
    """Captured in a HIP graph, split-K finishes in-kernel (the last slice of a
    tile sums the slabs -- 16-B agent-coherent stores / loads -- and runs the
    epilogue; no reduce launch).  Every replay (the tile counters re-zero
    themselves) equals the eager result (the same fixup on a ring slice of
    counters) and the fp32 reference."""
    monkeypatch.setenv("TFSERVE_SPLITK_FIXUP", "1")
    n, h, w, cin, cout, k, s, pads = shape
    x = rnd(n, h, w, cin, seed=61).to(BF)
    wt = rnd(k, k, cin, cout, scale=1 / math.sqrt(k * k * cin), seed=62).to(BF).float()
    b = rnd(cout, scale=0.1, seed=63)
    ho = (h + pads[0] + pads[1] - k) // s + 1
    wo = (w + pads[2] + pads[3] - k) // s + 1
    res = rnd(n, ho, wo, cout, seed=64).to(BF)
    kw = {}
    sc, sh = rnd(cout, seed=65).to(DEV), rnd(cout, seed=66).to(DEV)
    xd, wd, bd, rd = x.to(DEV), pack_w(wt), b.to(DEV), res.to(DEV)

    def call(out, out2):
        extra = dict(post_scale=sc, post_shift=sh, post_act=ACT["relu"], out2=out2) if post else {}
        return hip().conv2d(xd, wd, bd, rd, k, k, s, s, *pads, act=ACT["relu"], cfg=cfg, out=out, splits=splits,
                            **extra)
    eager = torch.empty(n, ho, wo, cout, device=DEV, dtype=BF)
    eager2 = torch.empty_like(eager)
    call(eager, eager2 if post else None)
    torch.cuda.synchronize()
    ref = ref_conv(x, wt, b, s, pads, res, "relu")
    assert (eager.float().cpu() - ref).abs().max() < 3e-2 * max(1.0, ref.abs().max().item())
    out = torch.empty_like(eager)
    out2 = torch.empty_like(eager)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            call(out, out2 if post else None)
    for _ in range(3):
        out.zero_()
        out2.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager), (out.float() - eager.float()).abs().max()
        if post:
            assert torch.equal(out2, eager2)


def test_splitk_counter_slices_return_with_their_graph(monkeypatch):
    """Counter slices a captured split-K launch takes go back to the pool when
    the graph captured under ops.capture_owner is collected: repeated
    capture / destroy cycles (graph tuning, reloads) do not use the pool up."""
    import gc
    from rust_tensorflow_serving2_amd import ops
    monkeypatch.setenv("TFSERVE_SPLITK_FIXUP", "1")
    x = rnd(2, 14, 14, 256, seed=71).to(BF).to(DEV)
    wt = pack_w(rnd(3, 3, 256, 256, scale=1 / 48, seed=72).to(BF).float())
    out = torch.empty(2, 14, 14, 256, device=DEV, dtype=BF)
    hip().conv2d(x, wt, None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=51, out=out, splits=4)   # pool allocated
    torch.cuda.synchronize()
    gc.collect()          # earlier tests' dead graphs return their slices first
    base = hip().splitk_counters_captured_in_use()
    stream = torch.cuda.Stream()
    for cycle in range(3):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream), ops.capture_owner(g), torch.cuda.graph(g, stream=stream):
            hip().conv2d(x, wt, None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=51, out=out, splits=4)
        assert hip().splitk_counters_captured_in_use() > base
        with torch.cuda.stream(stream):
            g.replay()
        torch.cuda.synchronize()
        del g
        gc.collect()
        assert hip().splitk_counters_captured_in_use() == base, cycle
        # released slices stay pending until their fences and zeroing complete
        assert hip().splitk_counters_pending() > 0
        _reclaim_all()
        assert hip().splitk_counters_captured_in_use() == base, cycle


def _reclaim_all(timeout_s=5.0):
    """reclaim() never blocks: call it until nothing is pending (idle streams)."""
    import time
    t0 = time.time()
    while hip().splitk_counters_pending() > 0:
        hip().splitk_counters_reclaim()
        assert time.time() - t0 < timeout_s, "released counter slices never became reusable"
        time.sleep(0.005)


def test_splitk_counter_slices_wait_for_a_queued_replay(monkeypatch):
    """a graph dropped with a replay still queued keeps its
    split-K counter slices out of the pool until that replay has completed
    (stream-ordered fence, no wall-clock quarantine): a capture made while it
    is queued takes fresh counters, and the slices come back only after the
    lane's stream has drained."""
    import gc
    import time
    from rust_tensorflow_serving2_amd import ops
    monkeypatch.setenv("TFSERVE_SPLITK_FIXUP", "1")
    x = rnd(2, 14, 14, 256, seed=73).to(BF).to(DEV)
    wt = pack_w(rnd(3, 3, 256, 256, scale=1 / 48, seed=74).to(BF).float())
    out = torch.empty(2, 14, 14, 256, device=DEV, dtype=BF)
    eager = hip().conv2d(x, wt, None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=51, splits=4)
    torch.cuda.synchronize()
    gc.collect()
    _reclaim_all()
    base = hip().splitk_counters_captured_in_use()
    lane, other = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(lane), ops.capture_owner(g) as tok, torch.cuda.graph(g, stream=lane):
        hip().conv2d(x, wt, None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=51, out=out, splits=4)
    took = hip().splitk_counters_captured_in_use() - base
    assert took > 0
    done = torch.cuda.Event()
    with torch.cuda.stream(lane):
        torch.cuda._sleep(600_000_000)     # ~0.25-0.3 s of GPU spin ahead of the replay
        g.replay()
        done.record()
    # the owner's release while its replay is still queued (the graph object
    # is kept: on ROCm 7 destroying a graph exec waits for its launches, so
    # the release is issued directly, as the finalizer would)
    assert hip().splitk_counters_release(tok) == took
    assert hip().splitk_counters_captured_in_use() == base
    assert hip().splitk_counters_pending() == took
    t_end = time.time() + 0.05
    while time.time() < t_end:
        assert hip().splitk_counters_reclaim() == 0      # fence not reached: nothing freed
    assert not done.query(), "the spin finished too early for this check"
    assert hip().splitk_counters_pending() == took
    # a capture made meanwhile gets fresh slices, not the queued replay's
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(other), ops.capture_owner(g2), torch.cuda.graph(g2, stream=other):
        hip().conv2d(x, wt, None, None, 3, 3, 1, 1, 1, 1, 1, 1, act=0, cfg=51, out=out, splits=4)
    assert hip().splitk_counters_pending() == took
    assert hip().splitk_counters_captured_in_use() - base == took
    lane.synchronize()                     # the queued replay completes (and its counters read zero)
    assert torch.equal(out, eager)
    _reclaim_all()
    del g
    gc.collect()                           # (its finalizer's release finds nothing left)
    assert hip().splitk_counters_pending() == 0
    with torch.cuda.stream(other):
        out.zero_()
        g2.replay()
    other.synchronize()
    assert torch.equal(out, eager)
    del g2
    gc.collect()
    _reclaim_all()
    assert hip().splitk_counters_captured_in_use() == base


def test_splitk_fixup_override_is_thread_local_and_restored():
    """ops.splitk_fixup_for_bucket sets the in-kernel split-K mode for the
    capturing thread only and restores the previous mode."""
    import threading
    from rust_tensorflow_serving2_amd import ops
    h = hip()
    assert h.get_splitk_fixup() == -1
    seen = []
    with ops.splitk_fixup_for_bucket(1):
        assert h.get_splitk_fixup() == 1
        with ops.splitk_fixup_for_bucket(32):
            assert h.get_splitk_fixup() == 0
        assert h.get_splitk_fixup() == 1
        t = threading.Thread(target=lambda: seen.append(h.get_splitk_fixup()))
        t.start()
        t.join()
    assert seen == [-1] and h.get_splitk_fixup() == -1


def test_classifier_head_host_rows_follow_the_launcher_predicate():
    h = hip()
    assert h.classifier_head_one_launch(1, 49, 2048, 1001, 1001)
    assert not h.classifier_head_one_launch(1, 49, 4096, 1001, 1001)     # 8 k-steps: three launches
    assert not h.classifier_head_one_launch(1, 49, 1536, 1001, 1001)
    assert not h.classifier_head_one_launch(32, 49, 2048, 1001, 1001)
    assert 84 not in h.halo_configs() and 80 in h.halo_configs()


# ResNet stem fused with its max pool (stem.hip): fp32 RGB in, pooled bf16 out.
# (n, h, w, C, cout, conv pads (t, b, l, r), pool pads (t, b, l, r), act, post)
STEM_CASES = [
    (2, 224, 224, 3, 64, (3, 3, 3, 3), (0, 1, 0, 1), "relu", False),   # ResNet-50 v1.5 stem (Pad 3 + VALID, SAME pool)
    (1, 224, 224, 3, 64, (3, 3, 3, 3), (0, 1, 0, 1), "none", True),    # v2: pool carries block 1's pre-activation
    (3, 160, 160, 3, 16, (3, 3, 3, 3), (0, 1, 0, 1), "relu", False),
    (2, 37, 53, 3, 32, (2, 3, 2, 3), (0, 1, 1, 1), "relu", False),     # odd sizes, partial tiles
    (1, 41, 29, 1, 48, (0, 0, 0, 0), (0, 0, 0, 0), "none", False),     # VALID conv + VALID pool, 1 channel
    (2, 64, 64, 4, 64, (3, 3, 3, 3), (1, 1, 1, 1), "relu", True),      # RGBA, symmetric pool padding
    # COUT = 64 with partial pooled tiles: the exact-store path's out-of-range
    # items go to a dropped offset (stem.hip kExactStores)
    (2, 37, 53, 3, 64, (2, 3, 2, 3), (0, 1, 1, 1), "relu", False),
    (1, 45, 71, 3, 64, (3, 3, 3, 3), (0, 1, 0, 1), "none", True),
]


@pytest.mark.parametrize("n,h,w,c,cout,cp,pp,act,post", STEM_CASES)
def test_stem_pool_fused_kernel(n, h, w, c, cout, cp, pp, act, post):
    x = torch.rand(n, h, w, c, generator=torch.Generator().manual_seed(h * w + cout))
    wt = rnd(cout, 7, 7, c, scale=0.05, seed=cout + c)
    w4 = torch.zeros(cout, 8, 8, 4)
    w4[:, :7, :7, :c] = wt
    wk = w4.reshape(cout, 256).to(BF)
    b = rnd(cout, scale=0.1, seed=7)
    kw = {}
    if post:
        sc, sh = rnd(cout, seed=8) * 0.5, rnd(cout, seed=9) * 0.2
        kw = dict(post_scale=sc.to(DEV), post_shift=sh.to(DEV), post_act=ACT["relu"])
    y = hip().stem_pool(x.to(DEV), wk.to(DEV), b.to(DEV), *cp, ACT[act], *pp, **kw)
    # reference: bf16-rounded operands, fp32 conv, conv output rounded to bf16
    # (as the unfused path stores it), -inf-padded max pool
    xr = x.to(BF).float().permute(0, 3, 1, 2)
    wr = wk.float().reshape(cout, 8, 8, 4)[:, :7, :7, :c].permute(0, 3, 1, 2)
    pt, pb, pl, pr = cp
    conv = F.conv2d(F.pad(xr, [pl, pr, pt, pb]), wr, stride=2) + b.view(1, -1, 1, 1)
    if act == "relu":
        conv = torch.relu(conv)
    conv = conv.to(BF).float()
    qt, qb, ql, qr = pp
    ref = F.max_pool2d(F.pad(conv, [ql, qr, qt, qb], value=float("-inf")), 3, 2).permute(0, 2, 3, 1)
    if post:
        ref = torch.relu(ref * sc + sh).to(BF).float()
    torch.cuda.synchronize()
    assert y.shape == ref.shape and y.dtype == BF
    err = (y.float().cpu() - ref).abs()
    assert err.max().item() < 2e-2 * max(1.0, ref.abs().max().item()), err.max()
    # most outputs agree exactly: only bf16 rounding ties of the conv values can differ
    assert (err == 0).float().mean().item() > 0.9


@pytest.mark.parametrize("cfg", [3, 36, 42])
def test_linear_row_strided_input(cfg):
    """BERT's pooler: rows are every sequence's first token of [B, S, H],
    read in place (lda = S * H) -- no gather copy."""
    B, S, H = 32, 16, 768
    seq = rnd(B, S, H, seed=21).to(BF).to(DEV)
    x = seq[:, 0, :]                                   # [B, H], stride (S*H, 1)
    assert not x.is_contiguous()
    w = rnd(H, H, scale=1 / math.sqrt(H), seed=22).to(BF)
    b = rnd(H, scale=0.1, seed=23)
    y = hip().linear(x, w.to(DEV), b.to(DEV), None, ACT["tanh"], cfg, True)
    ref = torch.tanh(seq[:, 0, :].float().cpu() @ w.float().t() + b)
    assert (y.cpu() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("b,n,k", [(32, 2, 768), (5, 3, 1024), (1, 16, 64)])
def test_dense_softmax_matches_fp32(b, n, k):
    x = rnd(b, k, seed=31).to(DEV)
    w = rnd(n + 3, k, scale=1 / math.sqrt(k), seed=32).to(BF)          # padded rows are ignored
    bias = rnd(n + 3, scale=0.5, seed=33)
    p = hip().dense_softmax(x, w.to(DEV), bias.to(DEV), n)
    ref = torch.softmax(x.cpu() @ w[:n].float().t() + bias[:n], -1)
    assert p.shape == (b, n)
    assert (p.cpu() - ref).abs().max().item() < 1e-5


def test_key_mask_adder_matches_fp32():
    m = torch.randint(0, 2, (7, 1, 33), dtype=torch.int32)
    out = hip().key_mask_adder(m.to(DEV), 1.0, -10000.0)
    torch.testing.assert_close(out.cpu(), (1.0 - m.float()) * -10000.0)
    mf = torch.rand(3, 1, 9)
    torch.testing.assert_close(hip().key_mask_adder(mf.to(DEV), 1.0, 2.5).cpu(), (1.0 - mf) * 2.5)


@pytest.mark.parametrize("k1,n1,n2", [(64, 256, 64), (64, 256, 128), (128, 512, 128), (128, 512, 256)])
@pytest.mark.parametrize("m,with_res,act1,act2", [(4 * 56 * 56, True, "relu", "relu"), (77, False, "none", "relu"),
                                                   (130, True, "relu", "none")])
def test_conv_chain_matches_fp32(k1, n1, n2, m, with_res, act1, act2):
    """expand 1x1 (+residual, act) -> next reduce 1x1 (+act) in one kernel vs
    fp32 torch; y2 is checked against the reference applied to the kernel's own
    bf16 y1 (what the separate reduce conv would read).  Row counts that are
    not a multiple of the 64-row tile included."""
    x = rnd(m, k1, seed=61).to(BF)
    w1 = rnd(n1, k1, scale=1 / math.sqrt(k1), seed=62).to(BF)
    b1 = rnd(n1, scale=0.1, seed=63)
    res = rnd(m, n1, seed=64).to(BF) if with_res else None
    w2 = rnd(n2, n1, scale=1 / math.sqrt(n1), seed=65).to(BF)
    b2 = rnd(n2, scale=0.1, seed=66)
    x4 = x.reshape(1, 1, m, k1)
    y1, y2 = hip().conv_chain(x4.to(DEV), w1.to(DEV), b1.to(DEV),
                              None if res is None else res.reshape(1, 1, m, n1).to(DEV), ACT[act1],
                              w2.to(DEV), b2.to(DEV), ACT[act2])
    assert y1.shape == (1, 1, m, n1) and y2.shape == (1, 1, m, n2)
    ref1 = x.float() @ w1.float().t() + b1 + (res.float() if res is not None else 0)
    ref1 = torch.relu(ref1) if act1 == "relu" else ref1
    y1c = y1.reshape(m, n1).float().cpu()
    assert (y1c - ref1).abs().max().item() < 2e-2 * max(1.0, ref1.abs().max().item())
    ref2 = y1c @ w2.float().t() + b2
    ref2 = torch.relu(ref2) if act2 == "relu" else ref2
    y2c = y2.reshape(m, n2).float().cpu()
    assert (y2c - ref2).abs().max().item() < 1e-2 * max(1.0, ref2.abs().max().item())


def test_conv_chain_is_deterministic():
    """Two launches on the same operands give the same bits (ResNet stage-1 b32 size)."""
    m, k1, n1, n2 = 32 * 56 * 56, 64, 256, 64
    x = rnd(1, 1, m, k1, seed=71).to(BF).to(DEV)
    w1 = rnd(n1, k1, scale=1 / 8, seed=72).to(BF).to(DEV)
    w2 = rnd(n2, n1, scale=1 / 16, seed=73).to(BF).to(DEV)
    b1, b2 = rnd(n1, seed=74).to(DEV), rnd(n2, seed=75).to(DEV)
    res = rnd(1, 1, m, n1, seed=76).to(BF).to(DEV)
    outs = [hip().conv_chain(x, w1, b1, res, ACT["relu"], w2, b2, ACT["relu"]) for _ in range(4)]
    for y1, y2 in outs[1:]:
        assert torch.equal(y1, outs[0][0]) and torch.equal(y2, outs[0][1])


@pytest.mark.parametrize("cfg", HALO_CFGS)
def test_halo_conv_is_deterministic(cfg):
    """Repeated launches give the same bits (the ring refill after each barrier
    must not race the previous step's LDS reads)."""
    n, h, w, cin, cout = 32, 56, 56, 64, 64
    x = rnd(n, h, w, cin, seed=81).to(BF).to(DEV)
    wt = rnd(3, 3, cin, cout, scale=1 / 24, seed=82).to(BF).float()
    b = rnd(cout, scale=0.1, seed=83).to(DEV)
    wp = pack_w(wt)
    ys = [hip().conv2d(x, wp, b, None, 3, 3, 1, 1, 1, 1, 1, 1, act=ACT["relu"], cfg=cfg) for _ in range(4)]
    for y in ys[1:]:
        assert torch.equal(y, ys[0])


@pytest.mark.parametrize("n,h,w,c", [(2, 224, 224, 3), (1, 33, 35, 3), (1, 17, 19, 1), (1, 21, 23, 4)])
def test_stem_pool_bf16_input_is_bit_identical(n, h, w, c):
    """The stem reading a request converted to bf16 on ingest (two dword loads
    per pixel, either parity, the tensor's last pixel included) gives exactly
    the output of reading the fp32 request."""
    x = rnd(n, h, w, c, seed=91) * 100.0
    wt = rnd(64, 224, scale=0.05, seed=92).to(BF).to(DEV)
    b = rnd(64, scale=0.1, seed=93).to(DEV)
    args = (wt, b, 3, 3, 3, 3, ACT["relu"], 1, 1, 1, 1)
    y32 = hip().stem_pool(x.to(DEV), *args)
    y16 = hip().stem_pool(x.to(BF).to(DEV), *args)
    assert torch.equal(y32, y16)


# Deferred LayerNorm (hip().linear_lnx, graph/fused.py defer_layernorm): GEMMs
# whose A rows / residual rows are pre-LayerNorm sums with (sum, sum sq)
# partials, and that emit their own rows' partials -- vs fp32 references with
# the LayerNorm materialised.
LNX_CFGS = [36, 47, 100, 72, 123, 38, 114, 37, 44, 45]


def _row_partials(t: torch.Tensor, parts: int) -> torch.Tensor:
    """[M][parts][2] (sum, sum sq) over `parts` column slices of t's rows."""
    f = t.float()
    cols = torch.tensor_split(torch.arange(f.shape[1]), parts)
    return torch.stack([torch.stack([f[:, c].sum(1), (f[:, c] ** 2).sum(1)], 1) for c in cols], 1).contiguous()


@pytest.mark.parametrize("cfg", LNX_CFGS)
@pytest.mark.parametrize("m,n,k", [(4096, 768, 768), (1000, 768, 3072), (77, 256, 128), (130, 512, 64)])
def test_linear_lnx_residual_side_and_stats(m, n, k, cfg):
    x = rnd(m, k, seed=61).to(BF)
    w = rnd(n, k, scale=1 / math.sqrt(k), seed=62).to(BF)
    b = rnd(n, scale=0.1, seed=63)
    zr = (rnd(m, n, seed=64) * 2 + 0.5).to(BF)               # the residual before its LayerNorm
    g, bt = 1 + rnd(n, scale=0.1, seed=65), rnd(n, scale=0.1, seed=66)
    y_ref = x.float() @ w.float().t() + b + F.layer_norm(zr.float(), (n,), g, bt, 1e-12)
    for parts in (1, 3):
        y, st = hip().linear_lnx(x.to(DEV), w.to(DEV), b.to(DEV), zr.to(DEV), 0, cfg,
                                 r_st=_row_partials(zr, parts).to(DEV), r_gamma=g.to(DEV), r_beta=bt.to(DEV),
                                 r_eps=1e-12, stats=True)
        torch.cuda.synchronize()
        y = y.float().cpu()
        assert (y - y_ref).abs().max().item() < 3e-2 * max(1.0, y_ref.abs().max().item())
        # the emitted partials are exactly the stored rows' sums (fp32 order aside)
        tot = st.cpu().sum(1)
        assert st.shape[0] == m and st.shape[2] == 2
        assert torch.allclose(tot[:, 0], y.sum(1), rtol=1e-4, atol=1e-2)
        assert torch.allclose(tot[:, 1], (y * y).sum(1), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("cfg", LNX_CFGS)
@pytest.mark.parametrize("m,n,k", [(4096, 768, 768), (1000, 3072, 768), (77, 256, 128), (130, 512, 64)])
def test_linear_lnx_input_side_matches_fp32(m, n, k, cfg):
    z = (rnd(m, k, seed=71) * 1.5 + 0.3).to(BF)                # A before its LayerNorm
    W = rnd(k, n, scale=1 / math.sqrt(k), seed=72)
    b = rnd(n, scale=0.1, seed=73)
    g, bt = 1 + rnd(k, scale=0.1, seed=74), rnd(k, scale=0.1, seed=75)
    ref = F.gelu(F.layer_norm(z.float(), (k,), g, bt, 1e-12) @ W + b, approximate="tanh")
    wf = (W * g[:, None]).t().contiguous().to(BF)
    colsum = wf.float().sum(1)
    bf = b + bt @ W
    y, st = hip().linear_lnx(z.to(DEV), wf.to(DEV), bf.to(DEV), None, ACT["gelu_tanh"], cfg,
                             a_st=_row_partials(z, 2).to(DEV), a_colsum=colsum.to(DEV), a_eps=1e-12)
    torch.cuda.synchronize()
    assert st.numel() == 0
    assert (y.float().cpu() - ref).abs().max().item() < 4e-2 * max(1.0, ref.abs().max().item())


def test_linear_lnx_in_graph_replays_and_rejections():
    m, n, k = 512, 768, 256
    z = rnd(m, k, seed=81).to(BF).to(DEV)
    w = rnd(n, k, scale=1 / math.sqrt(k), seed=82).to(BF).to(DEV)
    zr = rnd(m, n, seed=83).to(BF).to(DEV)
    cs = w.float().sum(1)
    ast, rst = _row_partials(z, 2), _row_partials(zr, 4)
    g1, b1 = torch.ones(n, device=DEV), torch.zeros(n, device=DEV)
    y = torch.empty(m, n, device=DEV, dtype=BF)
    kw = dict(a_st=ast, a_colsum=cs, r_st=rst, r_gamma=g1, r_beta=b1, stats=True)
    _, st0 = hip().linear_lnx(z, w, None, zr, 0, 100, False, y, **kw)
    torch.cuda.synchronize()
    eager, est = y.clone(), st0.clone()
    s = torch.cuda.Stream()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(gr, stream=s):
        _, st = hip().linear_lnx(z, w, None, zr, 0, 100, False, y, **kw)
    for _ in range(3):
        y.zero_()
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(y, eager) and torch.equal(st, est)
    with pytest.raises(RuntimeError):      # persistent configs: no deferred LayerNorm
        hip().linear_lnx(z, w, None, zr, 0, 130, **kw)
    with pytest.raises(RuntimeError):      # igemm configs: no deferred LayerNorm
        hip().linear_lnx(z, w, None, zr, 0, 0, **kw)
    with pytest.raises(RuntimeError):      # statistics of fp32 outputs
        hip().linear_lnx(z, w, None, zr, 0, 100, True, **kw)
    with pytest.raises(RuntimeError):      # partials must be [M][P][2]
        hip().linear_lnx(z, w, None, zr, 0, 100, r_st=rst[:100], r_gamma=g1, r_beta=b1)


def test_tuned_choice_picks_the_faster_option_and_caches_it():
    """ops.tuned_choice (ChainConv's chain-vs-two-convs pick): times each
    option, keeps the faster, skips options that raise, returns the cached
    pick afterwards without running anything."""
    from rust_tensorflow_serving2_amd import ops
    calls = {0: 0, 1: 0, 2: 0}

    def slow():
        calls[0] += 1
        torch.cuda._sleep(2_000_000)

    def fast():
        calls[1] += 1
        torch.cuda._sleep(10_000)

    def bad():
        calls[2] += 1
        raise RuntimeError("not launchable")
    key = ("test_choice", 1)
    assert ops.tuned_choice(key, {0: slow, 1: fast, 2: bad}, default=0) == 1
    seen = dict(calls)
    assert ops.tuned_choice(key, {0: slow, 1: fast, 2: bad}, default=0) == 1
    assert calls == seen                      # cached: nothing re-run
    assert ops._TUNED[key] == (1, 1) and [c for _t, c in ops._TUNE_TIMES[key]] == [(1, 1), (0, 1)]


def test_h2d_rows_reads_fresh_host_rows_in_graph_replays():
    """The small-bucket input copy: a kernel reading pinned host rows with
    system-scope loads.  The host rewrites the SAME rows before every replay
    of one captured graph; each replay must see that write (a line an earlier
    replay left in L2 must not satisfy the next one)."""
    for nbytes in (16, 512, 301056, 16 * 1024 + 16):
        host = torch.zeros(nbytes // 2, dtype=torch.int16).pin_memory()
        dev = torch.empty(nbytes // 2, dtype=torch.int16, device=DEV)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            hip().h2d_rows(host, dev)
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            hip().h2d_rows(host, dev)
        for i in range(12):
            want = torch.randint(-30000, 30000, (nbytes // 2,), dtype=torch.int16, generator=torch.Generator().manual_seed(i))
            host.copy_(want)
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(dev.cpu(), want), (nbytes, i)
    with pytest.raises(RuntimeError):
        hip().h2d_rows(torch.zeros(7, dtype=torch.int16).pin_memory(), torch.empty(7, dtype=torch.int16, device=DEV))
