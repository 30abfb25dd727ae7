"""Fused stage-1 ResNet bottleneck (bneck_fused.hip) vs a plain PyTorch fp32 reference of the
same block, and vs the unfused kernel path (conv3x3_patch / conv_chain / igemm)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _block(g, cin, dual):
    from aiko_services_amd.models.resnet50 import _rand_bn, _rand_conv
    from aiko_services_amd.ops import conv as C
    c1 = C.make_conv_spec(*C.fold_bn(_rand_conv(g, 64, cin, 1), *_rand_bn(g, 64)), act="relu", device=DEV)
    c2 = C.make_conv_spec(*C.fold_bn(_rand_conv(g, 64, 64, 3), *_rand_bn(g, 64)), pad=1, act="relu", device=DEV)
    c3 = C.make_conv_spec(*C.fold_bn(_rand_conv(g, 256, 64, 1), *_rand_bn(g, 256, (0.1, 0.3))), act="relu",
                          device=DEV)
    down = None
    if dual:
        down = C.make_conv_spec(*C.fold_bn(_rand_conv(g, 256, cin, 1), *_rand_bn(g, 256)), device=DEV)
    return c1, c2, c3, down


def _reference(x_nchw, c1, c2, c3, down):
    from aiko_services_amd.ops import reference as R
    t = R.conv_ref(x_nchw, c1)
    t = R.conv_ref(t.to(torch.bfloat16).float(), c2)          # the kernels round t1 / t2 to bf16
    idn = R.conv_ref(x_nchw, down) if down is not None else x_nchw
    return R.conv_ref(t.to(torch.bfloat16).float(), c3, residual_nchw=idn)


@pytest.mark.parametrize("B,H,dual,grid", [
    (3, 56, False, 0), (2, 56, True, 0),          # default grid: more CUs than rows, one row each
    (3, 56, False, 7), (2, 56, True, 3),          # ranges of 24 / 37-38 rows crossing image boundaries
    (9, 56, False, 5), (5, 56, True, 2),          # ranges spanning three or more images
    (2, 20, False, 1), (2, 20, True, 1),          # one workgroup streaming two images
    (1, 56, False, 1), (2, 13, False, 4),         # one image / uneven split (26 = 7 + 7 + 6 + 6)
    (4, 1, False, 1), (3, 2, True, 2),            # images of one / two rows: a boundary every row or two
    (40, 56, False, 0), (24, 56, True, 0),        # every CU streaming several rows: counted DMA waits
])
def test_bneck_fused_matches_torch(native, B, H, dual, grid):
    from aiko_services_amd.ops import conv as C
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + int(dual) + 7 * grid)
    cin = 64 if dual else 256
    c1, c2, c3, down = _block(g, cin, dual)
    conv3 = C.fuse_shortcut(c3, down) if dual else c3
    x = torch.relu(torch.randn(B, cin, H, 56, generator=g)).to(torch.bfloat16)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    out = torch.full((B, H, 56, 256), float("nan"), dtype=torch.bfloat16, device=DEV)
    y = C.bneck_fused(xd, c1, c2, conv3, out=out, grid=grid)
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all(), "unwritten / non-finite output pixels"
    ref = _reference(x.float().to(DEV), c1, c2, c3, down)
    err = _rel(y.permute(0, 3, 1, 2), ref)
    assert err < 1e-2, err
    # the unfused kernel path of the same block
    t1 = C.conv2d(xd, c1)
    t2 = C.conv2d(t1, c2)
    y2 = C.conv2d(t2, conv3, x2=xd) if dual else C.conv2d(t2, c3, residual=xd)
    assert _rel(y, y2) < 5e-3


def test_resnet50_stage1_fused_matches_unfused(native, monkeypatch):
    """The model's stage 1 on bneck_fused (default) against the round-3 kernel chain."""
    from aiko_services_amd.models.resnet50 import ResNet50
    m = ResNet50(device=DEV)
    frames = torch.randint(0, 256, (8, 224, 224, 3), dtype=torch.uint8, device=DEV)
    assert m.bneck
    a = m.logits(frames).float()
    m.bneck = False
    b = m.logits(frames).float()
    ref = m.reference_logits(frames)
    torch.cuda.synchronize()
    cos = torch.nn.functional.cosine_similarity
    assert cos(a.flatten(), b.flatten(), dim=0).item() > 0.999
    assert cos(a, ref, dim=1).min().item() > 0.995
