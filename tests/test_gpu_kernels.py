"""Numerics of the HIP kernels vs plain PyTorch fp32 references (run on MI355X: -m gpu)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _nhwc(x_nchw):
    return x_nchw.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("B,H,W,cin,cout,k,stride,pad,act,res,tile", [
    (2, 56, 56, 64, 64, 1, 1, 0, "relu", False, None),
    (2, 56, 56, 64, 256, 1, 1, 0, "relu", True, None),
    (2, 56, 56, 64, 64, 3, 1, 1, "relu", False, None),
    (2, 56, 56, 128, 128, 3, 2, 1, "relu", False, None),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (128, 128)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (64, 64)),
    (1, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (128, 64)),
    (2, 28, 28, 256, 512, 1, 2, 0, None, False, (64, 128)),
    (2, 20, 20, 16, 32, 3, 1, 1, "silu", False, None),    # Cin=16: 4 taps per K block
    (2, 20, 20, 48, 64, 3, 2, 1, "silu", False, None),    # Cin=48: padded chunk
    (1, 9, 11, 40, 24, 3, 1, 1, None, False, None),       # odd spatial, Cout=24 (N tail)
    # LDS-DMA variant (global_load_lds ring, zero-page padding)
    (2, 56, 56, 64, 256, 1, 1, 0, "relu", True, (128, 128, 1)),
    (2, 56, 56, 64, 64, 3, 1, 1, "relu", False, (128, 64, 1)),
    (2, 28, 28, 128, 128, 3, 2, 1, "relu", True, (64, 64, 1)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (64, 128, 1)),
    (1, 9, 11, 40, 24, 3, 1, 1, "silu", False, (64, 64, 1)),
    (2, 20, 20, 48, 64, 3, 2, 1, "silu", False, (128, 64, 1)),
    (2, 20, 20, 16, 64, 3, 1, 1, "relu", False, (128, 128, 1)),
    # exact-N LDS-DMA tiles (4 x 1 waves, N = 80: the YOLO class branch, Cc = 80 input)
    (2, 20, 20, 80, 80, 3, 1, 1, "silu", False, (128, 80, 1)),
    (1, 13, 17, 80, 80, 1, 1, 0, None, True, (128, 80, 1)),
    (2, 20, 20, 80, 80, 3, 1, 1, "silu", True, (256, 80, 1)),
    (1, 9, 11, 64, 80, 3, 2, 1, "relu", False, (256, 80, 1)),
    # buffer-LDS-DMA variant (Cc % 64 == 0: padding by out-of-range buffer reads)
    (2, 56, 56, 64, 256, 1, 1, 0, "relu", True, (128, 128, 2)),
    (2, 56, 56, 64, 64, 3, 1, 1, "relu", False, (128, 64, 2)),
    (2, 28, 28, 128, 128, 3, 2, 1, "relu", True, (64, 64, 2)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (64, 128, 2)),
    (1, 9, 11, 128, 64, 3, 1, 1, "silu", False, (64, 64, 2)),
    (2, 7, 7, 512, 512, 3, 1, 1, "relu", False, (128, 128, 2)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (128, 64, 2)),
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", True, (256, 128, 2)),   # 8-wave, 3-slot ring
    (3, 14, 14, 256, 512, 1, 1, 0, None, False, (128, 256, 2)),
    (1, 9, 11, 128, 64, 3, 2, 1, "silu", False, (256, 128, 2)),
    (2, 30, 30, 64, 64, 3, 1, 1, "relu", True, (256, 64, 2)),
    # 32x32x16-MFMA buffer-DMA (variant 5): every tile shape, 1x1 / 3x3 / strided, residual
    (2, 56, 56, 64, 256, 1, 1, 0, "relu", True, (128, 128, 5)),
    (2, 56, 56, 64, 64, 3, 1, 1, "relu", False, (128, 64, 5)),
    (2, 28, 28, 128, 128, 3, 2, 1, "relu", True, (64, 128, 5)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (64, 128, 5)),
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", True, (256, 128, 5)),
    (3, 14, 14, 256, 512, 1, 1, 0, None, False, (128, 256, 5)),
    (1, 9, 11, 128, 64, 3, 2, 1, "silu", False, (256, 128, 5)),
    (2, 7, 7, 512, 512, 3, 1, 1, "relu", False, (128, 128, 5)),
    # 4-wave wide tiles (variant 6): 128 x 64 / 64 x 128 per wave, one workgroup per CU
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", True, (256, 128, 6)),
    (3, 14, 14, 256, 512, 1, 1, 0, None, False, (128, 256, 6)),
    (1, 9, 11, 128, 256, 3, 2, 1, "silu", True, (128, 256, 6)),
    (2, 7, 7, 512, 128, 3, 1, 1, "relu", False, (256, 128, 6)),
    # direct narrow 3x3 kernel (variant 7): Cc / Cout 16 or 32, stride 1 / 2, ragged tiles
    (2, 40, 70, 16, 16, 3, 1, 1, "silu", True, (8, 32, 7)),
    (1, 33, 65, 16, 32, 3, 2, 1, "silu", False, (8, 32, 7)),
    (2, 17, 37, 32, 32, 3, 1, 1, "relu", True, (8, 32, 7)),
    (1, 20, 64, 32, 16, 3, 2, 1, None, False, (8, 32, 7)),
    (1, 9, 10, 16, 32, 3, 1, 1, "gelu", True, (8, 32, 7)),
    (2, 21, 45, 32, 32, 1, 1, 0, "silu", True, (8, 32, 7)),
    (1, 16, 32, 16, 32, 1, 1, 0, None, False, (8, 32, 7)),
    # the same kernel with 16-row output tiles
    (1, 20, 64, 32, 16, 3, 2, 1, None, False, (16, 32, 7)),
    (1, 9, 10, 16, 32, 3, 1, 1, "gelu", True, (16, 32, 7)),
    (2, 21, 45, 32, 32, 1, 1, 0, "silu", True, (16, 32, 7)),
    (2, 37, 70, 16, 16, 3, 1, 1, "silu", True, (16, 32, 7)),
    (1, 40, 66, 16, 32, 3, 2, 1, "relu", False, (16, 32, 7)),
    # Cc-32 weights in registers (bn = 64)
    (1, 9, 10, 32, 32, 3, 1, 1, "gelu", True, (16, 64, 7)),
    (2, 21, 45, 32, 16, 3, 2, 1, "silu", True, (8, 64, 7)),
    (2, 21, 45, 32, 32, 1, 1, 0, "silu", True, (16, 64, 7)),
    # high-occupancy buffer-DMA (variant 3)
    (2, 28, 28, 128, 512, 1, 1, 0, "relu", True, (64, 128, 3)),
    (1, 9, 11, 128, 64, 3, 1, 1, "silu", False, (64, 64, 3)),
    # persistent: one K-block stream across each workgroup's tiles (variant 4); K = 64 / 128
    # (1-2 blocks per tile, the ring spans several tiles), 3x3 taps, odd M tails
    (2, 56, 56, 64, 256, 1, 1, 0, "relu", True, (64, 128, 4)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (64, 128, 4)),
    (2, 28, 28, 128, 512, 1, 1, 0, "relu", True, (128, 128, 4)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (64, 64, 4)),
    (2, 28, 28, 128, 128, 3, 1, 1, "relu", False, (64, 128, 4)),
    (1, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (128, 128, 4)),
    # 8-wave wide tiles with the register-direct epilogue (variant 8): every tile, 1x1 / 3x3 /
    # strided, residual (prefetched or not), M and N tails, odd spatial sizes
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", True, (256, 256, 8)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (256, 256, 8)),
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", True, (256, 128, 8)),
    (3, 14, 14, 256, 512, 1, 1, 0, None, False, (128, 256, 8)),
    (1, 9, 11, 128, 64, 3, 2, 1, "silu", False, (256, 64, 8)),
    (2, 30, 30, 64, 64, 3, 1, 1, "relu", True, (256, 64, 8)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (128, 128, 8)),
    (2, 7, 7, 512, 512, 3, 1, 1, "relu", False, (256, 256, 8)),
    (1, 9, 11, 128, 200, 3, 1, 1, "silu", True, (256, 128, 8)),
    (2, 56, 56, 64, 256, 1, 1, 0, "relu", True, (128, 256, 8)),
    # variant 9: the same kernel at 2-3 workgroups per CU (4- and 8-wave shapes)
    (2, 28, 28, 128, 512, 1, 1, 0, "relu", True, (128, 128, 9)),
    (1, 9, 11, 128, 64, 3, 2, 1, "silu", False, (256, 64, 9)),
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (128, 64, 9)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (64, 128, 9)),
    (2, 30, 30, 64, 64, 3, 1, 1, "relu", True, (64, 64, 9)),
    # variant 11: 32-deep K blocks in a 4-slot ring — ring tails (K/32 = 2, 4, 54, 144 blocks),
    # 3x3 / strided / 1x1, M and N tails, residual prefetched or not
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", True, (256, 256, 11)),
    (3, 14, 14, 64, 1024, 1, 1, 0, None, True, (256, 256, 11)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (256, 128, 11)),
    (2, 7, 7, 512, 512, 3, 1, 1, "relu", False, (128, 256, 11)),
    (1, 9, 11, 128, 200, 3, 1, 1, "silu", True, (256, 128, 11)),
    (2, 30, 30, 64, 64, 3, 1, 1, "relu", True, (128, 256, 11)),
    # variant 12: persistent pointwise GEMM (1x1 / s1, K % 256 == 0, Cout % 128 == 0) — M tails,
    # several tiles per workgroup (B=64), K = 512 (8 blocks per tile), no residual, one column
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (128, 128, 12)),
    (2, 14, 14, 256, 1024, 1, 1, 0, "relu", True, (128, 128, 12)),
    (64, 14, 14, 256, 1024, 1, 1, 0, "relu", True, (128, 128, 12)),
    (1, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (128, 128, 12)),
    (64, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (128, 128, 12)),
    (2, 28, 28, 256, 128, 1, 1, 0, "relu", False, (128, 128, 12)),
    (40, 14, 14, 256, 512, 1, 1, 0, "gelu", True, (128, 128, 12)),
    # variant 13: resident 128 x 256 weight block, 64-pixel tiles, 8-slot ring (K == 256 only):
    # M tails, many tiles per workgroup (odd and even counts), no residual, one channel column
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (64, 128, 13)),
    (64, 14, 14, 256, 1024, 1, 1, 0, "relu", True, (64, 128, 13)),
    (65, 14, 14, 256, 1024, 1, 1, 0, "relu", True, (64, 128, 13)),
    (2, 28, 28, 256, 128, 1, 1, 0, "relu", False, (64, 128, 13)),
    (40, 14, 14, 256, 512, 1, 1, 0, "gelu", True, (64, 128, 13)),
    # K = 512: a 64 x 512 weight block per workgroup, one tile per ring cycle
    (1, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (64, 128, 13)),
    (64, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (64, 128, 13)),
    (8, 28, 28, 512, 128, 1, 1, 0, "relu", False, (64, 128, 13)),
    (9, 14, 14, 512, 256, 1, 1, 0, None, True, (64, 128, 13)),
    # K = 128: a 256 x 128 weight block per workgroup, 4-slot ring (1.5 tiles ahead), residual one
    # tile ahead in two 32 KB buffers — M tails, a single tile, odd / even tile counts, no residual
    (1, 7, 7, 128, 512, 1, 1, 0, "relu", True, (64, 128, 13)),
    (3, 28, 28, 128, 512, 1, 1, 0, "relu", True, (64, 128, 13)),
    (64, 28, 28, 128, 512, 1, 1, 0, "relu", True, (64, 128, 13)),
    (33, 28, 28, 128, 256, 1, 1, 0, None, True, (64, 128, 13)),
    (5, 20, 20, 128, 768, 1, 1, 0, "silu", False, (64, 128, 13)),
    # variant 18: exact-N tiles (80 / 144 channels computed per tile, 5 / 9 channel blocks per
    # wave: the odd last block stores 8 bytes) — YOLO head shapes, 1x1 / 3x3, M tails, residual
    # (prefetched), several channel tiles (Cout 160 / 288 = 2 tiles)
    (1, 20, 20, 64, 80, 3, 1, 1, "silu", False, (256, 80, 18)),
    (2, 10, 10, 64, 80, 3, 1, 1, "silu", True, (128, 80, 18)),
    (1, 20, 20, 128, 80, 1, 1, 0, None, False, (256, 80, 18)),
    (1, 17, 19, 64, 160, 3, 1, 1, "relu", True, (256, 80, 18)),
    (1, 20, 20, 64, 144, 3, 1, 1, "silu", False, (256, 144, 18)),
    (2, 9, 13, 128, 144, 3, 1, 1, "silu", True, (128, 144, 18)),
    (1, 11, 11, 64, 288, 1, 1, 0, "gelu", True, (256, 144, 18)),
    # variant 19: 4-wave 128 x 128 (2 per CU) and 128 x 256 tiles
    (2, 28, 28, 128, 128, 3, 1, 1, "relu", True, (128, 128, 19)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (128, 128, 19)),
    (3, 14, 14, 256, 512, 1, 1, 0, None, False, (128, 256, 19)),
    (1, 9, 11, 128, 200, 3, 1, 1, "silu", True, (128, 256, 19)),
    # variant 20: persistent walk (no residual) — K from 1 to 36 blocks, 3x3 / strided / dual
    # source below; several tiles per workgroup via AIKO_CONV_PERS_GRID in the test
    (2, 28, 28, 128, 256, 3, 1, 1, "relu", False, (256, 256, 20)),
    (3, 14, 14, 1024, 256, 1, 1, 0, "relu", False, (256, 256, 20)),
    (5, 14, 14, 256, 512, 1, 1, 0, None, False, (256, 128, 20)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", False, (256, 128, 20)),
    (4, 14, 14, 64, 1024, 1, 1, 0, "silu", False, (128, 256, 20)),
    (2, 7, 7, 512, 512, 3, 1, 1, "relu", False, (128, 256, 20)),
    # ... with a residual (3-slot forms, residual loaded D + 1 blocks ahead of each epilogue)
    (3, 14, 14, 256, 1024, 1, 1, 0, None, True, (256, 128, 20)),
    (2, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (128, 256, 20)),
    (1, 13, 9, 192, 72, 3, 2, 1, "gelu", True, (256, 128, 20)),
    # variant 14: the resident kernels with each tile's residual issued at its own tile
    (64, 28, 28, 128, 512, 1, 1, 0, "relu", True, (64, 128, 14)),
    (65, 14, 14, 256, 1024, 1, 1, 0, "relu", True, (64, 128, 14)),
    (64, 7, 7, 512, 2048, 1, 1, 0, "relu", True, (64, 128, 14)),
])
def test_conv_igemm_matches_torch(native, B, H, W, cin, cout, k, stride, pad, act, res, tile, monkeypatch):
    if tile is not None and len(tile) > 2 and tile[2] == 20:
        monkeypatch.setenv("AIKO_CONV_PERS_GRID", "3")    # 3 workgroups: many tiles each, odd tails
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(1234)
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, stride=stride, pad=pad, act=act, device=DEV)
    x = torch.randn(B, cin, H, W, generator=g).to(torch.bfloat16)
    x_nhwc = torch.zeros(B, H, W, spec.Cc, dtype=torch.bfloat16)
    x_nhwc[..., :cin] = _nhwc(x)
    x_nhwc = x_nhwc.to(DEV)
    Ho, Wo = spec.out_hw(H, W)
    r = torch.randn(B, cout, Ho, Wo, generator=g).to(torch.bfloat16) if res else None
    y = C.conv2d(x_nhwc, spec, residual=None if r is None else _nhwc(r).to(DEV), tile=tile)
    torch.cuda.synchronize()
    ref = R.conv_ref(x.float().to(DEV), spec, None if r is None else r.float().to(DEV))
    err = _rel_err(y.permute(0, 3, 1, 2), ref)
    assert err < 1e-2, err


@pytest.mark.parametrize("B,H,act,res,slices,grid", [
    (2, 80, "silu", None, False, 0), (3, 80, "silu", "after", True, 0), (1, 7, "relu", "before", False, 0),
    (4, 3, "silu", None, True, 5), (2, 1, None, "after", False, 1), (64, 80, "silu", "after", True, 0),
    (5, 80, "silu", None, False, 7)])
def test_conv3x3_rows_matches_torch(native, B, H, act, res, slices, grid):
    """Variant 17 (row-stream kernel, conv_rows.hip): 80-wide 32 -> 32 3x3 convs, row ranges that
    cross image boundaries (H = 7 / 3 / 1, grids of 1 / 5 / 7 workgroups), residual before / after
    the activation, channel-slice input, residual and output (the C2f layout)."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(B * 31 + H)
    w = torch.randn(32, 32, 3, 3, generator=g) / (32 * 9) ** 0.5
    b = torch.randn(32, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, stride=1, pad=1, act=act, device=DEV)
    x = torch.randn(B, 32, H, 80, generator=g).to(torch.bfloat16)
    r = torch.randn(B, 32, H, 80, generator=g).to(torch.bfloat16) if res else None
    if slices:
        cat = torch.zeros(B, H, 80, 96, dtype=torch.bfloat16)
        cat[..., 32:64] = _nhwc(x)
        if r is not None:
            cat[..., 64:96] = _nhwc(r)
        cat = cat.to(DEV)
        xin, rin = cat[..., 32:64], (cat[..., 64:96] if r is not None else None)
        ybig = torch.full((B, H, 80, 128), float("nan"), dtype=torch.bfloat16, device=DEV)
        out = ybig[..., 96:128]
    else:
        xin = _nhwc(x).to(DEV)
        rin = _nhwc(r).to(DEV) if r is not None else None
        out = torch.full((B, H, 80, 32), float("nan"), dtype=torch.bfloat16, device=DEV)
    assert C.rows_variant_ok(spec, xin, rin, None, out)
    act_code = spec.act | (C.ACT_RESIDUAL_AFTER if res == "after" else 0)
    torch.ops.aiko.conv3x3_rows_out(xin, C.rows_weight(spec), spec.bias, rin, out, act_code, grid)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all(), "unwritten output pixels"
    ref = R.conv_ref(x.float().to(DEV), spec, None if (r is None or res == "after") else r.float().to(DEV))
    if res == "after":
        ref = ref + r.float().to(DEV)
    assert _rel_err(out.permute(0, 3, 1, 2), ref) < 1e-2
    if slices:
        assert torch.isnan(ybig[..., :96].float()).all()


@pytest.mark.parametrize("B,H,act,slices,grid", [(2, 28, "relu", False, 0), (3, 28, None, False, 0),
                                                 (1, 30, "relu", False, 0), (2, 5, "relu", True, 0),
                                                 (5, 28, "relu", True, 3), (33, 28, "relu", False, 0),
                                                 (4, 14, None, False, 1)])
def test_conv3x3_patchw_matches_torch(native, B, H, act, slices, grid):
    """Variant 16 (streamed-weight patch kernel, conv_patchw.hip): 28-wide images, 14-row tiles
    with partial last tiles (H = 30, 5), several tiles per workgroup (grid 1 / 3, B = 33), a
    channel-slice input (pixel pitch 192) and output into a slice of a wider buffer."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(B * 100 + H)
    w = torch.randn(128, 128, 3, 3, generator=g) / (128 * 9) ** 0.5
    b = torch.randn(128, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, stride=1, pad=1, act=act, device=DEV)
    x = torch.randn(B, 128, H, 28, generator=g).to(torch.bfloat16)
    if slices:
        big = torch.zeros(B, H, 28, 192, dtype=torch.bfloat16)
        big[..., 32:160] = _nhwc(x)
        xin = big.to(DEV)[..., 32:160]
        ybig = torch.full((B, H, 28, 256), float("nan"), dtype=torch.bfloat16, device=DEV)
        out = ybig[..., 64:192]
    else:
        xin = _nhwc(x).to(DEV)
        out = torch.full((B, H, 28, 128), float("nan"), dtype=torch.bfloat16, device=DEV)
    assert C.patchw_variant_ok(spec, xin, None, None, out)
    torch.ops.aiko.conv3x3_patchw_out(xin, C.patchw_weight(spec), spec.bias, out, spec.act, grid)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all(), "unwritten output pixels"
    ref = R.conv_ref(x.float().to(DEV), spec)
    assert _rel_err(out.permute(0, 3, 1, 2), ref) < 1e-2
    if slices:
        assert torch.isnan(ybig[..., :64].float()).all() and torch.isnan(ybig[..., 192:].float()).all()
    # the tuner path picks it up through conv2d
    y = C.conv2d(xin, spec, tile=(392, 128, 16))
    torch.cuda.synchronize()
    assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("B,H,W,act", [(2, 56, 56, "relu"), (3, 13, 24, "silu"), (1, 30, 24, None), (3, 40, 40, "silu"),
                                          (2, 13, 40, "relu"),
                                          (2, 17, 56, "relu"), (1, 8, 56, "relu"), (3, 1, 24, "relu")])
def test_conv3x3_patch_matches_torch(native, B, H, W, act):
    """Variant 10 (LDS-resident input patch, conv_patch.hip): partial row tiles, narrow images,
    every activation, output into a channel slice of a wider buffer."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(B * 100 + H)
    w = torch.randn(64, 64, 3, 3, generator=g) / 24
    b = torch.randn(64, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, stride=1, pad=1, act=act, device=DEV)
    x = torch.randn(B, 64, H, W, generator=g).to(torch.bfloat16)
    xd = _nhwc(x).to(DEV)
    assert C.patch_variant_ok(spec, xd)
    y = C.conv2d(xd, spec, tile=(8, 64, 10))
    cat = torch.zeros(B, H, W, 96, dtype=torch.bfloat16, device=DEV)
    C.conv2d(xd, spec, out=cat[..., 16:80], tile=(8, 64, 10))
    torch.cuda.synchronize()
    ref = R.conv_ref(x.float().to(DEV), spec)
    assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2
    assert torch.equal(cat[..., 16:80], y)
    assert cat[..., :16].abs().max().item() == 0 and cat[..., 80:].abs().max().item() == 0


def test_conv_writes_into_channel_slice(native):
    """Output into a slice of a concat buffer and input from a channel slice (pitch != Cc)."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(7)
    B, H, W = 2, 16, 16
    big = torch.randn(B, H, W, 96, generator=g).to(torch.bfloat16).to(DEV)
    xin = big[..., 32:64]                      # 32-channel slice, pitch 96
    w = torch.randn(64, 32, 3, 3, generator=g) / 17
    spec = C.make_conv_spec(w, None, pad=1, act="silu", device=DEV)
    cat = torch.zeros(B, H, W, 128, dtype=torch.bfloat16, device=DEV)
    C.conv2d(xin, spec, out=cat[..., 64:128])
    torch.cuda.synchronize()
    ref = R.conv_ref(xin.permute(0, 3, 1, 2).float(), spec)
    assert _rel_err(cat[..., 64:].permute(0, 3, 1, 2), ref) < 1e-2
    assert cat[..., :64].abs().max().item() == 0


def test_conv_narrow_slices_post_residual(native):
    """Variant 7 as YOLO's C2f bottleneck runs it: 16-channel input slice of a concat buffer,
    output into another slice, residual (the input slice) added AFTER the SiLU."""
    from aiko_services_amd.ops import conv as C
    g = torch.Generator().manual_seed(11)
    B, H, W = 2, 24, 40
    cat = torch.randn(B, H, W, 48, generator=g).to(torch.bfloat16).to(DEV)
    xin = cat[..., 16:32]
    w = torch.randn(16, 16, 3, 3, generator=g) / 12
    b = torch.randn(16, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, pad=1, act="silu", device=DEV)
    out = torch.zeros(B, H, W, 64, dtype=torch.bfloat16, device=DEV)
    C.conv2d(xin, spec, residual=xin, out=out[..., 32:48], tile=(8, 32, 7), residual_after_act=True)
    ref_out = torch.zeros_like(out)
    C.conv2d(xin, spec, residual=xin, out=ref_out[..., 32:48], tile=(128, 32, 0), residual_after_act=True)
    torch.cuda.synchronize()
    assert _rel_err(out[..., 32:48].float(), ref_out[..., 32:48].float()) < 1e-2
    assert out[..., :32].abs().max().item() == 0 and out[..., 48:].abs().max().item() == 0


def test_stem_and_preprocess(native):
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(3)
    B = 3
    frames = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8)
    w = torch.randn(64, 3, 7, 7, generator=g) / (3 * 49) ** 0.5
    b = torch.randn(64, generator=g) * 0.1
    spec = C.make_stem_spec(w, b, act="relu", device=DEV)
    pre = V.preprocess_frames(frames.to(DEV))
    y = C.conv2d(pre, spec, image_hw=(224, 224))
    torch.cuda.synchronize()
    xr = R.preprocess_ref(frames.to(DEV))
    # the pre-processed image (interior) must match
    assert _rel_err(pre[:, 3:227, 3:227, :3].permute(0, 3, 1, 2), xr) < 5e-3
    assert pre[:, :3].abs().max().item() == 0 and pre[..., 3].abs().max().item() == 0
    ref = R.conv_ref(xr.to(torch.bfloat16).float(), spec)
    assert y.shape == (B, 112, 112, 64)
    assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_preprocess_resize(native):
    from aiko_services_amd.ops import reference as R
    from aiko_services_amd.ops import vision as V
    frames = torch.randint(0, 256, (2, 480, 640, 3), dtype=torch.uint8)
    pre = V.preprocess_frames(frames.to(DEV), (224, 224))
    ref = R.preprocess_ref(frames.to(DEV), (224, 224))
    assert _rel_err(pre[:, 3:227, 3:227, :3].permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("H,W,bgr", [(224, 224, False), (36, 100, True)])
def test_preprocess_rows_fast_path_exact(native, H, W, bgr):
    """No-resize frames take preprocess_rows_kernel (dword loads, a wave per row); the same
    frames at a 1-byte-offset base take the flat kernel.  Outputs must be bit-identical and the
    zero border must be written over whatever the buffer held."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(H + W)
    B = 3
    flat = torch.randint(0, 256, (B * H * W * 3 + 1,), generator=g, dtype=torch.uint8).to(DEV)
    odd = flat[1:].view(B, H, W, 3)                 # base % 4 == 1 -> flat kernel
    even = odd.clone()                              # aligned -> row kernel
    Hp, Wp = C.stem_geometry(H, W)
    outs = []
    for fr in (odd, even):
        out = torch.full((B, Hp, Wp, 4), 7.0, dtype=torch.bfloat16, device=DEV)
        outs.append(V.preprocess_frames(fr, (H, W), bgr=bgr, out=out))
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    assert outs[1][:, :3].abs().max().item() == 0 and outs[1][..., 3].abs().max().item() == 0
    assert outs[1][:, :, :3].abs().max().item() == 0 and outs[1][:, :, 3 + W:].abs().max().item() == 0


@pytest.mark.parametrize("B,H,W,c", [(3, 20, 20, 128), (2, 7, 33, 16), (1, 40, 40, 64)])
def test_sppf_pool_matches_chained_maxpools(native, B, H, W, c):
    """sppf_pool_ (one kernel, LDS separable pools) == three chained maxpool_out launches, exactly."""
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(H * W + c)
    cat = (torch.randn(B, H, W, 4 * c, generator=g) * 4).round().to(torch.bfloat16).to(DEV)
    ref = cat.clone()
    for i in range(3):
        V.maxpool2d(ref[..., i * c:(i + 1) * c], 5, 1, 2, out=ref[..., (i + 1) * c:(i + 2) * c])
    V.sppf_pool(cat, c, 5)
    torch.cuda.synchronize()
    assert torch.equal(cat, ref)


def test_linear_with_n_tail(native):
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(5)
    for B in (1, 7, 256):
        w = torch.randn(1000, 2048, generator=g) * 0.02
        b = torch.randn(1000, generator=g)
        spec = C.make_linear_spec(w, b, device=DEV)
        x = torch.randn(B, 2048, generator=g).to(torch.bfloat16).to(DEV)
        y = C.linear(x, spec)
        torch.cuda.synchronize()
        assert _rel_err(y, R.linear_ref(x.float(), spec)) < 1e-2


@pytest.mark.parametrize("B,N,K", [(256, 1000, 2048), (37, 1000, 2048), (1, 64, 1024), (300, 520, 4096)])
def test_linear_splitk(native, B, N, K):
    """Split-K classifier path (linear_splitk.hip: S K-slices of 32 x 32 one-wave tiles, fp32
    partials summed in a fixed order + bias): matches the igemm linear and the fp32 reference,
    M / N tails included, and repeats bit-identically (no atomics)."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(B + N)
    w = torch.randn(N, K, generator=g) * 0.02
    b = torch.randn(N, generator=g)
    spec = C.make_linear_spec(w, b, device=DEV)
    x = torch.randn(B, K, generator=g).to(torch.bfloat16).to(DEV)
    assert C.linear_splitk_ok(x, spec)
    work = torch.full((C.LINEAR_SPLITK * B * N,), float("nan"), device=DEV)
    y1 = C.linear(x, spec, work=work).clone()
    y2 = C.linear(x, spec, work=work).clone()
    base = C.linear(x, spec)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert _rel_err(y1, R.linear_ref(x.float(), spec)) < 1e-2
    assert _rel_err(y1.float(), base.float()) < 1e-2


def test_pools_and_topk(native):
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 112, 112, 64, generator=g).to(torch.bfloat16).to(DEV)
    y = V.maxpool2d(x, 3, 2, 1)
    ref = torch.nn.functional.max_pool2d(x.permute(0, 3, 1, 2).float(), 3, 2, 1)
    assert torch.equal(y.permute(0, 3, 1, 2).float(), ref)
    x = torch.randn(4, 7, 7, 2048, generator=g).to(torch.bfloat16).to(DEV)
    a = V.avgpool(x)
    assert _rel_err(a, x.float().mean(dim=(1, 2))) < 5e-3
    lg = torch.randn(37, 1000, generator=g).to(torch.bfloat16).to(DEV)
    p, i = V.softmax_topk(lg, 5)
    torch.cuda.synchronize()
    rp, ri = torch.softmax(lg.float(), -1).topk(5, -1)
    # bf16 logits can tie: compare the selected logit values, not tie-broken indices
    assert torch.equal(lg.float().gather(1, i.long()), lg.float().gather(1, ri))
    assert torch.allclose(p, rp, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("N,k", [(10, 8), (1000, 5), (2000, 7)])
def test_softmax_topk_exact_ties(native, N, k):
    """Packed-key arg-max: ties (incl. -0 vs +0) go to the lower column, like a stable sort."""
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(N)
    lg = torch.randint(-4, 5, (19, N), generator=g).float()
    lg[:, ::3] *= -0.0   # every third column becomes +0 or -0
    lg = lg.to(torch.bfloat16)
    p, i = V.softmax_topk(lg.to(DEV), k)
    torch.cuda.synchronize()
    order = torch.stack([torch.tensor(sorted(range(N), key=lambda c: (-float(r[c]), c)))
                         for r in lg.float()])[:, :k]
    assert torch.equal(i.cpu().long(), order)
    rp = torch.softmax(lg.float(), -1).gather(1, order)
    assert torch.allclose(p.cpu(), rp, rtol=1e-4, atol=1e-6)


def test_resnet50_matches_fp32_reference(native):
    from aiko_services_amd.models.resnet50 import ResNet50
    m = ResNet50(seed=0, device=DEV)
    frames = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8,
                           generator=torch.Generator().manual_seed(0)).to(DEV)
    lg = m.logits(frames).float()
    ref = m.reference_logits(frames)
    torch.cuda.synchronize()
    cos = torch.nn.functional.cosine_similarity(lg, ref, dim=1)
    assert cos.min().item() > 0.995, cos
    p, i = m(frames)
    torch.cuda.synchronize()
    assert p.shape == (4, 5) and i.shape == (4, 5)
    assert (i[:, 0].long() == lg.argmax(1)).all()


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 8, 11, 20])
@pytest.mark.parametrize("B,H,cin_main,cin_sc,cout,stride", [(2, 28, 64, 64, 256, 1), (2, 28, 128, 256, 512, 2),
                                                              (1, 14, 512, 1024, 2048, 2)])
def test_fused_projection_shortcut(native, B, H, cin_main, cin_sc, cout, stride, variant, monkeypatch):
    """conv3(t) + down(x) (+bias, ReLU) as one K-concatenated igemm with two A sources."""
    if variant == 20:
        monkeypatch.setenv("AIKO_CONV_PERS_GRID", "5")    # persistent walk over several tiles
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(21)
    Ho = H // stride
    w3 = torch.randn(cout, cin_main, 1, 1, generator=g) / cin_main ** 0.5
    wd = torch.randn(cout, cin_sc, 1, 1, generator=g) / cin_sc ** 0.5
    b3, bd = torch.randn(cout, generator=g), torch.randn(cout, generator=g)
    main = C.make_conv_spec(w3, b3, act="relu", device=DEV)
    down = C.make_conv_spec(wd, bd, stride=stride, device=DEV)
    fused = C.fuse_shortcut(main, down)
    t = torch.randn(B, Ho, Ho, cin_main, generator=g).to(torch.bfloat16).to(DEV)
    x = torch.randn(B, H, H, cin_sc, generator=g).to(torch.bfloat16).to(DEV)
    y = C.conv2d(t, fused, x2=x, tile=(256, 128, variant) if variant in (8, 11, 20) else (64, 128, variant))
    torch.cuda.synchronize()
    idn = R.conv_ref(x.permute(0, 3, 1, 2).float(), down)
    ref = R.conv_ref(t.permute(0, 3, 1, 2).float(), main, idn)
    assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2


@pytest.mark.parametrize("B,H,cout,stride", [(2, 56, 512, 2), (3, 56, 512, 2), (1, 28, 128, 1), (5, 18, 384, 2),
                                             (40, 56, 512, 2)])
def test_fused_projection_pw_dual(native, B, H, cout, stride):
    """Variant 13 with a second source (conv_pw.hip, K = 128 main + 256 strided shortcut columns,
    128 x 384 resident weight block): M tails, one / many tiles per workgroup, stride 1 and 2, odd
    output sizes (Ho = 9), every output written."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(B * 100 + H + cout)
    Ho = (H - 1) // stride + 1
    w3 = torch.randn(cout, 128, 1, 1, generator=g) / 128 ** 0.5
    wd = torch.randn(cout, 256, 1, 1, generator=g) / 256 ** 0.5
    b3, bd = torch.randn(cout, generator=g), torch.randn(cout, generator=g)
    main = C.make_conv_spec(w3, b3, act="relu", device=DEV)
    down = C.make_conv_spec(wd, bd, stride=stride, device=DEV)
    fused = C.fuse_shortcut(main, down)
    t = torch.randn(B, Ho, Ho, 128, generator=g).to(torch.bfloat16).to(DEV)
    x = torch.randn(B, H, H, 256, generator=g).to(torch.bfloat16).to(DEV)
    out = torch.full((B, Ho, Ho, cout), float("nan"), dtype=torch.bfloat16, device=DEV)
    y = C.conv2d(t, fused, x2=x, out=out, tile=(64, 128, 13))
    torch.cuda.synchronize()
    assert torch.isfinite(y.float()).all()
    idn = R.conv_ref(x.permute(0, 3, 1, 2).float(), down)
    ref = R.conv_ref(t.permute(0, 3, 1, 2).float(), main, idn)
    assert _rel_err(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_resize_u8(native):
    from aiko_services_amd.ops import vision as V
    frames = torch.randint(0, 256, (2, 37, 53, 3), dtype=torch.uint8, device=DEV)
    y = V.resize_u8(frames, (64, 80))
    ref = torch.nn.functional.interpolate(frames.permute(0, 3, 1, 2).float(), size=(64, 80), mode="bilinear",
                                          align_corners=False).round().clamp(0, 255).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() <= 1


def test_batchnorm_standalone(native):
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 9, 11, 64, generator=g).to(DEV, torch.bfloat16)
    gamma, beta = torch.rand(32, generator=g) + 0.5, torch.randn(32, generator=g)
    mean, var = torch.randn(32, generator=g), torch.rand(32, generator=g) + 0.5
    scale, shift = V.bn_scale_shift(gamma, beta, mean, var)
    out = torch.zeros(2, 9, 11, 64, dtype=torch.bfloat16, device=DEV)
    V.batchnorm(x[..., 32:], scale.to(DEV), shift.to(DEV), act=1, out=out[..., :32])
    ref = torch.nn.functional.batch_norm(x[..., 32:].permute(0, 3, 1, 2).float(), mean.to(DEV), var.to(DEV),
                                         gamma.to(DEV), beta.to(DEV), False, 0.0, 1e-5).relu()
    assert _rel_err(out[..., :32].permute(0, 3, 1, 2), ref) < 1e-2
    assert out[..., 32:].abs().max().item() == 0


@pytest.mark.parametrize("hw", [(224, 224), (160, 200), (96, 132)])
def test_stem_pool_fused(native, hw):
    """Fused stem + ReLU + max-pool kernel == conv2d stem + maxpool kernels (bit-exact), and
    the fp32 torch reference of the same ops."""
    import torch.nn.functional as F
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    from aiko_services_amd.ops import vision as V
    g = torch.Generator().manual_seed(11)
    B = 3
    frames = torch.randint(0, 256, (B, hw[0], hw[1], 3), generator=g, dtype=torch.uint8)
    w = torch.randn(64, 3, 7, 7, generator=g) / (3 * 49) ** 0.5
    b = torch.randn(64, generator=g) * 0.1
    spec = C.make_stem_spec(w, b, act="relu", device=DEV)
    pre = V.preprocess_frames(frames.to(DEV), hw)
    fused = C.stem_pool(pre, spec, hw, variant=0)
    unfused = V.maxpool2d(C.conv2d(pre, spec, image_hw=hw), 3, 2, 1)
    wide = C.stem_pool(pre, spec, hw, variant=1)
    torch.cuda.synchronize()
    assert fused.shape == unfused.shape
    assert torch.equal(fused, unfused) and torch.equal(wide, unfused)
    xr = R.preprocess_ref(frames.to(DEV), hw)
    ref = F.max_pool2d(R.conv_ref(xr.to(torch.bfloat16).float(), spec), 3, 2, 1)
    assert _rel_err(fused.permute(0, 3, 1, 2), ref) < 1e-2
    # uint8 frames straight into the fused stem (normalised in the kernel's patch fill): the
    # same values within bf16 rounding of the input / scaled weights, both tile widths
    if hw[1] % 4 == 0:
        outs = []
        for variant in (0, 1, 2, 3, 4):
            u8 = C.stem_pool_u8(frames.to(DEV), spec, V.IMAGENET_MEAN, V.IMAGENET_STD, variant=variant)
            torch.cuda.synchronize()
            assert u8.shape == fused.shape
            assert _rel_err(u8.permute(0, 3, 1, 2), ref) < 1e-2
            assert _rel_err(u8.float(), fused.float()) < 1e-2
            outs.append(u8)
        # the strip kernel (weights in registers, in-register horizontal max) is bit-identical
        # to the tile kernel: same patch values, same MFMA order per accumulator; so are the
        # half-channel-wave strip kernels (variants 3 / 4, carried pool row)
        assert torch.equal(outs[2], outs[0])
        assert torch.equal(outs[3], outs[0]) and torch.equal(outs[4], outs[0])


@pytest.mark.parametrize("tile,K", [((128, 128, 12), 256), ((64, 128, 13), 256), ((64, 128, 13), 128)])
def test_conv_pw_slices_and_post_residual(native, tile, K):
    """conv_pw (variants 12 / 13): input from a channel slice (pitch 384 != K), output into a
    slice of a concat buffer, residual added after the activation (YOLO bottleneck form) — the
    same result as the register-staged kernel within bf16 rounding, nothing outside the slice."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import reference as R
    g = torch.Generator().manual_seed(17)
    B, H, W, N = 9, 14, 14, 256
    big = torch.randn(B, H, W, 384, generator=g).to(torch.bfloat16).to(DEV)
    xin = big[..., 64:64 + K]
    w = torch.randn(N, K, 1, 1, generator=g) / 16
    b = torch.randn(N, generator=g) * 0.1
    spec = C.make_conv_spec(w, b, act="silu", device=DEV)
    res = torch.randn(B, H, W, N, generator=g).to(torch.bfloat16).to(DEV)
    cat = torch.zeros(B, H, W, 448, dtype=torch.bfloat16, device=DEV)
    C.conv2d(xin, spec, residual=res, out=cat[..., 128:128 + N], tile=tile, residual_after_act=True)
    ref_out = torch.zeros_like(cat)
    C.conv2d(xin, spec, residual=res, out=ref_out[..., 128:128 + N], tile=(128, 128, 0), residual_after_act=True)
    torch.cuda.synchronize()
    ref = R.conv_ref(xin.permute(0, 3, 1, 2).float(), spec) + res.permute(0, 3, 1, 2).float()
    assert _rel_err(cat[..., 128:128 + N].permute(0, 3, 1, 2), ref) < 1e-2
    assert _rel_err(cat.float(), ref_out.float()) < 1e-2
    assert cat[..., :128].abs().max().item() == 0 and cat[..., 128 + N:].abs().max().item() == 0
