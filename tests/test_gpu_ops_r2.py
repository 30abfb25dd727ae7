"""Round-2 HIP ops vs plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,T,C", [(16, 1500, 768), (3, 7, 64), (2, 33, 520), (64, 41, 1032)])
def test_mean_rows_f32(native, B, T, C):
    from aiko_services_amd.ops.vision import mean_rows
    x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    ref = x.float().mean(dim=1)
    got = mean_rows(x)
    torch.cuda.synchronize()
    assert torch.allclose(got, ref, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("B,W,n", [(16, 480000, 80000), (3, 64, 4), (2, 1024, 1024)])
def test_window_shift(native, B, W, n):
    """window_shift_kernel: dst = src[:, n:] ++ chunk, exactly (a copy) — the AudioWindow update."""
    from aiko_services_amd.ops.audio import window_shift
    g = torch.Generator(device="cuda").manual_seed(B + W)
    src = torch.randn(B, W, device="cuda", generator=g)
    chunk = torch.randn(B, n, device="cuda", generator=g)
    dst = torch.empty_like(src)
    window_shift(src, chunk, dst)
    assert torch.equal(dst, torch.cat([src[:, n:], chunk], 1))


def test_mean_rows_strided_prefix(native):
    """mean_rows reads a T-prefix view of a [B, Tp, C] buffer directly (FeatureSink's encoder
    output [:, :T]) — no .contiguous() copy."""
    from aiko_services_amd.ops.vision import mean_rows
    g = torch.Generator(device="cuda").manual_seed(3)
    full = torch.randn(4, 1501, 768, device="cuda", generator=g).to(torch.bfloat16)
    view = full[:, :1500]
    got = mean_rows(view)
    assert torch.allclose(got, view.float().mean(1), rtol=1e-4, atol=1e-5)


def test_zero_border_rows(native):
    """zero_border_rows_: rows b*rows and b*rows + rows - 1 of [B*rows, C] zeroed, others kept."""
    g = torch.Generator(device="cuda").manual_seed(4)
    B, rows, C = 5, 37, 768
    x = torch.randn(B * rows, C, device="cuda", generator=g).to(torch.bfloat16)
    ref = x.clone().view(B, rows, C)
    ref[:, 0] = 0
    ref[:, rows - 1] = 0
    torch.ops.aiko.zero_border_rows_(x, rows)
    assert torch.equal(x.view(B, rows, C), ref)
