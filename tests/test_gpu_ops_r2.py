"""Round-2 HIP ops vs plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,T,C", [(16, 1500, 768), (3, 7, 64), (2, 33, 520)])
def test_mean_rows_f32(native, B, T, C):
    from aiko_services_amd.ops.vision import mean_rows
    x = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    ref = x.float().mean(dim=1)
    got = mean_rows(x)
    torch.cuda.synchronize()
    assert torch.allclose(got, ref, atol=1e-5, rtol=1e-4)
