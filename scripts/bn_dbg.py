import sys, os, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
from aiko_services_amd.ops import require_native
require_native()
from aiko_services_amd.ops import conv as C
import test_gpu_bneck as T
for (B, H, dual, grid) in [(3, 56, False, 0), (3, 56, False, 7), (2, 56, True, 3), (4, 1, False, 1)]:
    g = torch.Generator().manual_seed(1)
    cin = 64 if dual else 256
    c1, c2, c3, down = T._block(g, cin, dual)
    conv3 = C.fuse_shortcut(c3, down) if dual else c3
    x = torch.relu(torch.randn(B, cin, H, 56, generator=g)).to(torch.bfloat16)
    xd = x.permute(0, 2, 3, 1).contiguous().cuda()
    out = torch.full((B, H, 56, 256), float("nan"), dtype=torch.bfloat16, device="cuda")
    y = C.bneck_fused(xd, c1, c2, conv3, out=out, grid=grid)
    torch.cuda.synchronize()
    bad = ~torch.isfinite(y.float())
    print(B, H, dual, grid, "nan count", bad.sum().item(), "of", y.numel())
    if bad.any():
        idx = bad.nonzero()
        for d, nm in enumerate("nhwc"):
            print(" ", nm, torch.unique(idx[:, d]).tolist()[:64])
    ref = T._reference(x.float().cuda(), c1, c2, c3, down).permute(0, 2, 3, 1)
    err = (y.float() - ref).abs()
    err[bad] = 0
    big = err > 0.05 * (ref.abs() + 0.5)
    print("  wrong (finite) count", big.sum().item())
    if big.any():
        idx = big.nonzero()
        for d, nm in enumerate("nhwc"):
            print(" ", nm, torch.unique(idx[:, d]).tolist()[:64])
