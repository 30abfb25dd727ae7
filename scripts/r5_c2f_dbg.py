"""Debug the fused C2f vs the unfused chain: per-stage comparison on YOLOv8-n l2."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from aiko_services_amd import ops  # noqa: E402
from aiko_services_amd.models.yolov8 import YOLOv8  # noqa: E402

ops.require_native()
m = YOLOv8("n", device="cuda")
g = torch.Generator().manual_seed(1)
x = (torch.randn(1, 160, 160, 32, generator=g) * 2).to("cuda", torch.bfloat16)
for rb in (160, 10):
    os.environ["AIKO_C2F_RB"] = str(rb)
    os.environ["AIKO_C2F_FUSED"] = "1"
    f = torch.zeros(1, 160, 160, 32, dtype=torch.bfloat16, device="cuda")
    m._run_c2f("f", m.l2, x, f)
    os.environ["AIKO_C2F_FUSED"] = "0"
    u = torch.zeros_like(f)
    m._run_c2f("u", m.l2, x, u)
    torch.cuda.synchronize()
    d = (f.float() - u.float()).abs()
    print("rb", rb, "max diff", d.max().item(), "ref max", u.float().abs().max().item(),
          "cos", torch.nn.functional.cosine_similarity(f.float().flatten(), u.float().flatten(), dim=0).item())
    bad = (d > 0.05 * u.float().abs().max()).nonzero()
    print(" bad count", bad.shape[0], "rows", sorted(set(bad[:, 1].tolist()))[:20], "cols", sorted(set(bad[:, 2].tolist()))[:20],
          "ch", sorted(set(bad[:, 3].tolist()))[:32])
    print(" row-wise max diff", [round(v, 3) for v in d.amax(dim=(0, 2, 3))[:24].tolist()])
# channel correspondence: which unfused channel does each fused channel match best
ff = f.float().reshape(-1, 32)
uu = u.float().reshape(-1, 32)
fn = ff / (ff.norm(dim=0, keepdim=True) + 1e-9)
un = uu / (uu.norm(dim=0, keepdim=True) + 1e-9)
cm = fn.T @ un
best = cm.argmax(dim=1)
print("best match per fused channel:", best.tolist())
print("cos of best:", [round(v, 3) for v in cm.max(dim=1).values.tolist()])
