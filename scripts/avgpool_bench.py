import sys, os
sys.path.insert(0, os.getcwd())
import torch
from aiko_services_amd.ops import vision as V, require_native
require_native()
x = torch.randn(256, 7, 7, 2048, device="cuda").to(torch.bfloat16)
for _ in range(3): V.avgpool(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): y = V.avgpool(x)
e1.record(); torch.cuda.synchronize()
print(f"avgpool: {e0.elapsed_time(e1)/20*1e3:.1f} us  exact={torch.equal(y.float(), x.float().mean((1,2)).to(torch.bfloat16).float()) }")
lg = torch.randn(256, 1000, device="cuda").to(torch.bfloat16)
for _ in range(3): V.softmax_topk(lg, 5)
torch.cuda.synchronize()
e0.record()
for _ in range(20): pr, ix = V.softmax_topk(lg, 5)
e1.record(); torch.cuda.synchronize()
ri = torch.softmax(lg.float(), -1).topk(5, -1)[1]
print(f"softmax_topk: {e0.elapsed_time(e1)/20*1e3:.1f} us  same_values={torch.equal(lg.float().gather(1, ix.long()), lg.float().gather(1, ri))}")
from aiko_services_amd.ops.vision import mean_rows
f = torch.randn(16, 1500, 768, device="cuda").to(torch.bfloat16)
for _ in range(3): mean_rows(f)
torch.cuda.synchronize()
e0.record()
for _ in range(20): m = mean_rows(f)
e1.record(); torch.cuda.synchronize()
print(f"mean_rows [16,1500,768]: {e0.elapsed_time(e1)/20*1e3:.1f} us  ok={torch.allclose(m, f.float().mean(1), rtol=1e-4, atol=1e-5)}")
