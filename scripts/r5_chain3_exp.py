"""conv_chain3 timing at B=320 (stage 3) for the AIKO_CHAIN3_EXP diagnostic variant in the env."""
import os
import torch
from aiko_services_amd import ops
from aiko_services_amd.ops import conv as C

ops.require_native()
os.environ["AIKO_CHAIN3"] = "1"
g = torch.Generator().manual_seed(0)
spec3 = C.make_conv_spec(torch.randn(1024, 256, 1, 1, generator=g) / 16, 0.1 * torch.randn(1024, generator=g),
                         act="relu", device="cuda")
spec1 = C.make_conv_spec(torch.randn(256, 1024, 1, 1, generator=g) / 32, 0.1 * torch.randn(256, generator=g),
                         act="relu", device="cuda")
B = 320
x = torch.randn(B, 14, 14, 256, generator=g).to("cuda", torch.bfloat16)
r = torch.randn(B, 14, 14, 1024, generator=g).to("cuda", torch.bfloat16)
y = torch.empty(B, 14, 14, 1024, dtype=torch.bfloat16, device="cuda")
z = torch.empty(B, 14, 14, 256, dtype=torch.bfloat16, device="cuda")
for _ in range(5):
    C.conv_chain(x, spec3, r, y, spec1, z)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
for _ in range(50):
    C.conv_chain(x, spec3, r, y, spec1, z)
e.record()
torch.cuda.synchronize()
print(f"EXP={os.environ.get('AIKO_CHAIN3_EXP', '0')} chain3 B=320: {s.elapsed_time(e) / 50 * 1e3:.1f} us", flush=True)
