import torch
torch.cuda._sleep(1000)
torch.cuda.synchronize()
for n in (100000, 1000000):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); torch.cuda._sleep(n); e.record(); torch.cuda.synchronize()
    print(f"_sleep({n}): {s.elapsed_time(e) * 1e3:.1f} us -> {n / (s.elapsed_time(e) * 1e3):.1f} cycles/us", flush=True)
