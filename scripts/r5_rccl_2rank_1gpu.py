"""Probe: can two ranks share one GPU under the RCCL backend?  (all_reduce, broadcast,
all_gather, send/recv).  Launched with torch.distributed.run --nproc-per-node 2."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.full((1024,), float(rank + 1), device="cuda")
dist.all_reduce(x)
ok = bool((x == 3).all())
y = torch.arange(8, device="cuda", dtype=torch.float32) * (rank + 1)
dist.broadcast(y, 0)
ok &= bool((y == torch.arange(8, device="cuda")).all())
g = [torch.empty(4, device="cuda") for _ in range(2)]
dist.all_gather(g, torch.full((4,), float(rank), device="cuda"))
ok &= bool((g[1] == 1).all())
if rank == 0:
    dist.send(torch.full((16,), 7.0, device="cuda"), 1)
else:
    r = torch.empty(16, device="cuda")
    dist.recv(r, 0)
    ok &= bool((r == 7).all())
torch.cuda.synchronize()
print(f"rank {rank}: rccl 2-rank/1-GPU collectives ok={ok}", flush=True)
dist.destroy_process_group()
