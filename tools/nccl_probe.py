"""Dev probe: RCCL process group at world size 1 -- eager all_reduce and graph capture."""
import os, sys, time
import torch, torch.distributed as dist
print("start", flush=True)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
print("init ok", flush=True)
x = torch.ones(1000, device=dev)
dist.all_reduce(x); torch.cuda.synchronize()
print("eager all_reduce ok", float(x.sum()), flush=True)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        dist.all_reduce(x)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    dist.all_reduce(x); x.mul_(0.5)
g.replay(); torch.cuda.synchronize()
print("graph all_reduce ok", float(x.sum()), flush=True)
t0 = time.perf_counter()
for _ in range(100): dist.all_reduce(x)
torch.cuda.synchronize(); print("eager us/all_reduce", (time.perf_counter()-t0)*1e4, flush=True)
dist.destroy_process_group()
print("done", flush=True)
