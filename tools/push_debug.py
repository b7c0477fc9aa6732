"""Debug of the push exchange (tools/push_debug.py N) at world 2 on one GPU: one standalone launch,
then a dump of this rank's push rows (the words its peer stored)."""
import ctypes
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))


def rank_main(rank, world, port, n):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.distributed import PeerExchange
    dev = torch.device("cuda:0")
    ex = PeerExchange.create(n, dist.group.WORLD, dev, mode="1")
    ex.reset(dist.group.WORLD)
    ex.protocol = N.TT_AR_PUSH
    ex.wait_us = 200_000
    x = torch.full((n,), float(rank + 1), device=dev)
    out = torch.empty_like(x)
    ex.run(x, grad_out=out, step_host=1)
    torch.cuda.synchronize()
    err = int(ex.err.item())
    L = N.lib()
    rb = int(L.tt_ar_region_bytes(n))
    slot = (n + 63) // 64 * 64
    ll_bytes = 2 * 16 * slot * 8
    off = rb - ll_bytes
    buf = torch.empty(ll_bytes // 8, dtype=torch.int64, device=dev)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(ex.own + off), ctypes.c_size_t(ll_bytes), 3) == 0
    torch.cuda.synchronize()
    w = buf.cpu().numpy().view(np.uint64).reshape(2, 16, slot)
    nz = [(p, s, int((w[p, s] != 0).sum())) for p in range(2) for s in range(16) if (w[p, s] != 0).any()]
    print(f"rank {rank}: err {err}, out[:3] {out[:3].tolist()}, nonzero rows {nz}, "
          f"word[1][peer][0] {hex(int(w[1, 1 - rank, 0]))}", flush=True)
    dist.barrier()
    ex.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 21313
    mp.spawn(rank_main, args=(2, 29533, n), nprocs=2)
