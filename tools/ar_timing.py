"""Device time per tt_ar_allreduce_adam launch (the standalone peer-memory
exchange + Adam of the data-parallel step, cfg-3 gradient of 21,313 floats)
with W ranks sharing this box's one GPU (gloo for setup, the exchange itself
over IPC-mapped peer memory): MAX over ranks of the mean of K back-to-back
launches, timed with HIP events behind a short GPU spin.

usage: python tools/ar_timing.py W [K]      (CEO_TT_LIB selects a build)
"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _rank(rank, world, port, K, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import _native as N
        from ceo_firm_matching.distributed import PeerExchange
        dev = torch.device("cuda:0")
        n = 21313
        ex = PeerExchange.create(n, dist.group.WORLD, dev, mode="1")
        hp = N.adam_hp(4e-4)
        p, m, v = (torch.zeros(n, device=dev) for _ in range(3))
        x = torch.randn(n, device=dev)
        out = torch.empty_like(x)

        def launch():
            ex.epoch += 1
            ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=ex.epoch)
        res = []
        for _ in range(3):
            for _ in range(10):
                launch()
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(1_000_000)
            e0.record()
            for _ in range(K):
                launch()
            e1.record()
            torch.cuda.synchronize()
            t = torch.tensor([1e3 * e0.elapsed_time(e1) / K], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            res.append(float(t))
        ok = int(ex.err.item()) == 0
        ex.close()
        q.put((rank, res, ok))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), False))
        raise
    finally:
        dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=_rank, args=(r, world, port, K, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    r0 = sorted(res)[0]
    print(f"world {world}: tt_ar_allreduce_adam us per launch (3 rounds, MAX over ranks): {r0[1]}, "
          f"ok={all(r[2] for r in res)}, lib={os.path.basename(os.environ.get('CEO_TT_LIB', 'libceo_tt.so'))}")


if __name__ == "__main__":
    main()
