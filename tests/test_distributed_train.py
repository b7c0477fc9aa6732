"""Data-parallel ``train_model`` (the north-star ``train()`` entry under
torchrun; SURVEY 8e, BASELINE cfg 4) on CPU over gloo.

* ``distributed.rank_epoch_order`` is torch's ``DistributedSampler`` order
  (seed + epoch permutation, padded to ceil(N / world) per rank);
* ``training.dp_epoch_order_plan`` gives the batches a DataLoader over that
  sampler yields;
* ``train_model`` with 2 ranks (reference CLI data, p = 0, 2 epochs) equals
  an oracle DDP loop: per-rank DistributedSampler shards, local BatchNorm
  statistics, gradients averaged over ranks, torch Adam -- on every rank,
  with the epoch lines printed by rank 0 only.

``oracle_ddp_train`` is shared with the GPU test of the fused path
(tests/test_gpu_training.py)."""
import contextlib
import io
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from conftest import excluded_param, normwise
from oracle import two_tower as O

TOL_TRAINED = 1e-4  # a few Adam steps (tests/test_gpu_training.py: TOL_TRAINED)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [1, 7, 800, 1003])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_epoch_order_is_distributed_sampler(n, world):
    from ceo_firm_matching.distributed import rank_epoch_order
    for shuffle in (True, False):
        for drop_last in ((False, True) if n >= world else (False,)):
            for epoch in (0, 3):
                for rank in range(world):
                    s = DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=shuffle, seed=5,
                                           drop_last=drop_last)
                    s.set_epoch(epoch)
                    got = rank_epoch_order(n, epoch, rank, world, shuffle=shuffle, seed=5, drop_last=drop_last)
                    assert got.tolist() == list(s), (n, world, rank, shuffle, drop_last, epoch)


def test_dp_epoch_order_plan_matches_a_distributed_loader():
    from ceo_firm_matching.training import dp_epoch_order_plan
    ds = torch.arange(1003)
    for bs, drop in ((256, False), (100, True)):
        for rank in range(3):
            plain = DataLoader(ds, batch_size=bs, shuffle=True, drop_last=drop)
            samp = DistributedSampler(ds, num_replicas=3, rank=rank, shuffle=True)
            ref = DataLoader(ds, batch_size=bs, sampler=samp, drop_last=drop)
            for epoch in range(3):
                samp.set_epoch(epoch)
                want = [b.tolist() for b in ref]
                # the global RNG is drawn like iter(loader): same state after both
                torch.manual_seed(epoch)
                order, sizes = dp_epoch_order_plan(plain, epoch, rank, 3)()
                after_plan = torch.rand(1)
                torch.manual_seed(epoch)
                iter(ref)
                after_iter = torch.rand(1)
                assert torch.equal(after_plan, after_iter)
                got, off = [], 0
                for s in sizes:
                    got.append(order[off:off + s].tolist())
                    off += s
                assert got == want, (bs, drop, rank, epoch)


def oracle_ddp_train(train, cfg, world, epochs, seed, bs=256):
    """The reference loop (training.py:36-57) under DDP, restated on the fp64
    oracle: parameters drawn as CEOFirmMatcher(train, cfg) does after
    torch.manual_seed(seed); per epoch, rank r's batches are
    DistributedSampler(num_replicas=world, rank=r, shuffle=True, seed=0) after
    set_epoch(epoch); each step averages the ranks' local-BN gradients and
    takes torch's Adam step.  Returns (params, rank 0's BN buffers, steps)."""
    meta = {k: train[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    torch.manual_seed(seed)
    P = O.init_params_like_reference(meta, cfg.LATENT_DIM, cfg.EMBEDDING_DIM_LARGE, cfg.EMBEDDING_DIM_MEDIUM)
    P = {k: v.double() for k, v in P.items()}
    buf = {k: (v if "num_batches" in k else v.double()) for k, v in O.fresh_buffers().items()}
    opt = O.Adam(P, lr=cfg.LEARNING_RATE)
    n = len(train["target"])
    keys = ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target", "weights")
    steps = 0
    for epoch in range(epochs):
        orders = []
        for r in range(world):
            s = DistributedSampler(range(n), num_replicas=world, rank=r, shuffle=True, seed=0)
            s.set_epoch(epoch)
            orders.append(torch.tensor(list(s), dtype=torch.int64))
        per = len(orders[0])
        for off in range(0, per, bs):
            shards = [{k: train[k][o[off:off + bs]] for k in keys} for o in orders]
            avg = O.ddp_average_grads(P, buf, shards, p=0.0)
            _, _, buf = O.forward(P, buf, shards[0], train=True)  # rank 0's local running stats
            opt.step(P, avg)
            steps += 1
    return P, buf, steps


def check_against_oracle(sd, P, buf, steps, lr):
    """Normwise parity of a trained state_dict with the oracle DDP run."""
    bad = {}
    for k, ref in list(P.items()) + list(buf.items()):
        if excluded_param(k):
            continue
        got = torch.as_tensor(sd[k])
        if "num_batches" in k:
            assert int(got) == int(ref) == steps, k
        elif "running_mean" in k:  # carries the pre-BN bias: absolute steps * lr
            assert float((got.double() - ref).abs().max()) <= steps * lr, k
        else:
            e = normwise(got.double().numpy(), ref.numpy())
            if e >= TOL_TRAINED:
                bad[k] = e
    assert not bad, bad


def _ddp_train_rank(rank, world, port, q, device, epochs, seed):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import Config
        from ceo_firm_matching.data import CEOFirmDataset
        from ceo_firm_matching.training import train_model
        from test_host_pipeline import cli_data
        cfg = Config()
        cfg.EPOCHS = epochs
        cfg.DROPOUT_P = 0.0
        cfg.DEVICE = torch.device(device)
        train, _ = cli_data(cfg)
        torch.manual_seed(seed)
        tl = DataLoader(CEOFirmDataset(train), batch_size=256, shuffle=True)
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            model = train_model(tl, None, train, cfg)
        sd = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
        flat = torch.cat([p.detach().cpu().reshape(-1) for p in model.parameters()])
        allp = [None] * world
        dist.all_gather_object(allp, flat.numpy().tobytes())
        steps = model._trainer.steps_done() if hasattr(model, "_trainer") else None
        q.put((rank, sd, out.getvalue(), all(a == allp[0] for a in allp), steps))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), "", False, None))
        raise
    finally:
        dist.destroy_process_group()


def run_ddp_train(world, device, epochs=2, seed=4321):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_train_rank, args=(r, world, port, q, device, epochs, seed)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=600) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps), [(p.exitcode, r[1] if isinstance(r[1], str) else "") for p, r in
                                              zip(ps, res)]
    return res


def test_train_model_data_parallel_gloo_cpu():
    from ceo_firm_matching import Config
    from test_host_pipeline import cli_data
    world, epochs, seed = 2, 2, 4321
    res = run_ddp_train(world, "cpu", epochs, seed)
    cfg = Config()
    cfg.DROPOUT_P = 0.0
    train, _ = cli_data(cfg)
    P, buf, steps = oracle_ddp_train(train, cfg, world, epochs, seed)
    assert steps == epochs * 2  # 800 pairs -> 400 per rank -> batches of 256 + 144
    for rank, sd, printed, same, _ in res:
        assert same is True, rank  # every rank holds the same parameters
        lines = [ln for ln in printed.splitlines() if ln.startswith(("Epoch", "Starting"))]
        assert len(lines) == (2 if rank == 0 else 0), (rank, lines)  # rank 0 prints
        if rank == 0:
            check_against_oracle(sd, P, buf, steps, cfg.LEARNING_RATE)
