"""BASELINE cfg 4: 8 data-parallel ranks, each one B = 16384
batch of the cfg-3 model (64 x 64 features, LATENT 128, dropout 0.1) with
LOCAL BatchNorm statistics, the gradient averaged over the ranks, one Adam
step -- the reference loop (training.py:44-57) under DDP.

The ranks are processes sharing the test box's one GPU (the 8-GPU run is the
driver's); the exchange is the peer-memory one (two-launch form: the fused
step stops at the gradient, tt_ar_allreduce_adam averages in rank order and
applies Adam) or gloo.  Checked against the fp64 oracle's 8-shard DDP step
(oracle ddp semantics: per-shard forward / backward, mean of the shards'
gradients, torch Adam), on unscreened data: the mean gradient and the
parameters inside the oracle's bound over ReLU branch choices at kink
elements (tests/kinks.py; = the 1e-5 normwise bar wherever no kink reaches),
and bitwise the same parameters on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import excluded_param, load_golden, meta_of, sub
from kinks import adam1_bounds, adam1_replay_error, bound_error, grad_bounds, kink_elements

pytestmark = pytest.mark.gpu
TOL = 1e-5
WORLD, B, P_DROP, SEED = 8, 16384, 0.1, 2024


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard(meta, r):
    rng = np.random.default_rng(5000 + r)
    return {
        "firm_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.zeros(B, 0, dtype=torch.int64),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.zeros(B, 0, dtype=torch.int64),
        "target": torch.from_numpy(rng.standard_normal((B, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (B, 1)).astype(np.float32)),
    }


def _rank(rank, world, port, q, exchange):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      CEO_TT_PEER_AR="1" if exchange == "peer" else "0")
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import CEOFirmMatcher, Config
        from ceo_firm_matching import _native as N
        from ceo_firm_matching.engine import FusedTrainer
        dev = torch.device("cuda:0")
        g = load_golden("cfg3")
        meta = meta_of(g)
        cfg = Config()
        cfg.LATENT_DIM = int(g["meta/latent"])
        cfg.DROPOUT_P = P_DROP
        cfg.DEVICE = dev
        m = CEOFirmMatcher(meta, cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
        m = m.to(dev)
        assert N.step_plan(m.tt_desc(), B)["folded_bn0_backward"]
        tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=SEED, process_group=dist.group.WORLD)
        assert (tr.peer is not None) == (exchange == "peer")
        tr.set_data({k: v.to(dev) for k, v in _shard(meta, rank).items()})
        tr.step(None, 0, B)
        loss = tr.pop_loss_sum()
        torch.cuda.synchronize()
        flat = tr.arena.params.cpu().numpy().copy()
        allp = [None] * world
        dist.all_gather_object(allp, flat.tobytes())
        q.put((rank, tr.grad.cpu().numpy().copy(), flat, all(a == allp[0] for a in allp), loss,
               tr.steps_done(), tr.exp_avg.cpu().numpy().copy(), tr.exp_avg_sq.cpu().numpy().copy()))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), None, False, None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def _oracle_bounds():
    """Mean over the 8 shards of the oracle's gradient and of its kink
    bounds, and the Adam-step parameter bounds."""
    from oracle import two_tower as O
    g = load_golden("cfg3")
    meta = meta_of(g)
    P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
    buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
    buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
    masks = {(t, l): torch.from_numpy(O.dropout_keep_mask(SEED, 1, t, l, B, H, P_DROP)).double()
             for t in range(2) for l, H in enumerate((64, 32))}
    gsum = lsum = hsum = None
    losses, n_kinks = [], 0
    for r in range(WORLD):
        data = _shard(meta, r)
        score, cache, _ = O.forward(P, buf, data, train=True, masks=masks, p=P_DROP)
        loss, dscore = O.weighted_mse(score, data["target"], data["weights"])
        losses.append(float(loss))
        grads = O.backward(P, cache, dscore)
        elems = kink_elements(cache, masks)
        n_kinks += len(elems)
        lo, hi = grad_bounds(O, P, cache, dscore, elems)
        if gsum is None:
            gsum, lsum, hsum = grads, lo, hi
        else:
            for k in gsum:
                gsum[k] = gsum[k] + grads[k]
                lsum[k] = lsum[k] + lo[k]
                hsum[k] = hsum[k] + hi[k]
    avg = {k: v / WORLD for k, v in gsum.items()}
    lo = {k: v / WORLD for k, v in lsum.items()}
    hi = {k: v / WORLD for k, v in hsum.items()}
    plo, phi = adam1_bounds(O, P, lo, hi, 4e-4, ref=avg, slack=TOL)
    return meta, avg, lo, hi, plo, phi, losses, n_kinks


def _slots(meta):
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching import _native as N
    cfg = Config()
    cfg.LATENT_DIM = 128
    cfg.DEVICE = torch.device("cpu")
    m = CEOFirmMatcher(meta, cfg)
    a = m.bind_arena()
    return [(name, p.shape, off) for name, p, off in m._named_slots(N.param_offsets(a.desc))]


@pytest.mark.parametrize("exchange", ["peer", "gloo"])
def test_cfg4_eight_ranks_one_step_vs_oracle_ddp(exchange):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, WORLD, port, q, exchange)) for r in range(WORLD)]
    for p in ps:
        p.start()
    try:
        meta, avg, lo, hi, plo, phi, losses, n_kinks = _oracle_bounds()
        res = sorted((q.get(timeout=300) for _ in ps), key=lambda r: r[0])
    finally:
        for p in ps:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps), [(p.exitcode, r[1] if isinstance(r[1], str) else "") for p, r in
                                              zip(ps, res)]
    slots = _slots(meta)
    g = load_golden("cfg3")
    init = {k: np.asarray(v, np.float32) for k, v in sub(g, "init").items()}
    for rank, grad, params, same, loss, steps, m1, v1 in res:
        assert same is True, rank
        assert steps == 1
        assert abs(loss - losses[rank]) <= TOL * abs(losses[rank]), (rank, loss, losses[rank])
        for name, shape, off in slots:
            if excluded_param(name):
                continue
            n = int(np.prod(shape)) if len(shape) else 1
            eg = bound_error(grad[off:off + n], lo[name].numpy(), hi[name].numpy(), avg[name].numpy())
            assert eg < TOL, ("grad", rank, name, eg, n_kinks)
            ep = bound_error(params[off:off + n], plo[name].numpy(), phi[name].numpy(), plo[name].numpy())
            assert ep < TOL, ("param", rank, name, ep, n_kinks)
        for name, shape, off in slots:  # Adam on the exchanged mean gradient, element by element
            n = int(np.prod(shape)) if len(shape) else 1
            sl = slice(off, off + n)
            ea = adam1_replay_error(init[name].reshape(-1), grad[sl], params[sl], m1[sl], v1[sl], 4e-4)
            assert ea < 1.0, ("adam replay", rank, name, ea)
