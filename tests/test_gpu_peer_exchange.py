"""Data-parallel gradient exchange over peer memory (tt_ar_*, distributed.
PeerExchange): ranks are processes sharing the one GPU of the test box (the
IPC mapping and the flag protocol are the same as across xGMI; the fabric is
not).  Checked: the mean equals the reference sum / world and is bitwise the
same on every rank, the fused Adam equals torch's, both gradient slots (step
parity) and epochs > 2 work, and a full data-parallel FusedTrainer step on
the exchange matches the reference's DDP step (tests/golden/ddp.npz)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import excluded_param, load_golden, meta_of, normwise, sub

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    return sorted(res)


def _exchange_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import _native as N
        from ceo_firm_matching.distributed import PeerExchange
        dev = torch.device("cuda:0")
        n = 21313
        ex = PeerExchange.create(n, dist.group.WORLD, dev, mode="1")
        assert ex is not None, "peer exchange could not be set up"
        hp = N.adam_hp(4e-4)
        p = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(7))  # same on all ranks
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        pr, mr, vr = p.double().cpu(), torch.zeros(n, dtype=torch.float64), torch.zeros(n, dtype=torch.float64)
        worst, outs = 0.0, []
        for step in range(1, 7):
            gens = [torch.Generator().manual_seed(100 * step + r) for r in range(world)]
            xs = [torch.randn(n, generator=gg) for gg in gens]
            x = xs[rank].to(dev)
            out = torch.empty_like(x)
            ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=step)
            torch.cuda.synchronize()
            assert int(ex.err.item()) == 0
            ref = sum(t.double() for t in xs) / world
            worst = max(worst, float((out.cpu().double() - ref).abs().max() / ref.abs().max()))
            outs.append(out.cpu().numpy().copy())
            # torch Adam (fp64) on the reference mean
            mr = 0.9 * mr + 0.1 * ref
            vr = 0.999 * vr + 0.001 * ref * ref
            bc1, bc2 = 1 - 0.9 ** step, 1 - 0.999 ** step
            pr = pr - (4e-4 / bc1) * mr / ((vr.sqrt() / bc2 ** 0.5) + 1e-8)
        adam_err = float((p.cpu().double() - pr).abs().max() / pr.abs().max())
        allo = [None] * world
        dist.all_gather_object(allo, [o.tobytes() for o in outs])
        same = all(a == allo[0] for a in allo)
        q.put((rank, worst, adam_err, same))
        ex.close()
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, float("inf"), float("inf"), repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_peer_exchange_mean_and_adam(world):
    """The standalone exchange + Adam at world sizes on either side of the
    kernel's unrolled rank bounds (rank_order_sum<W>: W = 2, 4, 8; world 3
    loads this rank's own slot in the fourth lane): bitwise one mean on every
    rank, 1e-6 of the fp64 mean, Adam at 1e-5 of torch's fp64 formula."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    for rank, worst, adam_err, same in _spawn(_exchange_rank, world):
        assert same is True, (rank, same)  # bitwise the same mean on every rank
        assert worst < 1e-6, (rank, worst)
        assert adam_err < 1e-5, (rank, adam_err)


def _ddp_peer_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CEO_TT_PEER_AR="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import CEOFirmMatcher, Config
        from ceo_firm_matching.engine import FusedTrainer
        dev = torch.device("cuda:0")
        g = load_golden("ddp")
        meta = meta_of(load_golden("cfg2"))
        cfg = Config()
        cfg.LATENT_DIM = 64
        cfg.DROPOUT_P = 0.0
        cfg.DEVICE = dev
        m = CEOFirmMatcher(meta, cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
        m = m.to(dev)
        tr = FusedTrainer(m, lr=cfg.LEARNING_RATE, max_batch=64, seed=0, process_group=dist.group.WORLD)
        assert tr.peer is not None
        shard = {k: torch.from_numpy(v) for k, v in sub(g, f"G{world}/shard{rank}").items()}
        tr.set_data(shard)
        tr.step(None, 0, shard["target"].shape[0])
        tr.pop_loss_sum()
        ref = sub(g, f"G{world}/after_step")
        errs = {k: normwise(p.detach().cpu().numpy(), ref[k]) for k, p in m.named_parameters()
                if not excluded_param(k)}
        q.put((rank, max(errs.values()), max(errs, key=errs.get)))
    except Exception as e:
        q.put((rank, float("inf"), repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_data_parallel_step_on_peer_exchange(world):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    for rank, err, where in _spawn(_ddp_peer_rank, world):
        assert err < 1e-5, (rank, err, where)


def test_exchange_timeout_leaves_parameters_and_raises():
    """A peer that never launches: the waiting rank's exchange times out,
    leaves params / exp_avg / exp_avg_sq / grad_out untouched (never the local
    gradient), every later launch is a device-side no-op that publishes
    nothing, and the host check raises.  One process owns both regions (the
    second rank simply never runs)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.distributed import PeerExchange
    L = N.lib()
    dev = torch.device("cuda:0")
    n = 5000
    nbytes = int(L.tt_ar_region_bytes(n))
    regs = []
    for _ in range(2):
        r = ctypes.c_void_p()
        h = (ctypes.c_uint8 * N.TT_AR_HANDLE_BYTES)()
        N.check(L.tt_ar_alloc(nbytes, ctypes.byref(r), h), "tt_ar_alloc")
        regs.append(r.value)
    ex = PeerExchange(L, regs, regs[0], 0, 2, n, dev)
    ex.regions = [regs[0], None]  # close() must not IPC-close the second (local) region
    ex.wait_us = 20_000
    try:
        g = torch.Generator(device=dev).manual_seed(3)
        p = torch.randn(n, device=dev, generator=g)
        m = torch.randn(n, device=dev, generator=g).abs()
        v = torch.randn(n, device=dev, generator=g).abs()
        x = torch.randn(n, device=dev, generator=g)
        out = torch.full((n,), 7.0, device=dev)
        p0, m0, v0 = p.clone(), m.clone(), v.clone()
        hp = N.adam_hp(4e-4)
        ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=1)
        torch.cuda.synchronize()
        assert ex.failed()
        assert torch.equal(p, p0) and torch.equal(m, m0) and torch.equal(v, v0)
        assert bool((out == 7.0).all())
        # the peer's flag array holds rank 0's step-1 flags (published before the wait)
        flags1 = torch.empty(N.TT_AR_MAX_RANKS * 32, dtype=torch.int64, device=dev)
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(flags1.data_ptr()), ctypes.c_void_p(regs[1]),
                             ctypes.c_size_t(flags1.numel() * 8), 3) == 0  # device to device
        torch.cuda.synchronize()
        assert bool((flags1[:32] == 1).all())
        err_before = int(ex.err.item())
        # sticky: step 2 neither waits, nor publishes, nor updates
        ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=2)
        torch.cuda.synchronize()
        assert int(ex.err.item()) == err_before
        assert torch.equal(p, p0) and bool((out == 7.0).all())
        assert hip.hipMemcpy(ctypes.c_void_p(flags1.data_ptr()), ctypes.c_void_p(regs[1]),
                             ctypes.c_size_t(flags1.numel() * 8), 3) == 0
        torch.cuda.synchronize()
        assert bool((flags1[:32] == 1).all())
        with pytest.raises(RuntimeError, match="did not publish"):
            ex.check()
    finally:
        torch.cuda.synchronize()
        L.tt_ar_free(ctypes.c_void_p(regs[1]))
        ex.close()


def _ddp_fold_rank(rank, world, port, q):
    """B = 8192 per rank on the cfg-3 model: the folded BN0 backward
    (k_bwd_mid_fold + the reduce's P/Q combine, apply_adam = 0) feeding the
    peer exchange + Adam, vs the oracle's per-shard local-BN DDP step (ranks
    sharing the GPU: the two-launch form)."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CEO_TT_PEER_AR="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import CEOFirmMatcher, Config
        from ceo_firm_matching import _native as N
        from ceo_firm_matching.engine import FusedTrainer
        from oracle import two_tower as O
        dev = torch.device("cuda:0")
        g = load_golden("cfg3")
        meta = meta_of(g)
        B = 8192
        rng = np.random.default_rng(5)  # every rank draws all shards, keeps its own
        shards = []
        for _ in range(world):
            shards.append({
                "firm_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_firm_numeric"])).astype(np.float32)),
                "firm_cat": torch.zeros(B, 0, dtype=torch.int64),
                "ceo_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32)),
                "ceo_cat": torch.zeros(B, 0, dtype=torch.int64),
                "target": torch.from_numpy(rng.standard_normal((B, 1)).astype(np.float32)),
                "weights": torch.from_numpy(rng.uniform(1, 10, (B, 1)).astype(np.float32)),
            })
        cfg = Config()
        cfg.LATENT_DIM = int(g["meta/latent"])
        cfg.DROPOUT_P = 0.0
        cfg.DEVICE = dev
        m = CEOFirmMatcher(meta, cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
        m = m.to(dev)
        assert N.step_plan(m.tt_desc(), B)["folded_bn0_backward"]
        tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=0, process_group=dist.group.WORLD)
        assert tr.peer is not None
        tr.set_data({k: v.to(dev) for k, v in shards[rank].items()})
        tr.step(None, 0, B)
        tr.pop_loss_sum()
        P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
        buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
        buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
        avg = O.ddp_average_grads(P, buf, shards, p=0.0)
        O.Adam(P, lr=4e-4).step(P, avg)
        errs = {k: normwise(p.detach().cpu().double().numpy(), P[k].numpy()) for k, p in m.named_parameters()
                if not excluded_param(k)}
        q.put((rank, max(errs.values()), max(errs, key=errs.get)))
    except Exception as e:
        q.put((rank, float("inf"), repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_data_parallel_folded_step_on_peer_exchange():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    for rank, err, where in _spawn(_ddp_fold_rank, 2):
        assert err < 1e-5, (rank, err, where)


# ---- the exchange inside the step's gradient reduction (tt_train_step_dp) ----

def _cfg2_model(dev, g):
    from ceo_firm_matching import CEOFirmMatcher, Config
    cfg = Config()
    cfg.LATENT_DIM = 64
    cfg.DROPOUT_P = 0.1
    cfg.DEVICE = dev
    m = CEOFirmMatcher(meta_of(load_golden("cfg2")), cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
    return m.to(dev)


def _fused_vs_two_launch_rank(rank, world, port, q, steps):
    """K deterministic data-parallel steps with the exchange inside
    k_reduce_adam vs the same steps as reduce -> standalone exchange + Adam
    (fused_exchange forced off): bitwise the same parameters, Adam moments
    and BN buffers; parameters and moments the same on every rank."""
    import torch.distributed as dist
    # CEO_TT_FUSED_EX: the in-reduction exchange although the ranks share the
    # GPU (small kernels: the co-located ranks' steps still fit beside it)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CEO_TT_PEER_AR="1", CEO_TT_FUSED_EX="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching.engine import FusedTrainer
        dev = torch.device("cuda:0")
        g = load_golden("ddp")
        shard = {k: torch.from_numpy(v) for k, v in sub(g, f"G2/shard{rank % 2}").items()}
        B = shard["target"].shape[0]
        outs, times = [], None
        for fused in (True, False):
            m = _cfg2_model(dev, g)
            tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=5, process_group=dist.group.WORLD, deterministic=True)
            assert tr.peer is not None
            if not fused:
                tr.fused_exchange = False
            tr.set_data(shard)
            for _ in range(steps):
                tr.step(None, 0, B)
            tr.pop_loss_sum()
            assert tr.fused_exchange is fused, (fused, tr.fused_exchange)
            if fused:  # validation timed both forms (device us per step, MAX over ranks)
                times = tr.fused_vs_two_launch_us
            outs.append(np.concatenate([tr.arena.params.cpu().numpy(), tr.exp_avg.cpu().numpy(),
                                        tr.exp_avg_sq.cpu().numpy(), tr.arena.buffers.cpu().numpy()]))
            tr.peer.close()
        allo = [None] * world  # parameters and Adam moments (BN buffers are per rank: local statistics)
        dist.all_gather_object(allo, outs[0][:3 * tr.arena.params.numel()].tobytes())
        q.put((rank, bool(np.array_equal(outs[0], outs[1])), all(a == allo[0] for a in allo), times))
    except Exception as e:
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_exchange_inside_reduction_matches_two_launch_form(world):
    """World 1 (bench --dp): the N > 1 step degenerates to the single-GPU
    arithmetic; world 2 (two ranks on the test box's GPU): the in-reduction
    exchange equals the standalone exchange bitwise, and every rank holds the
    same parameters."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    res = _spawn(_fused_vs_two_launch_rank, world, 3)
    for rank, same, ranks_equal, times in res:
        assert same is True, (rank, same)
        assert ranks_equal is True, rank
        assert times is not None and all(0 < t < 1e5 for t in times), (rank, times)
    assert len({r[3] for r in res}) == 1  # one agreed pair of timings
    print(f"world {world}: fused vs two-launch step us {res[0][3]}")


@pytest.mark.parametrize("protocol", ["pull", "push"])
def test_exchange_inside_reduction_timeout_leaves_parameters(protocol):
    """tt_train_step_dp with a peer that never runs: the reduction's waits
    time out, parameters / Adam moments stay at their values (never an
    update from the local gradient alone), later steps are device-side
    no-ops for the exchange, and the host check raises -- on both protocols."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.distributed import PeerExchange
    from ceo_firm_matching.engine import FusedTrainer
    dev = torch.device("cuda:0")
    g = load_golden("ddp")
    m = _cfg2_model(dev, g)
    tr = FusedTrainer(m, lr=4e-4, max_batch=64, seed=5)
    L = N.lib()
    n = tr.arena.params.numel()
    nbytes = int(L.tt_ar_region_bytes(n))
    regs = []
    for _ in range(2):
        r = ctypes.c_void_p()
        h = (ctypes.c_uint8 * N.TT_AR_HANDLE_BYTES)()
        N.check(L.tt_ar_alloc(nbytes, ctypes.byref(r), h), "tt_ar_alloc")
        regs.append(r.value)
    ex = PeerExchange(L, regs, regs[0], 0, 2, n, dev)
    ex.regions = [regs[0], None]
    ex.wait_us = 20_000
    ex.protocol = N.TT_AR_PUSH if protocol == "push" else N.TT_AR_PULL
    try:
        tr.peer, tr.dp, tr.world, tr.fused_exchange = ex, True, 2, True  # (no validation: the peer never runs)
        shard = {k: torch.from_numpy(v) for k, v in sub(g, "G2/shard0").items()}
        tr.set_data(shard)
        B = shard["target"].shape[0]
        p0, m0, v0 = tr.arena.params.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone()
        with pytest.raises(RuntimeError, match="did not publish"):
            tr.step(None, 0, B)  # eager data-parallel steps check the exchange
        assert tr.fused_exchange is True
        assert torch.equal(tr.arena.params, p0) and torch.equal(tr.exp_avg, m0) and torch.equal(tr.exp_avg_sq, v0)
        err1 = int(ex.err.item())
        assert err1 > 0
        with pytest.raises(RuntimeError, match="did not publish"):
            tr.step(None, 0, B)
        torch.cuda.synchronize()
        assert int(ex.err.item()) == err1  # sticky: no new waits
        assert torch.equal(tr.arena.params, p0)
    finally:
        torch.cuda.synchronize()
        L.tt_ar_free(ctypes.c_void_p(regs[1]))
        ex.close()


def test_failed_exchange_leaves_no_stale_embedding_gradients():
    """tt_train_step_dp whose exchange times out must still clear the
    step's embedding-gradient accumulators (k_reduce_adam kind 1): a later
    step on the same workspace (here a single-GPU step after the error is
    cleared) gets exactly its own embedding gradients, not the failed step's
    added in.  Embedding geometry (meta_test), p = 0, vs the fp64 oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.distributed import PeerExchange
    from ceo_firm_matching.engine import FusedTrainer
    from oracle import two_tower as O
    dev = torch.device("cuda:0")
    g = load_golden("meta_test")
    meta = meta_of(g)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = 0.0
    cfg.DEVICE = dev
    m = CEOFirmMatcher(meta, cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
    m = m.to(dev)
    tr = FusedTrainer(m, lr=4e-4, max_batch=256, seed=5)
    L = N.lib()
    n = tr.arena.params.numel()
    nbytes = int(L.tt_ar_region_bytes(n))
    regs = []
    for _ in range(2):
        r = ctypes.c_void_p()
        h = (ctypes.c_uint8 * N.TT_AR_HANDLE_BYTES)()
        N.check(L.tt_ar_alloc(nbytes, ctypes.byref(r), h), "tt_ar_alloc")
        regs.append(r.value)
    ex = PeerExchange(L, regs, regs[0], 0, 2, n, dev)
    ex.regions = [regs[0], None]
    ex.wait_us = 20_000
    try:
        batch = {k: torch.from_numpy(v) for k, v in sub(g, "batch").items()}
        B = batch["target"].shape[0]
        tr.set_data(batch)
        tr.peer, tr.dp, tr.world, tr.fused_exchange = ex, True, 2, True
        with pytest.raises(RuntimeError, match="did not publish"):
            tr.step(None, 0, B)
        # clear the error, leave the exchange: the next step is a single-GPU one
        torch.cuda.synchronize()
        tr.peer, tr.dp, tr.world, tr.fused_exchange = None, False, 1, False
        tr.state[0] = 0  # the failed step did not count
        tr.step(None, 0, B)
        torch.cuda.synchronize()
        P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
        buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
        buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
        score, cache, _ = O.forward(P, buf, batch, train=True)
        _, dscore = O.weighted_mse(score, batch["target"], batch["weights"])
        grads = O.backward(P, cache, dscore)
        base = tr.arena.params.data_ptr()
        checked = 0
        for name, prm in m.named_parameters():
            if "embeddings" not in name:
                continue
            off = (prm.data_ptr() - base) // 4
            got = tr.grad[off:off + prm.numel()].view(prm.shape).cpu().double().numpy()
            assert normwise(got, grads[name].numpy()) < 1e-5, name
            checked += 1
        assert checked == len(meta["firm_cat_counts"]) + len(meta["ceo_cat_counts"])
    finally:
        torch.cuda.synchronize()
        L.tt_ar_free(ctypes.c_void_p(regs[1]))
        ex.close()


# ---- the push protocol (TT_AR_PUSH, round 6): value|epoch words stored into
# every peer's region, local polls -- bitwise the pull protocol's mean ------

def _push_vs_pull_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching import _native as N
        from ceo_firm_matching.distributed import PeerExchange
        dev = torch.device("cuda:0")
        res = {}
        for n in (21313, 300_017):  # cfg 3's arena; a slice of > AR_EPT x 256 per 32 blocks
            ex = PeerExchange.create(n, dist.group.WORLD, dev, mode="1")
            assert ex is not None, "peer exchange could not be set up"
            hp = N.adam_hp(4e-4)
            for proto in (N.TT_AR_PULL, N.TT_AR_PUSH):
                ex.reset(dist.group.WORLD)
                ex.protocol = proto
                p = torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
                m = torch.zeros(n, device=dev)
                v = torch.zeros(n, device=dev)
                outs = []
                for step in range(1, 5):  # both parities, epochs > 2
                    x = torch.randn(n, generator=torch.Generator().manual_seed(100 * step + rank)).to(dev)
                    out = torch.empty_like(x)
                    ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=step)
                    torch.cuda.synchronize()
                    assert int(ex.err.item()) == 0, (proto, step)
                    outs.append(out.cpu().numpy().copy())
                res[(n, proto)] = (np.concatenate(outs), p.cpu().numpy().copy(), m.cpu().numpy().copy(),
                                   v.cpu().numpy().copy())
            ex.close()
        same = all(all(np.array_equal(a, b) for a, b in zip(res[(n, N.TT_AR_PULL)], res[(n, N.TT_AR_PUSH)]))
                   for n in (21313, 300_017))
        digest = [res[k][0].tobytes() for k in sorted(res)]
        allo = [None] * world
        dist.all_gather_object(allo, digest)
        q.put((rank, same, all(a == allo[0] for a in allo)))
    except Exception as e:
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_push_exchange_bitwise_equals_pull(world):
    """The standalone exchange + Adam on the push protocol: every grad_out,
    parameter and Adam moment bitwise the pull protocol's, over four steps
    (both parities), at n = cfg 3's arena and at 300k elements (a grid of more
    than the pull form's 32 blocks), the same on every rank."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    for rank, same, ranks_equal in _spawn(_push_vs_pull_rank, world):
        assert same is True, (rank, same)
        assert ranks_equal is True, rank


def _forms_rank(rank, world, port, q, steps):
    """Every exchange form of the data-parallel step forced in turn
    (CEO_TT_EXCHANGE_FORM: chosen when the validation finds it bitwise equal
    to the reference form), K deterministic steps each: bitwise the same
    parameters, moments and buffers whichever form runs."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CEO_TT_PEER_AR="1", CEO_TT_FUSED_EX="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching.engine import FusedTrainer
        dev = torch.device("cuda:0")
        g = load_golden("ddp")
        shard = {k: torch.from_numpy(v) for k, v in sub(g, f"G2/shard{rank % 2}").items()}
        B = shard["target"].shape[0]
        outs, chosen, times = {}, {}, None
        for form in ("fused", "fused_push", "two_launch", "two_launch_push"):
            os.environ["CEO_TT_EXCHANGE_FORM"] = form
            m = _cfg2_model(dev, g)
            tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=5, process_group=dist.group.WORLD, deterministic=True)
            tr.set_data(shard)
            for _ in range(steps):
                tr.step(None, 0, B)
            tr.pop_loss_sum()
            chosen[form] = tr.exchange_form
            times = tr.exchange_form_us
            outs[form] = np.concatenate([tr.arena.params.cpu().numpy(), tr.exp_avg.cpu().numpy(),
                                         tr.exp_avg_sq.cpu().numpy(), tr.arena.buffers.cpu().numpy()])
            tr.peer.close()
        os.environ.pop("CEO_TT_EXCHANGE_FORM")
        same = all(np.array_equal(outs["fused"], o) for o in outs.values())
        q.put((rank, same, chosen, times))
    except Exception as e:
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_every_exchange_form_gives_the_same_step(world):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    res = _spawn(_forms_rank, world, 3)
    for rank, same, chosen, times in res:
        assert same is True, (rank, same)
        assert chosen == {f: f for f in chosen}, (rank, chosen)  # each forced form passed the bitwise check
        assert set(times) == {"two_launch", "fused", "fused_push", "two_launch_push"}, times
    print(f"world {world}: exchange form us {res[0][3]}")


def test_push_exchange_timeout_leaves_parameters_and_raises():
    """The standalone push exchange with a peer that never runs: every block
    times out and leaves its slice of params / exp_avg / exp_avg_sq /
    grad_out untouched, the words it stored are in the peer's region (epoch
    1, this rank's row), later launches are device-side no-ops, the host
    check raises."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.distributed import PeerExchange
    L = N.lib()
    dev = torch.device("cuda:0")
    n = 5000
    nbytes = int(L.tt_ar_region_bytes(n))
    regs = []
    for _ in range(2):
        r = ctypes.c_void_p()
        h = (ctypes.c_uint8 * N.TT_AR_HANDLE_BYTES)()
        N.check(L.tt_ar_alloc(nbytes, ctypes.byref(r), h), "tt_ar_alloc")
        regs.append(r.value)
    ex = PeerExchange(L, regs, regs[0], 0, 2, n, dev)
    ex.regions = [regs[0], None]
    ex.wait_us = 20_000
    ex.protocol = N.TT_AR_PUSH
    try:
        g = torch.Generator(device=dev).manual_seed(3)
        p = torch.randn(n, device=dev, generator=g)
        m = torch.randn(n, device=dev, generator=g).abs()
        v = torch.randn(n, device=dev, generator=g).abs()
        x = torch.randn(n, device=dev, generator=g)
        out = torch.full((n,), 7.0, device=dev)
        p0, m0, v0 = p.clone(), m.clone(), v.clone()
        hp = N.adam_hp(4e-4)
        ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=1)
        torch.cuda.synchronize()
        assert ex.failed()
        assert torch.equal(p, p0) and torch.equal(m, m0) and torch.equal(v, v0)
        assert bool((out == 7.0).all())
        # the peer's region holds this rank's words: row [parity 1][source 0], epoch 1 | x
        slot = (n + 63) // 64 * 64
        ll_off = nbytes - 2 * N.TT_AR_MAX_RANKS * slot * 8
        words = torch.empty(n, dtype=torch.int64, device=dev)
        hip = ctypes.CDLL("libamdhip64.so")
        row = ll_off + (1 * N.TT_AR_MAX_RANKS + 0) * slot * 8
        assert hip.hipMemcpy(ctypes.c_void_p(words.data_ptr()), ctypes.c_void_p(regs[1] + row),
                             ctypes.c_size_t(n * 8), 3) == 0
        torch.cuda.synchronize()
        w = words.cpu().numpy().view(np.uint64)
        assert bool(((w >> np.uint64(32)) == 1).all())
        assert np.array_equal((w & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.float32), x.cpu().numpy())
        err_before = int(ex.err.item())
        ex.run(x, grad_out=out, params=p, exp_avg=m, exp_avg_sq=v, hp=hp, step_host=2)  # sticky
        torch.cuda.synchronize()
        assert int(ex.err.item()) == err_before
        assert torch.equal(p, p0) and bool((out == 7.0).all())
        with pytest.raises(RuntimeError, match="did not publish"):
            ex.check()
    finally:
        torch.cuda.synchronize()
        L.tt_ar_free(ctypes.c_void_p(regs[1]))
        ex.close()
