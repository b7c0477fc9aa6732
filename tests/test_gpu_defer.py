"""Deferred late half of the gradient reduction (TT_FLAG_DEFER_LATE,
DESIGN 10): a step's W4 / BN1-affine / W8 / logit_scale reduction + Adam and
its loss fold run inside the NEXT step's first kernel (or in tt_train_flush),
so the step keeps five launches and that work leaves the critical path.

* K deferred steps back to back, then the flush: the same training as K
  plain steps (training.py:44-57) -- parameters, Adam moments, BN buffers
  and the loss sum (the late half sums its slabs in another fixed order, so
  at the optimizer-scale bound, as graph-vs-eager in atomic mode), and both
  against the fp64 oracle's K-step trajectory at the trained bar;
* graph-replayed deferred steps are bitwise the eager deferred steps
  (deterministic mode), across the replay boundaries;
* a stale TT_FLAG_LATE_PENDING (nothing deferred on the workspace) is a
  no-op on the device: bitwise the plain step;
* a batch-size change flushes first; reading the model (state_dict, forward)
  flushes.
"""
import numpy as np
import pytest
import torch

from conftest import excluded_param, load_golden, meta_of, normwise, sub

pytestmark = pytest.mark.gpu
B = 16384


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _setup(p=0.1, n_rows=8 * B, seed=5):
    from ceo_firm_matching import CEOFirmMatcher, Config
    g = load_golden("cfg3")
    meta = meta_of(g)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = p
    cfg.DEVICE = _dev()
    rng = np.random.default_rng(seed)
    data = {
        "firm_numeric": torch.from_numpy(rng.standard_normal((n_rows, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.zeros(n_rows, 0, dtype=torch.int64),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((n_rows, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.zeros(n_rows, 0, dtype=torch.int64),
        "target": torch.from_numpy(rng.standard_normal((n_rows, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (n_rows, 1)).astype(np.float32)),
    }
    init = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()}

    def make(defer, det=True, max_batch=B):
        from ceo_firm_matching.engine import FusedTrainer
        m = CEOFirmMatcher(meta, cfg)
        m.load_state_dict(init)
        m = m.to(_dev())
        tr = FusedTrainer(m, lr=4e-4, max_batch=max_batch, seed=77, deterministic=det, defer_late=defer)
        tr.set_data({k: v.to(_dev()) for k, v in data.items()})
        return m, tr
    return g, meta, data, make


def _state(m, tr):
    tr.flush()
    torch.cuda.synchronize()
    return np.concatenate([tr.arena.params.cpu().numpy(), tr.exp_avg.cpu().numpy(), tr.exp_avg_sq.cpu().numpy(),
                           tr.arena.buffers.cpu().numpy()])


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_deferred_steps_equal_plain_steps_and_the_oracle(p):
    from oracle import two_tower as O
    g, meta, data, make = _setup(p=p)
    K = 4
    out = {}
    for defer in (False, True):
        m, tr = make(defer)
        for k in range(K):
            tr.step(None, k * B, B)
        assert tr._late_rows == (B if defer else 0)
        loss = tr.pop_loss_sum()  # flushes the last late half first
        assert tr._late_rows == 0 and m._pending_flush is None
        assert tr.steps_done() == K
        out[defer] = ({n: q.detach().cpu().double().numpy().copy() for n, q in m.named_parameters()}, loss,
                      {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items() if "running" in k})
    (pp, lp, bp), (pd, ld, bd) = out[False], out[True]
    assert abs(ld - lp) <= 1e-5 * abs(lp), (ld, lp)
    lr_steps = 4e-4 * K
    for n in pp:
        if excluded_param(n):
            continue
        ok = normwise(pd[n], pp[n]) < 1e-5 or np.max(np.abs(pd[n] - pp[n])) <= 5e-2 * lr_steps
        assert ok, (n, normwise(pd[n], pp[n]))
    for k in bp:
        if "running_mean" in k:
            assert np.max(np.abs(bd[k] - bp[k])) <= lr_steps, k
        else:
            assert normwise(bd[k], bp[k]) < 1e-5, k
    # the deferred run against the fp64 oracle's trajectory (its masks: the kernels' hash stream)
    P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
    buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
    buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
    opt = O.Adam(P, lr=4e-4)
    l64 = 0.0
    for k in range(K):
        bk = {n: v[k * B:(k + 1) * B] for n, v in data.items()}
        masks = None
        if p > 0:
            masks = {(t, l): torch.from_numpy(O.dropout_keep_mask(77, k + 1, t, l, B, H, p)).double()
                     for t in range(2) for l, H in enumerate((64, 32))}
        loss, _, buf = O.train_step(P, buf, opt, bk, masks=masks, p=p)
        l64 += float(loss)
    assert abs(ld - l64) <= 1e-5 * abs(l64), (ld, l64)
    for n, v in P.items():
        if excluded_param(n):
            continue
        ok = normwise(pd[n], v.numpy()) < 1e-4 or np.max(np.abs(pd[n] - v.numpy())) <= 5e-2 * lr_steps
        assert ok, (n, normwise(pd[n], v.numpy()))


def test_deferred_graph_replay_bitwise_equals_eager():
    """Cycle-mode deferred steps replayed from two captured 4-step graphs vs
    the same 8 steps eager: bitwise (deterministic mode), loss included."""
    _, _, data, make = _setup(p=0.1)
    rows = torch.randperm(8 * B, device=_dev(), generator=torch.Generator(device=_dev()).manual_seed(3))
    res = []
    for use_graph in (False, True):
        m, tr = make(True)
        tr.step_cycle(rows, B, 8)  # eager first step: the graphs start with a late half pending
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(4):
                    tr.step_cycle(rows, B, 8)
            graph.replay()
            graph.replay()
        else:
            for _ in range(8):
                tr.step_cycle(rows, B, 8)
        loss = tr.pop_loss_sum()
        res.append((_state(m, tr), loss, tr.steps_done()))
    (a, la, na), (b, lb, nb) = res
    assert na == nb == 9
    assert la == lb
    assert np.array_equal(a, b)


def test_stale_pending_flag_is_a_noop():
    """TT_FLAG_LATE_PENDING with nothing deferred on the workspace (a host
    that lost track) runs no late half: bitwise the plain step."""
    from ceo_firm_matching import _native as N
    _, _, _, make = _setup(p=0.1)
    res = []
    for stale in (False, True):
        m, tr = make(False)
        tr.step(None, 0, B)
        if stale:  # pretend the previous step deferred: the next step carries a late half
            tr._late_rows, tr._late_batch = B, tr._batch(None, 0, B)
        tr.step(None, B, B)
        assert tr._late_rows == 0
        res.append((_state(m, tr), tr.pop_loss_sum()))
    (a, la), (b, lb) = res
    assert la == lb and np.array_equal(a, b)
    assert N.lib().tt_train_flush is not None


def test_batch_size_change_and_model_reads_flush():
    from ceo_firm_matching import _native as N
    _, _, data, make = _setup(p=0.0)
    sizes = [B, B, 12288, 12288, B]
    out = []
    for defer in (False, True):
        m, tr = make(defer)
        off = 0
        for bs in sizes:
            tr.step(None, off, bs)
            off += bs
        if defer:
            assert tr._late_rows == B and m._pending_flush is not None
            sd = m.state_dict()  # reading the model finishes the deferred step
            assert tr._late_rows == 0 and m._pending_flush is None
            with torch.no_grad():
                m.eval()
                s1 = m(data["firm_numeric"][:256].to(_dev()), data["firm_cat"][:256].to(_dev()),
                       data["ceo_numeric"][:256].to(_dev()), data["ceo_cat"][:256].to(_dev()))
        else:
            sd = m.state_dict()
        out.append(({k: v.detach().cpu().double().numpy().copy() for k, v in sd.items()}, tr.pop_loss_sum()))
    (a, la), (b, lb) = out
    assert abs(la - lb) <= 1e-5 * abs(la)
    for k in a:
        if excluded_param(k) or "num_batches" in k or "running_mean" in k:
            continue
        ok = normwise(b[k], a[k]) < 1e-5 or np.max(np.abs(b[k] - a[k])) <= 5e-2 * 4e-4 * len(sizes)
        assert ok, (k, normwise(b[k], a[k]))
    assert N.step_plan(m.tt_desc(), 12288)["folded_bn0_backward"]


def test_workspace_growth_flushes_the_pending_late_half():
    """A step whose batch exceeds the trainer's max_batch replaces the
    workspace: the previous step's pending late half (its slabs, replicas and
    deferral record live there) must run first.  Deferred steps
    of 8192 rows on an 8192-row workspace, then 16384-row steps: the same
    training as plain steps, loss included."""
    from ceo_firm_matching import _native as N
    _, _, data, make = _setup(p=0.0)
    sizes = [B // 2, B // 2, B, B]
    out = []
    for defer in (False, True):
        m, tr = make(defer, max_batch=B // 2)
        off = 0
        for bs in sizes:
            tr.step(None, off, bs)
            off += bs
        assert tr.max_batch == B and tr.steps_done() == len(sizes)
        loss = tr.pop_loss_sum()
        sd = m.state_dict()
        mom = {}
        for name, prm, off in m._named_slots(N.param_offsets(tr.desc)):
            mom[name] = tuple(t[off:off + prm.numel()].cpu().double().numpy().copy() for t in (tr.exp_avg, tr.exp_avg_sq))
        out.append(({k: v.detach().cpu().double().numpy().copy() for k, v in sd.items()}, loss, mom))
    (a, la, ma), (b, lb, mb) = out
    assert abs(la - lb) <= 1e-5 * abs(la), (la, lb)
    # Adam moments of every parameter but the pre-BN biases: normwise, at the
    # gradients' reduction-order level (a lost late half would leave W4 / W8 /
    # logit_scale's moments a whole step behind: O(1) relative)
    for k in ma:
        if excluded_param(k):
            continue
        for i, what in enumerate(("exp_avg", "exp_avg_sq")):
            assert normwise(mb[k][i], ma[k][i]) < 1e-4, (k, what, normwise(mb[k][i], ma[k][i]))
    # parameters at the optimizer-scale bound (the late half sums its slabs in
    # another fixed order; the pre-BN biases, whose true gradient is 0, and
    # the running means that carry them are excluded as everywhere else): a
    # lost late half moves W4 / W8 / logit_scale by a whole Adam step (lr)
    for k in a:
        if excluded_param(k) or "num_batches" in k or "running_mean" in k:
            continue
        ok = normwise(b[k], a[k]) < 1e-5 or np.max(np.abs(b[k] - a[k])) <= 5e-2 * 4e-4 * len(sizes)
        assert ok, (k, normwise(b[k], a[k]), np.max(np.abs(b[k] - a[k])))


def test_dropped_trainer_keeps_its_pending_late_half():
    """A FusedTrainer(defer_late=True) dropped while a late half is pending
    (ADVICE r05): the model keeps the trainer's flush alive until it reads its
    parameters, so state_dict() after `del trainer` is the plain run's."""
    import gc
    _, _, data, make = _setup(p=0.0)
    out = []
    for defer in (False, True):
        m, tr = make(defer)
        for k in range(3):
            tr.step(None, k * B, B)
        if defer:
            assert m._pending_flush is not None
        ref = tr.model  # noqa: F841 -- the model outlives the trainer
        del tr
        gc.collect()
        sd = m.state_dict()
        assert m._pending_flush is None
        out.append({k: v.detach().cpu().double().numpy().copy() for k, v in sd.items()})
    a, b = out
    for k in a:
        if excluded_param(k) or "num_batches" in k or "running_mean" in k:
            continue
        # a lost late half would leave W4 / W8 / logit_scale a whole Adam step (lr) behind
        ok = normwise(b[k], a[k]) < 1e-5 or np.max(np.abs(b[k] - a[k])) <= 5e-2 * 4e-4 * 3
        assert ok, (k, normwise(b[k], a[k]), np.max(np.abs(b[k] - a[k])))


def test_deferred_six_kernel_path_cfg2():
    """The cfg-2 geometry (32 x 32 features, LATENT 64, B = 4000: the
    six-kernel path, no folded BN0 backward) deferred vs plain: the same
    training at the optimizer-scale bound, loss at 1e-5."""
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.engine import FusedTrainer
    g = load_golden("cfg2")
    meta = meta_of(g)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = 0.1
    cfg.DEVICE = _dev()
    Bc, K = 4000, 5
    rng = np.random.default_rng(12)
    data = {
        "firm_numeric": torch.from_numpy(rng.standard_normal((K * Bc, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.zeros(K * Bc, 0, dtype=torch.int64),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((K * Bc, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.zeros(K * Bc, 0, dtype=torch.int64),
        "target": torch.from_numpy(rng.standard_normal((K * Bc, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (K * Bc, 1)).astype(np.float32)),
    }
    out = []
    for defer in (False, True):
        m = CEOFirmMatcher(meta, cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
        m = m.to(_dev())
        assert not N.step_plan(m.tt_desc(), Bc)["folded_bn0_backward"]
        tr = FusedTrainer(m, lr=4e-4, max_batch=Bc, seed=9, deterministic=True, defer_late=defer)
        tr.set_data({k: v.to(_dev()) for k, v in data.items()})
        for k in range(K):
            tr.step(None, k * Bc, Bc)
        assert tr._late_rows == (Bc if defer else 0)
        loss = tr.pop_loss_sum()
        out.append(({n: q.detach().cpu().numpy().copy() for n, q in m.named_parameters()}, loss))
    (a, la), (b, lb) = out
    assert abs(la - lb) <= 1e-5 * abs(la)
    for n in a:
        if excluded_param(n):
            continue
        ok = normwise(b[n], a[n]) < 1e-5 or np.max(np.abs(b[n] - a[n])) <= 5e-2 * 4e-4 * K
        assert ok, (n, normwise(b[n], a[n]))


def test_replays_after_a_flush_keep_every_late_half():
    """bench.py's timed region: a flush before the replays (the warm-up loss
    read), graph replays (outside step(), so the host's pending record is
    stale), then after_replay(the capture's final record) + flush: every
    step's late half runs exactly once -- bitwise the same steps eager."""
    _, _, data, make = _setup(p=0.1)
    rows = torch.randperm(8 * B, device=_dev(), generator=torch.Generator(device=_dev()).manual_seed(4))
    res = []
    for use_graph in (False, True):
        m, tr = make(True)
        tr.step_cycle(rows, B, 8)
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(4):
                    tr.step_cycle(rows, B, 8)
            st = tr.deferral_state()
            assert st[0] == B
            graph.replay()
            tr.flush()  # the capture's record: runs the first replay's last late half
            assert tr.deferral_state()[0] == 0
            graph.replay()
            tr.after_replay(st)
        else:
            for _ in range(8):
                tr.step_cycle(rows, B, 8)
        loss = tr.pop_loss_sum()
        res.append((_state(m, tr), loss, tr.steps_done()))
    (a, la, na), (b, lb, nb) = res
    assert na == nb == 9
    assert la == lb
    assert np.array_equal(a, b)
