"""ReLU-kink and zero-variance BatchNorm semantics of the fused path against
the reference (model.py:39-41,54-56 -- BatchNorm1d, ReLU, Dropout -- and
autograd's backward of them), WITHOUT screening or nudging the inputs.

* exact kinks: a Linear row of zeros with BN beta = 0 makes a whole BN
  column constant -- batch variance 0, invstd = 1/sqrt(eps), Zhat = 0 and
  y = 0 exactly -- so ReLU sits exactly on its kink for every row and
  ATen's threshold_backward gives that column zero gradient; the running
  variance decays to 0.9 * rv.  Both BN layers, both towers, the six-kernel
  path (B = 3000), the folded step on 32-row k_top_pair blocks (B = 4096)
  and the folded cfg-3 step (B = 16384), dropout off and on,
  atomic and deterministic reductions: the fused step's gradient arena and
  the parameters after Adam at 1e-5 of the fp64 oracle;
* unscreened data at B = 16384 (the bench batch): elements whose pre-ReLU
  value lies within rounding of the kink may take either branch in fp32, so
  the gradient is held to the oracle's bound over every branch choice
  (tests/kinks.py) -- exactly the 1e-5 normwise bar for every entry no kink
  reaches.
"""
import numpy as np
import pytest
import torch

from conftest import excluded_param, load_golden, meta_of, normwise, sub
from kinks import adam1_bounds, adam1_replay_error, bound_error, grad_bounds, kink_elements

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _oracle_state(O, g, meta, edit=None):
    P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
    buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
    buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
    if edit:
        edit(P)
    return P, buf


def _draw(meta, B, seed):
    rng = np.random.default_rng(seed)
    return {
        "firm_numeric": torch.from_numpy((rng.standard_normal((B, meta["n_firm_numeric"])) * 2 + 0.5)
                                         .astype(np.float32)),
        "firm_cat": torch.zeros(B, 0, dtype=torch.int64),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.zeros(B, 0, dtype=torch.int64),
        "target": torch.from_numpy(rng.standard_normal((B, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (B, 1)).astype(np.float32)),
    }


def _fused_step(g, meta, P, data, B, p, seed, det):
    """One fused train step (FusedTrainer) from the oracle parameters P;
    returns (model, trainer)."""
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching.engine import FusedTrainer
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = p
    cfg.DEVICE = _dev()
    m = CEOFirmMatcher(meta, cfg)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()}
    sd.update({k: v.float() for k, v in P.items()})
    m.load_state_dict(sd)
    m = m.to(_dev())
    tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=seed, deterministic=det)
    tr.set_data({k: v.to(_dev()) for k, v in data.items()})
    tr.step(None, 0, B)
    torch.cuda.synchronize()
    return m, tr


def _grad_of(m, tr, name):
    base = tr.arena.params.data_ptr()
    prm = dict(m.named_parameters())[name]
    off = (prm.data_ptr() - base) // 4
    return tr.grad[off:off + prm.numel()].view(prm.shape).cpu().double().numpy()


def _state_of(tr, m, name, which):
    """the fused trainer's fp32 exp_avg / exp_avg_sq slice of one parameter"""
    base = tr.arena.params.data_ptr()
    prm = dict(m.named_parameters())[name]
    off = (prm.data_ptr() - base) // 4
    return getattr(tr, which)[off:off + prm.numel()].cpu().numpy()


def _check_adam_replay(m, tr, P):
    """every parameter: the fused Adam step equals torch's Adam applied to
    the fused gradient (kinks.adam1_replay_error)"""
    sd = m.state_dict()
    for n in P:
        err = adam1_replay_error(P[n].float().numpy(), _grad_of(m, tr, n), sd[n].cpu().numpy(),
                                 _state_of(tr, m, n, "exp_avg"), _state_of(tr, m, n, "exp_avg_sq"), 4e-4)
        assert err < 1.0, ("adam replay", n, err, P[n].float().numpy().reshape(-1)[:2], _grad_of(m, tr, n).reshape(-1)[:2],
                           sd[n].cpu().numpy().reshape(-1)[:2], _state_of(tr, m, n, "exp_avg")[:2],
                           _state_of(tr, m, n, "exp_avg_sq")[:2])


def _zero_columns(P):
    """firm tower: W0 row 5 and BN0 beta[5]; ceo tower: W4 row 7 and BN1
    beta[7] and W0 row 40 and BN0 beta[40] (both layers, both towers)."""
    P["firm_tower.0.weight"][5] = 0
    P["firm_tower.1.bias"][5] = 0
    P["ceo_tower.4.weight"][7] = 0
    P["ceo_tower.5.bias"][7] = 0
    P["ceo_tower.0.weight"][40] = 0
    P["ceo_tower.1.bias"][40] = 0


@pytest.mark.parametrize("det", [False, True], ids=["atomics", "deterministic"])
@pytest.mark.parametrize("B,p", [(3000, 0.0), (3000, 0.1), (4096, 0.0), (4096, 0.1), (16384, 0.0), (16384, 0.1)])
def test_exact_kink_zero_variance_columns(B, p, det):
    from ceo_firm_matching import _native as N
    from oracle import two_tower as O
    g = load_golden("cfg3")
    meta = meta_of(g)
    P, buf = _oracle_state(O, g, meta, _zero_columns)
    data = _draw(meta, B, 300 + B)
    seed = 41
    m, tr = _fused_step(g, meta, P, data, B, p, seed, det)
    assert N.step_plan(m.tt_desc(), B)["folded_bn0_backward"] == (B >= 4096)
    masks = None
    if p > 0:
        masks = {(t, l): torch.from_numpy(O.dropout_keep_mask(seed, 1, t, l, B, H, p)).double()
                 for t in range(2) for l, H in enumerate((64, 32))}
    score, cache, nbuf = O.forward(P, buf, data, train=True, masks=masks, p=p)
    # the oracle's own view of the constructed columns: y == 0 exactly
    for ti, li, col in ((0, 0, 5), (1, 1, 7), (1, 0, 40)):
        assert bool((cache["towers"][ti][f"y{li}"][:, col] == 0).all()), (ti, li, col)
    _, dscore = O.weighted_mse(score, data["target"], data["weights"])
    grads = O.backward(P, cache, dscore)
    # zero gradient through y == 0 (threshold_backward), in the reference's terms
    assert float(grads["firm_tower.1.weight"][5]) == 0.0 and float(grads["firm_tower.1.bias"][5]) == 0.0
    assert float(grads["ceo_tower.5.weight"][7]) == 0.0 and float(grads["ceo_tower.5.bias"][7]) == 0.0
    assert bool((grads["firm_tower.0.weight"][5] == 0).all())
    elems = [e for e in kink_elements(cache, masks) if not (e[:2], e[3]) in (((0, 0), 5), ((1, 1), 7), ((1, 0), 40))]
    lo, hi = grad_bounds(O, P, cache, dscore, elems)
    for n, prm in m.named_parameters():
        if excluded_param(n):
            continue
        got = _grad_of(m, tr, n)
        err = bound_error(got, lo[n].numpy(), hi[n].numpy(), grads[n].numpy())
        assert err < TOL, ("grad", n, err)
    # the constructed columns' gradients are exactly zero in the fused step too
    assert not _grad_of(m, tr, "firm_tower.1.weight")[5] and not _grad_of(m, tr, "firm_tower.1.bias")[5]
    assert not _grad_of(m, tr, "ceo_tower.5.weight")[7] and not _grad_of(m, tr, "ceo_tower.5.bias")[7]
    assert not np.any(_grad_of(m, tr, "firm_tower.0.weight")[5])
    assert not np.any(_grad_of(m, tr, "ceo_tower.4.weight")[7])
    # parameters after Adam, BN buffers (running_var of a constant column: 0.9 * rv + 0.1 * 0)
    plo, phi = adam1_bounds(O, P, lo, hi, 4e-4, ref=grads, slack=TOL)
    sd = m.state_dict()
    for n in P:
        if excluded_param(n):
            continue
        err = bound_error(sd[n].cpu().double().numpy(), plo[n].numpy(), phi[n].numpy(), plo[n].numpy())
        assert err < TOL, ("param", n, err)
    for k, v in nbuf.items():
        if "num_batches" in k:
            assert int(sd[k]) == int(v), k
        elif "running_mean" not in k:
            assert normwise(sd[k].cpu().numpy(), v.numpy()) < TOL, k
    assert float(sd["firm_tower.1.running_var"][5]) == pytest.approx(0.9, abs=1e-7)
    assert float(sd["ceo_tower.5.running_var"][7]) == pytest.approx(0.9, abs=1e-7)
    _check_adam_replay(m, tr, P)


@pytest.mark.parametrize("det", [False, True], ids=["atomics", "deterministic"])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_unscreened_large_batch_vs_kink_bounds(p, det):
    """B = 16384 cfg-3 step on unscreened draws (no kink-free seed search, no
    nudged rows): gradient arena and parameters after Adam inside the fp64
    oracle's bound over every ReLU branch choice at kink elements."""
    from oracle import two_tower as O
    g = load_golden("cfg3")
    meta = meta_of(g)
    B = 16384
    P, buf = _oracle_state(O, g, meta)
    data = _draw(meta, B, 77)  # the seed whose row 1652 sits at y = -3.5e-7
    seed = 1000
    m, tr = _fused_step(g, meta, P, data, B, p, seed, det)
    masks = None
    if p > 0:
        masks = {(t, l): torch.from_numpy(O.dropout_keep_mask(seed, 1, t, l, B, H, p)).double()
                 for t in range(2) for l, H in enumerate((64, 32))}
    score, cache, _ = O.forward(P, buf, data, train=True, masks=masks, p=p)
    _, dscore = O.weighted_mse(score, data["target"], data["weights"])
    grads = O.backward(P, cache, dscore)
    elems = kink_elements(cache, masks)
    lo, hi = grad_bounds(O, P, cache, dscore, elems)
    worst = {}
    for n, _ in m.named_parameters():
        if excluded_param(n):
            continue
        worst[n] = bound_error(_grad_of(m, tr, n), lo[n].numpy(), hi[n].numpy(), grads[n].numpy())
    bad = {k: v for k, v in worst.items() if v >= TOL}
    assert not bad, (len(elems), bad)
    plo, phi = adam1_bounds(O, P, lo, hi, 4e-4, ref=grads, slack=TOL)
    sd = m.state_dict()
    for n in P:
        if excluded_param(n):
            continue
        err = bound_error(sd[n].cpu().double().numpy(), plo[n].numpy(), phi[n].numpy(), plo[n].numpy())
        assert err < TOL, ("param", n, err, len(elems))
    _check_adam_replay(m, tr, P)


@pytest.mark.parametrize("det", [False, True], ids=["atomics", "deterministic"])
def test_every_step_gradient_at_the_fused_parameters(det):
    """Beyond step 1 the parameter comparisons loosen (Adam turns the fp32
    noise of ~0 gradient components into +-lr steps), so every step of a
    4-step cfg-3 run (B = 16384, dropout 0.1, unscreened data) is held to the
    1e-5 bar on its own: the fused step's gradient against the fp64 oracle's
    gradient AT THE FUSED PARAMETERS of that step (the oracle re-synced to the
    kernels' trajectory each step), inside the kink bounds; and the step's
    parameters and moments against torch's Adam applied to that gradient
    from the step's starting state (kinks.adam1_replay_error)."""
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching.engine import FusedTrainer
    from oracle import two_tower as O
    g = load_golden("cfg3")
    meta = meta_of(g)
    B, K, p, seed = 16384, 4, 0.1, 2222
    data = _draw(meta, K * B, 909)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = p
    cfg.DEVICE = _dev()
    m = CEOFirmMatcher(meta, cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
    m = m.to(_dev())
    tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=seed, deterministic=det)
    tr.set_data({k: v.to(_dev()) for k, v in data.items()})
    _, buf = _oracle_state(O, g, meta)
    names = [n for n, _ in m.named_parameters()]
    for k in range(K):
        P = {n: prm.detach().cpu().double().clone() for n, prm in m.named_parameters()}
        M0 = {n: _state_of(tr, m, n, "exp_avg") for n in P}
        V0 = {n: _state_of(tr, m, n, "exp_avg_sq") for n in P}
        tr.step(None, k * B, B)
        torch.cuda.synchronize()
        sd = m.state_dict()
        for n in names:  # the optimizer arithmetic of step k + 1 on the fused gradient
            err, info = adam1_replay_error(P[n].float().numpy(), _grad_of(m, tr, n), sd[n].cpu().numpy(),
                                           _state_of(tr, m, n, "exp_avg"), _state_of(tr, m, n, "exp_avg_sq"), 4e-4,
                                           M0[n], V0[n], k + 1, detail=True)
            assert err < 1.0, ("adam replay", k, n, err, info)
        bk = {n: v[k * B:(k + 1) * B] for n, v in data.items()}
        masks = {(t, l): torch.from_numpy(O.dropout_keep_mask(seed, k + 1, t, l, B, H, p)).double()
                 for t in range(2) for l, H in enumerate((64, 32))}
        score, cache, _ = O.forward(P, buf, bk, train=True, masks=masks, p=p)
        _, dscore = O.weighted_mse(score, bk["target"], bk["weights"])
        grads = O.backward(P, cache, dscore)
        lo, hi = grad_bounds(O, P, cache, dscore, kink_elements(cache, masks))
        for n in names:
            if excluded_param(n):
                continue
            err = bound_error(_grad_of(m, tr, n), lo[n].numpy(), hi[n].numpy(), grads[n].numpy())
            assert err < TOL, (k, n, err)
    assert tr.steps_done() == K
