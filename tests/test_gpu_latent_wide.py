"""LATENT_DIM above 128: the generic top of the towers (tt_topgen.hip).

The reference accepts any config.LATENT_DIM (model.py:46,61); the fused
k_top / k_top_pair hold W8 images and U / V rows in LDS up to 128, so wider
latent spaces (the contrastive configurations' 256 / 512) run U / V, the
cosine / loss closed form and the top backward as three kernels over the
workspace.  Checked against the fp64 oracle at 1e-5: train
forward + backward (embeddings, ragged B), eval forward, fused Adam steps,
the tower-embedding node (contrastive.py:52-72) in train and eval mode,
and bitwise repeatability in deterministic mode.
"""
import numpy as np
import pytest
import torch

from conftest import excluded_param, normwise

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _cfg(latent, p):
    from ceo_firm_matching import Config
    c = Config()
    c.LATENT_DIM = latent
    c.DROPOUT_P = p
    c.DEVICE = torch.device("cuda")
    return c


def _batch(meta, B, seed):
    rng = np.random.default_rng(seed)
    cat = lambda counts: (np.stack([rng.integers(0, n, B) for n in counts], 1) if counts  # noqa: E731
                          else np.zeros((B, 0), np.int64))
    return {
        "firm_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.from_numpy(cat(meta["firm_cat_counts"]).astype(np.int64)),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.from_numpy(cat(meta["ceo_cat_counts"]).astype(np.int64)),
        "target": torch.from_numpy(rng.standard_normal((B, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (B, 1)).astype(np.float32)),
    }


def _oracle_state(O, meta, sd0):
    P = {k: sd0[k].double() for k in O.param_names(meta)}
    buf = {k: (sd0[k] if "num_batches" in k else sd0[k].double()) for k in O.buffer_names()}
    return P, buf


WIDE = [
    # (firm n_num, firm cats, ceo n_num, ceo cats, latent, B)
    (64, [], 64, [], 256, 300),
    (12, [4, 4, 2, 2], 2, [2, 4, 2, 2, 2, 2, 2], 512, 97),
    (32, [], 32, [], 200, 4100),
]


@pytest.mark.parametrize("geo", WIDE, ids=[f"D{g[4]}-B{g[5]}" for g in WIDE])
def test_wide_latent_train_and_eval_vs_oracle(geo):
    from ceo_firm_matching import CEOFirmMatcher
    from ceo_firm_matching import _native as N
    from oracle import two_tower as O
    nf, fc, nc, cc, latent, B = geo
    meta = {"n_firm_numeric": nf, "firm_cat_counts": fc, "n_ceo_numeric": nc, "ceo_cat_counts": cc}
    torch.manual_seed(latent + B)
    m = CEOFirmMatcher(meta, _cfg(latent, 0.0))
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(_dev()).train()
    assert not N.step_plan(m.tt_desc(), B)["top_pair"]
    bc = _batch(meta, B, B + latent)
    b = {k: v.to(_dev()) for k, v in bc.items()}
    s = m(b["firm_numeric"], b["firm_cat"], b["ceo_numeric"], b["ceo_cat"])
    loss = (b["weights"] * (s - b["target"]) ** 2).mean()
    loss.backward()
    P, buf = _oracle_state(O, meta, sd0)
    score, cache, nbuf = O.forward(P, buf, bc, train=True)
    l64, dscore = O.weighted_mse(score, bc["target"], bc["weights"])
    grads = O.backward(P, cache, dscore)
    assert normwise(s.detach().cpu().numpy().reshape(-1), score.numpy()) < TOL
    assert abs(loss.item() - float(l64)) <= TOL * float(l64)
    for n, p in m.named_parameters():
        if excluded_param(n):
            continue
        assert normwise(p.grad.cpu().numpy(), grads[n].numpy()) < TOL, (n, normwise(p.grad.cpu().numpy(),
                                                                                  grads[n].numpy()))
    sd = m.state_dict()
    for k in O.buffer_names():
        if "running" in k:
            assert normwise(sd[k].cpu().numpy(), nbuf[k].numpy()) < TOL, k
    m.eval()
    with torch.no_grad():
        se = m(b["firm_numeric"], b["firm_cat"], b["ceo_numeric"], b["ceo_cat"])
    bufe = {k: (v.detach().cpu() if "num_batches" in k else v.detach().cpu().double())
            for k, v in m.state_dict().items() if k in O.buffer_names()}
    se_ref, _, _ = O.forward(P, bufe, bc, train=False)
    assert normwise(se.cpu().numpy().reshape(-1), se_ref.numpy()) < TOL


@pytest.mark.parametrize("det", [False, True], ids=["atomics", "deterministic"])
def test_wide_latent_fused_adam_steps(det):
    """Three fused train steps (tt_train_step: the generic top inside the
    step) at LATENT 256, B 2048, vs the oracle's fp64 steps and torch Adam;
    deterministic mode: two runs bitwise equal."""
    from ceo_firm_matching import CEOFirmMatcher
    from ceo_firm_matching.engine import FusedTrainer
    from oracle import two_tower as O
    meta = {"n_firm_numeric": 48, "firm_cat_counts": [], "n_ceo_numeric": 40, "ceo_cat_counts": []}
    B, K = 2048, 3
    data = _batch(meta, K * B, 7)
    runs = []
    for rep in range(2 if det else 1):
        torch.manual_seed(17)
        m = CEOFirmMatcher(meta, _cfg(256, 0.0))
        sd0 = {k: v.clone() for k, v in m.state_dict().items()}
        m = m.to(_dev())
        tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=3, deterministic=det)
        tr.set_data({k: v.to(_dev()) for k, v in data.items()})
        losses = []
        for k in range(K):
            tr.step(None, k * B, B)
            losses.append(tr.pop_loss_sum())
        runs.append((losses, {n: v.cpu().numpy().copy() for n, v in m.state_dict().items()}))
    P, buf = _oracle_state(O, meta, sd0)
    opt = O.Adam(P, lr=4e-4)
    for k in range(K):
        bk = {n: v[k * B:(k + 1) * B] for n, v in data.items()}
        l64, _, buf = O.train_step(P, buf, opt, bk, p=0.0)
        assert abs(runs[0][0][k] - float(l64)) <= TOL * abs(float(l64)), k
    for n, v in P.items():
        if excluded_param(n):
            continue
        got = runs[0][1][n].astype(np.float64)
        assert normwise(got, v.numpy()) < 1e-4 or np.max(np.abs(got - v.numpy())) <= 5e-2 * 4e-4, n
    if det:
        assert runs[0][0] == runs[1][0]
        for n in runs[0][1]:
            assert np.array_equal(runs[0][1][n], runs[1][1][n]), n


@pytest.mark.parametrize("train", [True, False], ids=["train", "eval"])
def test_wide_latent_tower_embeddings(train):
    """tower_embeddings (the encoder half contrastive.py:52-72 builds on) at
    LATENT 512: U, V and the gradients of sum(U R1) + sum(V R2) w.r.t. every
    parameter and the numeric inputs, vs the oracle (p = 0)."""
    from ceo_firm_matching import CEOFirmMatcher
    from oracle import two_tower as O
    meta = {"n_firm_numeric": 12, "firm_cat_counts": [4, 4, 2, 2], "n_ceo_numeric": 2,
            "ceo_cat_counts": [2, 4, 2, 2, 2, 2, 2]}
    B = 200
    torch.manual_seed(4)
    m = CEOFirmMatcher(meta, _cfg(512, 0.0))
    with torch.no_grad():
        for t in (m.firm_tower, m.ceo_tower):
            for i in (1, 5):
                t[i].running_mean.uniform_(-0.3, 0.3)
                t[i].running_var.uniform_(0.5, 2.0)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(_dev()).train(train)
    bc = _batch(meta, B, 9)
    b = {k: v.to(_dev()) for k, v in bc.items()}
    f_num = b["firm_numeric"].clone().requires_grad_(True)
    c_num = b["ceo_numeric"].clone().requires_grad_(True)
    u, v = m.tower_embeddings(f_num, b["firm_cat"], c_num, b["ceo_cat"])
    gen = torch.Generator(device=_dev()).manual_seed(5)
    r1 = torch.randn(u.shape, device=_dev(), generator=gen)
    r2 = torch.randn(v.shape, device=_dev(), generator=gen)
    ((u * r1).sum() + (v * r2).sum()).backward()
    P, buf = _oracle_state(O, meta, sd0)
    _, cache, _ = O.forward(P, buf, bc, train=train)
    U, V = cache["towers"][0]["u"], cache["towers"][1]["u"]
    assert normwise(u.detach().cpu().numpy(), U.numpy()) < TOL
    assert normwise(v.detach().cpu().numpy(), V.numpy()) < TOL
    import copy
    c = copy.copy(cache)
    c.update(s=torch.tensor(1.0, dtype=torch.float64), cos=torch.zeros(B, dtype=torch.float64),
             score=torch.zeros(B, dtype=torch.float64), un=r2.double().cpu(), vn=r1.double().cpu(),
             nu=torch.ones(B, 1, dtype=torch.float64), nv=torch.ones(B, 1, dtype=torch.float64))
    ref = O.backward(P, c, torch.ones(B, dtype=torch.float64), input_grads=True)
    for n, p in m.named_parameters():
        if n == "logit_scale" or (train and excluded_param(n)):
            continue
        assert normwise(p.grad.cpu().numpy(), ref[n].numpy()) < TOL, n
    assert normwise(f_num.grad.cpu().numpy(), ref["firm_numeric"].numpy()) < TOL
    assert normwise(c_num.grad.cpu().numpy(), ref["ceo_numeric"].numpy()) < TOL
