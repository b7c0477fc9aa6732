"""Eval-mode backward and input gradients through the fused autograd node.

The reference forward is plain autograd (model.py:67-89), so a caller may
run it in eval mode and differentiate it w.r.t. the numeric inputs:
run_deep_extensions.py:550-603 (integrated gradients) calls model.eval(),
requires_grad_ on f_num / c_num, score.backward() and reads f_num.grad.
Here that goes through tt_backward_ex (C-ABI) on the HIP kernels: eval-mode
BatchNorm as the affine map of the running statistics, dX = dZ0 W0 stored for
the numeric columns.  Pinned to tests/golden/ig.npz (made by importing the
reference: its own integrated_gradients and an eval-mode weighted-MSE
backward) and to the fp64 oracle; tolerance 1e-5 normwise.
"""
import numpy as np
import pytest
import torch

from conftest import excluded_param, load_golden, meta_of, normwise, sub

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _cfg(latent, p=0.1):
    from ceo_firm_matching import Config
    c = Config()
    c.LATENT_DIM = latent
    c.DROPOUT_P = p
    c.DEVICE = torch.device("cuda")
    return c


def _ig_model(case):
    from ceo_firm_matching import CEOFirmMatcher
    g = load_golden("ig")
    meta = meta_of(load_golden(case))
    m = CEOFirmMatcher(meta, _cfg(int(g[f"{case}/latent"])))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, f"{case}/state").items()})
    batch = {k: torch.from_numpy(v).to(_dev()) for k, v in sub(g, f"{case}/batch").items()}
    return g, m.to(_dev()), batch


@pytest.mark.parametrize("case", ["meta_test", "cfg2"])
def test_eval_backward_param_and_input_grads(case):
    """model.eval(); loss = weighted MSE; loss.backward(): every parameter's
    gradient (the pre-BN Linear biases too: in eval mode BatchNorm does not
    cancel them) and dL/d f_numeric, dL/d c_numeric vs the reference fp64."""
    g, m, b = _ig_model(case)
    m.eval()
    f_num = b["firm_numeric"].clone().requires_grad_(True)
    c_num = b["ceo_numeric"].clone().requires_grad_(True)
    s = m(f_num, b["firm_cat"], c_num, b["ceo_cat"])
    loss = (b["weights"] * (s - b["target"]) ** 2).mean()
    loss.backward()
    assert normwise(s.detach().cpu().numpy(), g[f"{case}/f64/score"]) < TOL
    ref = sub(g, f"{case}/f64/grad")
    for n, p in m.named_parameters():
        assert p.grad is not None, n
        assert normwise(p.grad.cpu().numpy(), ref[n]) < TOL, (n, normwise(p.grad.cpu().numpy(), ref[n]))
    assert normwise(f_num.grad.cpu().numpy(), g[f"{case}/f64/dx_firm"]) < TOL
    assert normwise(c_num.grad.cpu().numpy(), g[f"{case}/f64/dx_ceo"]) < TOL
    # running statistics untouched by an eval forward + backward
    for k, v in sub(g, f"{case}/state").items():
        if "running" in k:
            assert np.array_equal(m.state_dict()[k].cpu().numpy(), v), k


@pytest.mark.parametrize("case", ["meta_test", "cfg2"])
def test_integrated_gradients_loop_on_fused_model(case):
    """The integrated-gradients loop of run_deep_extensions.py:564-590 (batch-1
    eval forwards, requires_grad_ inputs, score.backward(), f_num.grad) on
    the fused model, and the batched form (attribution.integrated_gradients:
    the whole path as one eval forward + backward), vs the reference's own
    integrated_gradients in fp64 (n_steps = 8, zero baseline)."""
    from ceo_firm_matching.attribution import integrated_gradients
    g, m, b = _ig_model(case)
    inputs = {k: b[k][:1] for k in ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat")}
    base = {k: torch.zeros_like(inputs[k]) for k in ("firm_numeric", "ceo_numeric")}
    m.eval()
    n_steps = 8
    alphas = torch.linspace(0, 1, n_steps + 1, device=_dev())
    gf, gc = [], []
    for a in alphas:
        f = (base["firm_numeric"] + a * (inputs["firm_numeric"] - base["firm_numeric"])).clone().requires_grad_(True)
        c = (base["ceo_numeric"] + a * (inputs["ceo_numeric"] - base["ceo_numeric"])).clone().requires_grad_(True)
        score = m(f, inputs["firm_cat"], c, inputs["ceo_cat"])
        m.zero_grad()
        score.backward()
        gf.append(f.grad.detach().clone())
        gc.append(c.grad.detach().clone())
    ig_f = (torch.stack(gf).mean(0) * (inputs["firm_numeric"] - base["firm_numeric"])).reshape(-1).cpu().numpy()
    ig_c = (torch.stack(gc).mean(0) * (inputs["ceo_numeric"] - base["ceo_numeric"])).reshape(-1).cpu().numpy()
    assert normwise(ig_f, g[f"{case}/f64/ig_firm"]) < TOL
    assert normwise(ig_c, g[f"{case}/f64/ig_ceo"]) < TOL
    ig = integrated_gradients(m, inputs, base, n_steps=n_steps)
    assert normwise(ig["firm_numeric"], g[f"{case}/f64/ig_firm"]) < TOL
    assert normwise(ig["ceo_numeric"], g[f"{case}/f64/ig_ceo"]) < TOL


@pytest.mark.parametrize("case,B", [("meta_test", 96), ("cfg3", 512), ("cfg3", 8192)])
def test_train_mode_input_grads_vs_oracle(case, B):
    """Train-mode (batch statistics) backward with input gradients: the
    folded BN0 backward never forms dZ0 per row, so a step that needs dX runs
    the unfolded kernels (k_bwd_mid + k_bwd_first) at any B; dX and every
    parameter gradient vs the fp64 oracle (p = 0)."""
    from ceo_firm_matching import CEOFirmMatcher
    from oracle import two_tower as O
    g = load_golden(case)
    meta = meta_of(g)
    rng = np.random.default_rng(B + 3)
    cats = lambda counts: (np.stack([rng.integers(0, n, B) for n in counts], 1) if counts  # noqa: E731
                           else np.zeros((B, 0), np.int64))
    bc = {
        "firm_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.from_numpy(cats(meta["firm_cat_counts"])),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.from_numpy(cats(meta["ceo_cat_counts"])),
        "target": torch.from_numpy(rng.standard_normal((B, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (B, 1)).astype(np.float32)),
    }
    m = CEOFirmMatcher(meta, _cfg(int(g["meta/latent"]), 0.0))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
    m = m.to(_dev()).train()
    b = {k: v.to(_dev()) for k, v in bc.items()}
    f_num = b["firm_numeric"].clone().requires_grad_(True)
    c_num = b["ceo_numeric"].clone().requires_grad_(True)
    s = m(f_num, b["firm_cat"], c_num, b["ceo_cat"])
    loss = (b["weights"] * (s - b["target"]) ** 2).mean()
    loss.backward()
    P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
    buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
    buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
    score, cache, _ = O.forward(P, buf, bc, train=True)
    _, dscore = O.weighted_mse(score, bc["target"], bc["weights"])
    grads = O.backward(P, cache, dscore, input_grads=True)
    assert normwise(s.detach().cpu().numpy().reshape(-1), score.numpy()) < TOL
    for n, p in m.named_parameters():
        if excluded_param(n):
            continue
        assert normwise(p.grad.cpu().numpy(), grads[n].numpy()) < TOL, n
    assert normwise(f_num.grad.cpu().numpy(), grads["firm_numeric"].numpy()) < TOL
    assert normwise(c_num.grad.cpu().numpy(), grads["ceo_numeric"].numpy()) < TOL


def test_eval_backward_batch_of_one_and_tower_embeddings():
    """Eval mode allows B = 1 (BatchNorm uses running statistics), and the
    tower-embedding node (contrastive.py:52-72 get_embeddings) has the same
    eval / input-gradient backward: vs the fp64 oracle."""
    from oracle import two_tower as O
    g, m, b = _ig_model("meta_test")
    meta = meta_of(load_golden("meta_test"))
    sd = sub(g, "meta_test/state")
    P = {k: torch.from_numpy(sd[k]).double() for k in O.param_names(meta)}
    buf = {k: (torch.from_numpy(np.asarray(sd[k])) if "num_batches" in k else torch.from_numpy(sd[k]).double())
           for k in O.buffer_names()}
    m.eval()
    one = {k: v[:1] for k, v in b.items()}
    f_num = one["firm_numeric"].clone().requires_grad_(True)
    c_num = one["ceo_numeric"].clone().requires_grad_(True)
    s = m(f_num, one["firm_cat"], c_num, one["ceo_cat"])
    s.sum().backward()
    bc = {k: v.cpu() for k, v in one.items()}
    score, cache, _ = O.forward(P, buf, bc, train=False)
    grads = O.backward(P, cache, torch.ones_like(score), input_grads=True)
    assert normwise(s.detach().cpu().numpy().reshape(-1), score.numpy()) < TOL
    for n, p in m.named_parameters():
        assert normwise(p.grad.cpu().numpy(), grads[n].numpy()) < TOL, n
    assert normwise(f_num.grad.cpu().numpy(), grads["firm_numeric"].numpy()) < TOL
    assert normwise(c_num.grad.cpu().numpy(), grads["ceo_numeric"].numpy()) < TOL
    # tower embeddings: d(sum U * R1 + sum V * R2) in eval mode, B = 32
    m.zero_grad()
    f_num = b["firm_numeric"].clone().requires_grad_(True)
    c_num = b["ceo_numeric"].clone().requires_grad_(True)
    u, v = m.tower_embeddings(f_num, b["firm_cat"], c_num, b["ceo_cat"])
    gen = torch.Generator(device=_dev()).manual_seed(3)
    r1 = torch.randn(u.shape, device=_dev(), generator=gen)
    r2 = torch.randn(v.shape, device=_dev(), generator=gen)
    ((u * r1).sum() + (v * r2).sum()).backward()
    bc = {k: x.cpu() for k, x in b.items()}
    _, cache, _ = O.forward(P, buf, bc, train=False)
    # the oracle's backward from dU / dV: inject them through the cosine-free
    # path by differentiating the tower outputs directly
    ref = _oracle_tower_backward(O, P, cache, r1.double().cpu(), r2.double().cpu())
    for n, p in m.named_parameters():
        if n == "logit_scale":
            continue
        assert normwise(p.grad.cpu().numpy(), ref[n].numpy()) < TOL, n
    assert normwise(f_num.grad.cpu().numpy(), ref["firm_numeric"].numpy()) < TOL
    assert normwise(c_num.grad.cpu().numpy(), ref["ceo_numeric"].numpy()) < TOL


def _oracle_tower_backward(O, P, cache, du, dv):
    """Gradients of sum(U * du) + sum(V * dv) through the oracle's towers
    (eval-mode cache), by driving O.backward with a cosine cache whose
    closed-form dU / dV equal du / dv."""
    import copy
    c = copy.copy(cache)
    # O.backward forms du = dc (vn - un cos) / nu: choose nu = 1, cos = 0,
    # vn = du, un = dv, dc = 1 -> du_out = du, dv_out = dv
    B = du.shape[0]
    c.update(s=torch.tensor(1.0, dtype=torch.float64), cos=torch.zeros(B, dtype=torch.float64),
             score=torch.zeros(B, dtype=torch.float64), un=dv, vn=du,
             nu=torch.ones(B, 1, dtype=torch.float64), nv=torch.ones(B, 1, dtype=torch.float64))
    return O.backward(P, c, torch.ones(B, dtype=torch.float64), input_grads=True)
