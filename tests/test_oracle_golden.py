"""Pin the CPU oracle (oracle/two_tower.py) to the reference's own outputs.

The golden vectors were produced by running the reference implementation
(tests/golden/make_golden.py).  Every case the oracle will later be used as a
checker for is pinned here first.
"""
import numpy as np
import pytest
import torch

from conftest import excluded_param, load_golden, meta_of, normwise, sub
from oracle import two_tower as O

CASES = ["meta_test", "cfg2", "cfg3"]


def _params(g, prefix="init", dtype=torch.float32):
    meta = meta_of(g)
    d = sub(g, prefix)
    return {k: torch.from_numpy(d[k]).to(dtype) for k in O.param_names(meta)}


def _buffers(g, prefix="init", dtype=torch.float32):
    d = sub(g, prefix)
    out = {}
    for k in O.buffer_names():
        t = torch.from_numpy(np.asarray(d[k]))
        out[k] = t if "num_batches" in k else t.to(dtype)
    return out


def _batch(g, prefix="batch"):
    d = sub(g, prefix)
    return {k: torch.from_numpy(v) for k, v in d.items()}


@pytest.mark.parametrize("case", CASES)
def test_eval_forward(case):
    g = load_golden(case)
    P = _params(g, dtype=torch.float64)
    buf = _buffers(g, dtype=torch.float64)
    for k, v in sub(g, "eval_buffers").items():
        buf[k] = torch.from_numpy(v).double()
    score, _, _ = O.forward(P, buf, _batch(g), train=False)
    assert normwise(score.numpy(), g["eval/score"].reshape(-1)) < 1e-6


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("variant", ["train_p0", "train_mask"])
def test_train_grads(case, variant):
    g = load_golden(case)
    P = _params(g, dtype=torch.float64)
    buf = _buffers(g, dtype=torch.float64)
    batch = _batch(g)
    masks = None
    if variant == "train_mask":
        masks = {(t, l): torch.from_numpy(g[f"mask/{t}_{l}"]).double() for t in range(2) for l in range(2)}
    score, cache, newbuf = O.forward(P, buf, batch, train=True, masks=masks, p=0.1)
    loss, dscore = O.weighted_mse(score, batch["target"], batch["weights"])
    assert normwise(score.numpy(), g[f"{variant}/score"].reshape(-1)) < 2e-6
    assert abs(float(loss) - float(g[f"{variant}/loss"])) <= 2e-6 * abs(float(g[f"{variant}/loss"]))
    grads = O.backward(P, cache, dscore)
    ref = sub(g, f"{variant}/grad")
    assert set(grads) == set(ref)
    for k, v in ref.items():
        if excluded_param(k):
            continue
        assert normwise(grads[k].numpy(), v) < 1e-5, k
    if variant == "train_p0":
        # fp64 oracle vs fp64 reference: agreement to rounding
        ref64 = sub(g, "train_p0_f64/grad")
        for k, v in ref64.items():
            tol = 1e-6 if excluded_param(k) else 1e-11
            if excluded_param(k):
                assert np.max(np.abs(grads[k].numpy())) < 1e-9, k
                continue
            assert normwise(grads[k].numpy(), v) < tol, k
        for k, v in sub(g, "train_p0/buffers").items():
            assert normwise(np.asarray(newbuf[k]), v) < 1e-6, k


@pytest.mark.parametrize("case", CASES)
def test_adam_steps(case):
    g = load_golden(case)
    P = _params(g, dtype=torch.float32)
    buf = _buffers(g)
    opt = O.Adam(P, lr=4e-4)
    for k in range(5):
        b = _batch(g, f"steps/batch{k}")
        loss, _, buf = O.train_step(P, buf, opt, b, masks=None)
        assert abs(float(loss) - g["steps/losses"][k]) <= 1e-5 * abs(g["steps/losses"][k]) + 1e-6
        if k in (0, 4):
            ref = sub(g, f"steps/after{k + 1}")
            for name in O.param_names(meta_of(g)):
                if excluded_param(name):
                    continue
                assert normwise(P[name].numpy(), ref[name]) < 1e-5, (k, name)
            for name in O.buffer_names():
                if "running_mean" in name:
                    # running_mean carries the pre-BN bias (excluded above):
                    # it can drift by at most ~lr per step.
                    assert np.max(np.abs(np.asarray(buf[name]) - ref[name])) < 10 * 4e-4, (k, name)
                    continue
                assert normwise(np.asarray(buf[name]), ref[name]) < 1e-5, (k, name)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_ddp_simulation(G):
    g = load_golden("ddp")
    meta = meta_of(load_golden("cfg2"))
    d = sub(g, "init")
    P = {k: torch.from_numpy(d[k]).double() for k in O.param_names(meta)}
    buf = {k: (torch.from_numpy(np.asarray(d[k])) if "num_batches" in k else torch.from_numpy(d[k]).double())
           for k in O.buffer_names()}
    shards = [_batch(g, f"G{G}/shard{s}") for s in range(G)]
    avg = O.ddp_average_grads(P, buf, shards)
    ref = sub(g, f"G{G}/avg_grad")
    for k, v in ref.items():
        if excluded_param(k):
            continue
        assert normwise(avg[k].numpy(), v) < 1e-5, k


def test_dropout_mask_statistics():
    m = O.dropout_keep_mask(42, 7, 1, 0, 4096, 64, 0.1)
    assert abs(m.mean() - 0.9) < 0.005
    # different streams are different
    m2 = O.dropout_keep_mask(42, 8, 1, 0, 4096, 64, 0.1)
    assert (m != m2).mean() > 0.1
    assert O.dropout_keep_mask(1, 1, 0, 0, 8, 8, 0.0).all()
    # the two columns sharing one hash (32 apart in layer 0, adjacent in
    # layer 1) are independent draws: P(both kept) = 0.81
    for layer, hb in ((0, 32), (1, 1)):
        m = O.dropout_keep_mask(42, 7, 0, layer, 8192, 64, 0.1)
        c = np.arange(64)
        lo = c[(c & hb) == 0]
        both = (m[:, lo] & m[:, lo + hb]).mean()
        assert abs(both - 0.81) < 0.005, (layer, both)
        assert abs(m.mean() - 0.9) < 0.003


def test_init_consumes_rng_like_reference():
    g = load_golden("meta_test")
    meta = meta_of(g)
    torch.manual_seed(0)
    P = O.init_params_like_reference(meta, 60)
    ref = sub(g, "init")
    for k in O.param_names(meta):
        assert normwise(P[k].numpy(), ref[k]) < 1e-6, k


def _ig_case(case):
    g = load_golden("ig")
    meta = meta_of(load_golden(case))
    sd = sub(g, f"{case}/state")
    P = {k: torch.from_numpy(sd[k]).double() for k in O.param_names(meta)}
    buf = {k: (torch.from_numpy(np.asarray(sd[k])) if "num_batches" in k else torch.from_numpy(sd[k]).double())
           for k in O.buffer_names()}
    batch = {k: torch.from_numpy(v) for k, v in sub(g, f"{case}/batch").items()}
    return g, meta, P, buf, batch


def oracle_integrated_gradients(P, buf, row, n_steps):
    """The integrated-gradients path of run_deep_extensions.py:550-603 on the
    oracle: eval-mode forward + backward at each of n_steps + 1 points from a
    zero baseline to the row; mean input gradient x (input - baseline)."""
    acc = {"firm_numeric": 0, "ceo_numeric": 0}
    alphas = torch.linspace(0, 1, n_steps + 1)
    for a in alphas:
        b = dict(row)
        for k in acc:
            b[k] = (a.double() * row[k].double())
        score, cache, _ = O.forward(P, buf, b, train=False)
        grads = O.backward(P, cache, torch.ones_like(score), input_grads=True)
        for k, t in (("firm_numeric", "firm"), ("ceo_numeric", "ceo")):
            acc[k] = acc[k] + grads[f"{t}_numeric"]
    return {k: (v / (n_steps + 1) * row[k].double()).reshape(-1).numpy() for k, v in acc.items()}


@pytest.mark.parametrize("case", ["meta_test", "cfg2"])
def test_eval_backward_and_input_grads(case):
    """Eval-mode backward (running-stat BatchNorm, no dropout) with the
    numeric inputs' gradients, vs the reference's autograd (fp64)."""
    g, meta, P, buf, batch = _ig_case(case)
    score, cache, _ = O.forward(P, buf, batch, train=False)
    loss, dscore = O.weighted_mse(score, batch["target"], batch["weights"])
    grads = O.backward(P, cache, dscore, input_grads=True)
    assert normwise(score.numpy(), g[f"{case}/f64/score"].reshape(-1)) < 1e-12
    assert abs(float(loss) - float(g[f"{case}/f64/loss"])) < 1e-12
    ref = sub(g, f"{case}/f64/grad")
    for n in O.param_names(meta):
        assert normwise(grads[n].numpy(), ref[n]) < 1e-10, n
    assert normwise(grads["firm_numeric"].numpy(), g[f"{case}/f64/dx_firm"]) < 1e-10
    assert normwise(grads["ceo_numeric"].numpy(), g[f"{case}/f64/dx_ceo"]) < 1e-10


@pytest.mark.parametrize("case", ["meta_test", "cfg2"])
def test_integrated_gradients_vs_reference(case):
    g, meta, P, buf, batch = _ig_case(case)
    row = {k: v[:1] for k, v in batch.items()}
    ig = oracle_integrated_gradients(P, buf, row, 8)
    assert normwise(ig["firm_numeric"], g[f"{case}/f64/ig_firm"]) < 1e-10
    assert normwise(ig["ceo_numeric"], g[f"{case}/f64/ig_ceo"]) < 1e-10
