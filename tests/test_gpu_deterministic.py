"""Deterministic-reduction mode (TT_FLAG_DETERMINISTIC).

The reference CPU loop (training.py:36-57) is bitwise repeatable under
torch.manual_seed.  By default the fused kernels add cross-block partial sums
(BatchNorm moments, BN-affine gradients, the loss / logit_scale partials,
the folded BN0 sums, embedding gradients) with float atomics in arrival
order; with the flag every block stores its partial in its own slot and a
fold kernel adds the slots in block order.  Checked here: two runs of the
same fused steps are bitwise equal (parameters, Adam moments, BN buffers,
losses) on the six-kernel path with embeddings, the paired top kernel, and
the folded cfg-3 step; the deterministic results stay at the parity bar
against the fp64 oracle; the module's autograd node is repeatable too.
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


def _cfg(latent, p):
    from ceo_firm_matching import Config
    c = Config()
    c.LATENT_DIM = latent
    c.DROPOUT_P = p
    c.DEVICE = torch.device("cuda")
    return c


def _data(meta, n, seed):
    rng = np.random.default_rng(seed)
    cat = lambda counts: (np.stack([rng.integers(0, c, n) for c in counts], 1) if counts  # noqa: E731
                          else np.zeros((n, 0), np.int64))
    return {
        "firm_numeric": torch.from_numpy((rng.standard_normal((n, meta["n_firm_numeric"])) * 2 + 0.5)
                                         .astype(np.float32)),
        "firm_cat": torch.from_numpy(cat(meta["firm_cat_counts"]).astype(np.int64)),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((n, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.from_numpy(cat(meta["ceo_cat_counts"]).astype(np.int64)),
        "target": torch.from_numpy(rng.standard_normal((n, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (n, 1)).astype(np.float32)),
    }


def _run(case, B, K, p, seed, det=True, data_seed=99):
    """K fused train steps (graph-free, host mode) from the golden init;
    returns (state_dict, exp_avg, exp_avg_sq, losses, first-step grad)."""
    from ceo_firm_matching import CEOFirmMatcher
    from ceo_firm_matching.engine import FusedTrainer
    g = load_golden(case)
    meta = meta_of(g)
    m = CEOFirmMatcher(meta, _cfg(int(g["meta/latent"]), p))
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
    m = m.to(_dev())
    tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=seed, deterministic=det)
    tr.set_data({k: v.to(_dev()) for k, v in _data(meta, K * B, data_seed).items()})
    losses, grad0 = [], None
    for k in range(K):
        tr.step(None, k * B, B)
        losses.append(tr.pop_loss_sum())
        if k == 0:
            grad0 = tr.grad.detach().cpu().numpy().copy()
    torch.cuda.synchronize()
    sd = {n: v.detach().cpu().numpy().copy() for n, v in m.state_dict().items()}
    return sd, tr.exp_avg.cpu().numpy(), tr.exp_avg_sq.cpu().numpy(), losses, grad0, m, tr


@pytest.mark.parametrize("case,B,p", [("meta_test", 300, 0.1), ("cfg2", 3000, 0.1), ("cfg2", 4096, 0.1),
                                      ("cfg3", 16384, 0.1)],
                         ids=["embeddings-6k", "unfolded-3000", "pair32-folded-4096", "folded-16384"])
def test_deterministic_steps_are_bitwise_repeatable(case, B, p):
    a = _run(case, B, 4, p, seed=21)
    b = _run(case, B, 4, p, seed=21)
    for n in a[0]:
        assert np.array_equal(a[0][n], b[0][n]), (n, np.max(np.abs(a[0][n].astype(np.float64) - b[0][n])))
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    assert a[3] == b[3]
    assert np.array_equal(a[4], b[4])


@pytest.mark.parametrize("case,B", [("meta_test", 300), ("cfg3", 16384)])
def test_deterministic_step_parity_vs_oracle(case, B):
    """One deterministic fused step (p = 0): gradient arena and loss vs the
    fp64 oracle at the parity bar (the same bar as the atomic mode), on a
    batch with no BatchNorm output within 5e-7 of the ReLU kink (there fp32
    and fp64 may take different branches: test_gpu_parity._kink_free_seed)."""
    from oracle import two_tower as O
    g = load_golden(case)
    meta = meta_of(g)
    P = {k: torch.from_numpy(v).double() for k, v in sub(g, "init").items() if k in O.param_names(meta)}
    buf = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items() if k in O.buffer_names()}
    buf = {k: (v if "num_batches" in k else v.double()) for k, v in buf.items()}
    for data_seed in range(99, 99 + 32):
        bc = _data(meta, B, data_seed)
        score, cache, _ = O.forward(P, buf, bc, train=True)
        if all(int((c[f"y{li}"].abs() < 5e-7).sum()) == 0 for c in cache["towers"] for li in (0, 1)):
            break
    else:
        raise AssertionError("no kink-free batch")
    _, _, _, losses, grad0, m, tr = _run(case, B, 1, 0.0, seed=21, data_seed=data_seed)
    loss64, dscore = O.weighted_mse(score, bc["target"], bc["weights"])
    grads = O.backward(P, cache, dscore)
    assert abs(losses[0] - float(loss64)) <= TOL * abs(float(loss64))
    base = tr.arena.params.data_ptr()
    for n, prm in m.named_parameters():
        if excluded_param(n):
            continue
        off = (prm.data_ptr() - base) // 4
        gk = grad0[off:off + prm.numel()].reshape(prm.shape)
        assert normwise(gk, grads[n].numpy()) < TOL, (n, normwise(gk, grads[n].numpy()))


def test_deterministic_module_backward_is_repeatable():
    """model.deterministic = True (or torch.use_deterministic_algorithms):
    the autograd node's forward + backward twice -> bitwise equal scores,
    parameter gradients and running statistics (embeddings included)."""
    from ceo_firm_matching import CEOFirmMatcher
    g = load_golden("meta_test")
    meta = meta_of(g)
    B = 500
    d = {k: v.to(_dev()) for k, v in _data(meta, B, 5).items()}
    outs = []
    for _ in range(2):
        torch.manual_seed(3)
        m = CEOFirmMatcher(meta, _cfg(60, 0.1)).to(_dev()).train()
        m.deterministic = True
        s = m(d["firm_numeric"], d["firm_cat"], d["ceo_numeric"], d["ceo_cat"])
        loss = (d["weights"] * (s - d["target"]) ** 2).mean()
        loss.backward()
        outs.append((s.detach().cpu().numpy(), {n: p.grad.cpu().numpy() for n, p in m.named_parameters()},
                     {n: v.cpu().numpy() for n, v in m.state_dict().items() if "running" in n}))
    (s0, g0, b0), (s1, g1, b1) = outs
    assert np.array_equal(s0, s1)
    for n in g0:
        assert np.array_equal(g0[n], g1[n]), n
    for n in b0:
        assert np.array_equal(b0[n], b1[n]), n


def test_deterministic_embedding_gradients_large_vocabulary():
    """Deterministic mode with a label-encoded vocabulary of 5,000 codes
    (k_det_scatter: each block keeps only its own codes' rows): the step's
    embedding-table gradients -- every entry, codes absent from the batch
    included -- vs the fp64 oracle at the parity bar, and bitwise repeatable
    (model.py:69,74 EmbeddingBackward)."""
    from ceo_firm_matching import CEOFirmMatcher
    from ceo_firm_matching.engine import FusedTrainer
    from oracle import two_tower as O
    meta = {"n_firm_numeric": 8, "firm_cat_counts": [5000, 7], "n_ceo_numeric": 4, "ceo_cat_counts": [300]}
    B = 1024
    torch.manual_seed(3)
    m0 = CEOFirmMatcher(meta, _cfg(32, 0.0))
    sd0 = {k: v.clone() for k, v in m0.state_dict().items()}
    P = {k: sd0[k].double() for k in O.param_names(meta)}
    buf = {k: (sd0[k] if "num_batches" in k else sd0[k].double()) for k in O.buffer_names()}
    for data_seed in range(7, 7 + 32):
        bc = _data(meta, B, data_seed)
        score, cache, _ = O.forward(P, buf, bc, train=True)
        if all(int((c[f"y{li}"].abs() < 5e-7).sum()) == 0 for c in cache["towers"] for li in (0, 1)):
            break
    else:
        raise AssertionError("no kink-free batch")
    _, dscore = O.weighted_mse(score, bc["target"], bc["weights"])
    grads = O.backward(P, cache, dscore)
    outs = []
    for _ in range(2):
        m = CEOFirmMatcher(meta, _cfg(32, 0.0))
        m.load_state_dict(sd0)
        m = m.to(_dev())
        tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=5, deterministic=True)
        tr.set_data({k: v.to(_dev()) for k, v in bc.items()})
        tr.step(None, 0, B)
        torch.cuda.synchronize()
        outs.append(tr.grad.detach().cpu().numpy().copy())
        base = tr.arena.params.data_ptr()
        for n, prm in m.named_parameters():
            if "embeddings" not in n:
                continue
            off = (prm.data_ptr() - base) // 4
            gk = outs[-1][off:off + prm.numel()].reshape(prm.shape)
            assert normwise(gk, grads[n].numpy()) < TOL, (n, normwise(gk, grads[n].numpy()))
    assert np.array_equal(outs[0], outs[1])
