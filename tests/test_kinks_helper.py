"""CPU checks of the parity helpers in tests/kinks.py (no GPU)."""
import numpy as np
import torch

from kinks import adam1_replay_error, bound_error


def _adam(p0, g, lr, state=None):
    P = torch.tensor(p0).clone()
    P.grad = torch.tensor(g)
    o = torch.optim.Adam([P], lr=lr, foreach=False)
    if state:
        o.state[P] = state
    o.step()
    st = o.state[P]
    return P.detach().numpy().copy(), st["exp_avg"].numpy().copy(), st["exp_avg_sq"].numpy().copy()


def test_adam_replay_accepts_torch_and_rejects_a_wrong_step():
    rng = np.random.default_rng(0)
    p0 = rng.standard_normal(4096).astype(np.float32)
    g = (rng.standard_normal(4096) * 1e-3).astype(np.float32)
    g[:16] = 1e-9  # components near eps: where the parameter box of adam1_bounds is loose
    lr = 4e-4
    p1, m1, v1 = _adam(p0, g, lr)
    assert adam1_replay_error(p0, g, p1, m1, v1, lr) == 0.0
    bad = p1.copy()
    bad[3] += 1e-3 * lr  # a 0.1 %-of-lr error in one near-zero-gradient component
    assert adam1_replay_error(p0, g, bad, m1, v1, lr) > 1.0
    badm = m1.copy()
    badm[7] *= 1.001
    assert adam1_replay_error(p0, g, p1, badm, v1, lr) > 1.0
    # a later step from given moments
    g2 = (rng.standard_normal(4096) * 1e-3).astype(np.float32)
    st = {"step": torch.tensor(1.0), "exp_avg": torch.tensor(m1), "exp_avg_sq": torch.tensor(v1)}
    p2, m2, v2 = _adam(p1, g2, lr, st)
    assert adam1_replay_error(p1, g2, p2, m2, v2, lr, m1, v1, 2) == 0.0
    assert adam1_replay_error(p1, g2, p2, m2, v2, lr) > 1.0  # replayed as a first step: wrong


def test_bound_error_is_normwise_distance_outside_the_box():
    lo = np.array([0.0, -1.0]); hi = np.array([1.0, 1.0]); ref = np.array([2.0, 0.0])
    assert bound_error(np.array([0.5, 0.0]), lo, hi, ref) == 0.0
    assert bound_error(np.array([1.5, 0.0]), lo, hi, ref) == 0.25
