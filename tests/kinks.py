"""Parity at ReLU kinks without editing the inputs (test helper).

A BatchNorm output y within rounding (~1e-7 .. 1e-6) of 0 may land on either
side of the ReLU kink in an fp32 step -- which side can even change with the
float-atomic order of the BN moment sums -- while the fp64 oracle decides it
once.  Both branches are the reference's arithmetic at a rounding-level
perturbation of its inputs, so instead of screening such inputs out, the
oracle's gradient is bounded over every branch choice:

* ``kink_elements``: the (tower, layer, row, column) elements whose pre-ReLU
  value lies within ``thr`` of 0 (and that dropout keeps);
* the backward is linear in ReLU's pass mask (given the forward), so with the
  kink elements all blocked (g_off) and each one opened alone (g_off + d_e),
  any mix of branches gives g_off + sum_{e in S} d_e, which lies inside
  [g_off + sum min(d_e, 0), g_off + sum max(d_e, 0)] (``grad_bounds``);
* ``bound_error``: how far a gradient lies outside that box, normwise
  (divided by max |g_ref|), compared with the usual 1e-5 bar.

Entries no kink reaches have lo == hi == the fp64 gradient, so for them this
is exactly the plain normwise check.  A one-step Adam update is monotone in
the gradient, so parameter bounds are Adam applied to lo and to hi.
"""
from typing import Dict, List, Tuple

import numpy as np
import torch


def kink_elements(cache, masks=None, thr: float = 2e-6) -> List[Tuple[int, int, int, int]]:
    out = []
    for ti, c in enumerate(cache["towers"]):
        for li in (0, 1):
            near = c[f"y{li}"].abs() < thr
            if masks is not None and (ti, li) in masks:
                near &= masks[(ti, li)] > 0
            for r, col in torch.nonzero(near).tolist():
                out.append((ti, li, r, col))
    return out


def grad_bounds(O, P, cache, dscore, elems, max_elems: int = 64):
    """(lo, hi) dicts of per-parameter gradient bounds over every ReLU branch
    choice at ``elems`` (see the module docstring)."""
    assert len(elems) <= max_elems, f"{len(elems)} kink elements: raise thr or max_elems deliberately"
    base = {(ti, li): (c[f"y{li}"] > 0) for ti, c in enumerate(cache["towers"]) for li in (0, 1)}
    for ti, li, r, col in elems:
        base[(ti, li)][r, col] = False
    g_off = O.backward(P, cache, dscore, relu_masks=base)
    lo = {k: v.clone() for k, v in g_off.items()}
    hi = {k: v.clone() for k, v in g_off.items()}
    for ti, li, r, col in elems:
        m = dict(base)
        m[(ti, li)] = base[(ti, li)].clone()
        m[(ti, li)][r, col] = True
        g_e = O.backward(P, cache, dscore, relu_masks=m)
        for k in lo:
            d = g_e[k] - g_off[k]
            lo[k] += d.clamp(max=0)
            hi[k] += d.clamp(min=0)
    return lo, hi


def bound_error(got, lo, hi, ref) -> float:
    """max(0, lo - got, got - hi) over the tensor, / max |ref|."""
    got = np.asarray(got, np.float64).reshape(-1)
    lo = np.asarray(lo, np.float64).reshape(-1)
    hi = np.asarray(hi, np.float64).reshape(-1)
    ref = np.asarray(ref, np.float64).reshape(-1)
    out = np.maximum(np.maximum(lo - got, got - hi), 0.0)
    den = np.max(np.abs(ref)) if ref.size else 0.0
    num = float(out.max()) if out.size else 0.0
    return num / den if den > 0 else num


def adam1_bounds(O, P, lo: Dict[str, torch.Tensor], hi: Dict[str, torch.Tensor], lr: float,
                 ref: Dict[str, torch.Tensor] = None, slack: float = 0.0):
    """Parameter bounds after ONE Adam step (fresh moments: monotone in g).

    With ``ref`` the gradient box is first widened by ``slack * max |ref|``
    per tensor -- the band the gradient check itself accepts (bound_error <
    slack).  The first Adam step is g / (|g| + eps): a component within that
    band of 0 may move the parameter by anything up to +-lr (its fp32 sum's
    order, atomic or not, picks the side), which the widened box covers; a
    wrong update (step size, moments, bias correction) still falls outside."""
    if ref is not None:
        pad = {k: slack * float(ref[k].abs().max()) if ref[k].numel() else 0.0 for k in lo}
        lo = {k: v - pad[k] for k, v in lo.items()}
        hi = {k: v + pad[k] for k, v in hi.items()}
    outs = []
    for g in (lo, hi):
        Pc = {k: v.clone() for k, v in P.items()}
        O.Adam(Pc, lr=lr).step(Pc, g)
        outs.append(Pc)
    a, b = outs
    return {k: torch.minimum(a[k], b[k]) for k in a}, {k: torch.maximum(a[k], b[k]) for k in a}


def adam1_replay_error(p0, g, p1, m1, v1, lr: float, m0=None, v0=None, t: int = 1, detail: bool = False):
    """The fused state after ONE Adam step against torch.optim.Adam
    (single-tensor, fp32, on the CPU) applied to the fused step's OWN
    gradient ``g`` from the same parameters ``p0``.  The gradient itself is
    held to the fp64 oracle by ``bound_error``; this pins the optimizer
    arithmetic element by element, which the parameter box of
    ``adam1_bounds`` cannot (a first Adam step is g / (|g| + eps): near-zero
    components may move by anything up to +-lr there).  Returns the largest
    deviation in units of 2 ulp of each element (of its terms' magnitude
    for exp_avg, whose terms may cancel; + 1e-6 lr for the parameters) --
    < 1 passes;
    the kernel's fp32 sequence is torch's, up to an FMA contraction (1 ulp
    of exp_avg_sq).  ``m0``, ``v0``, ``t``: the moments before step t > 1."""
    P = torch.as_tensor(np.asarray(p0, np.float32)).clone()
    P.grad = torch.as_tensor(np.asarray(g, np.float32)).clone()
    opt = torch.optim.Adam([P], lr=lr, foreach=False, fused=False)
    if t > 1:
        opt.state[P] = {"step": torch.tensor(float(t - 1)),
                        "exp_avg": torch.as_tensor(np.asarray(m0, np.float32)).clone().view_as(P),
                        "exp_avg_sq": torch.as_tensor(np.asarray(v0, np.float32)).clone().view_as(P)}
    opt.step()
    st = opt.state[P]
    worst, info = 0.0, None
    # the magnitude each result is rounded at: exp_avg = b1 m0 + (1 - b1) g
    # may cancel far below its terms (torch's CPU lerp and the kernel's may
    # round the terms differently: FMA or not), so its ulp is the terms'
    gv = np.abs(np.asarray(g, np.float64).reshape(-1))
    m_mag = 0.1 * gv + (0.9 * np.abs(np.asarray(m0, np.float64).reshape(-1)) if t > 1 else 0.0)
    for name, got, want, mag, floor in (("p", p1, P.detach(), None, 1e-6 * lr),
                                        ("exp_avg", m1, st["exp_avg"], m_mag, 1e-38),
                                        ("exp_avg_sq", v1, st["exp_avg_sq"], None, 1e-38)):
        got = np.asarray(got, np.float32).reshape(-1).astype(np.float64)
        want = want.numpy().reshape(-1)
        mag = np.abs(want).astype(np.float64) if mag is None else np.maximum(mag, np.abs(want))
        tol = 2.0 * np.spacing(mag.astype(np.float32)).astype(np.float64) + floor
        if got.size:
            r = np.abs(got - want.astype(np.float64)) / tol
            i = int(np.argmax(r))
            if r[i] > worst:
                worst = float(r[i])
                gi = np.asarray(g, np.float32).reshape(-1)[i]
                info = (name, i, float(got[i]), float(want[i]), float(gi),
                        float(np.asarray(p0, np.float32).reshape(-1)[i]))
    return (worst, info) if detail else worst
