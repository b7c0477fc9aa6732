"""Integrated gradients on the fused eval-mode backward.

Reference: ``run_deep_extensions.py:550-603`` ``integrated_gradients(model,
inputs, baselines, n_steps=50)`` -- ``model.eval()``, then for each of the
``n_steps + 1`` points on the straight path from the baseline to the input a
batch-1 forward, ``requires_grad_`` on the numeric inputs, ``score.backward()``
and a read of ``f_num.grad`` / ``c_num.grad``; the attributions are the mean
gradient times (input - baseline).

In eval mode BatchNorm is the affine map of the running statistics, so the
rows of a batch do not interact: the gradient of row ``k`` of one batched
forward equals the batch-1 gradient at that point.  Here the whole path is
ONE fused eval forward + backward of ``n_steps + 1`` rows (the kernels'
``tt_backward_ex`` with input gradients) instead of ``n_steps + 1`` batch-1
round trips.  Parameter ``.grad`` fields are left untouched (the gradients
are taken with ``torch.autograd.grad`` on the inputs only).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch


def integrated_gradients(model, inputs: Dict[str, torch.Tensor], baselines: Dict[str, torch.Tensor],
                         n_steps: int = 50) -> Dict[str, np.ndarray]:
    """{'firm_numeric': [n_firm], 'ceo_numeric': [n_ceo]} attributions of one
    input row (every tensor of ``inputs`` / ``baselines`` shaped [1, n])."""
    model.eval()
    f_in, c_in = inputs["firm_numeric"], inputs["ceo_numeric"]
    dev = f_in.device
    alphas = torch.linspace(0, 1, n_steps + 1, device=dev)
    f_b = baselines["firm_numeric"].to(device=dev, dtype=f_in.dtype)
    c_b = baselines["ceo_numeric"].to(device=dev, dtype=c_in.dtype)
    a_f = alphas.to(f_in.dtype)[:, None]
    a_c = alphas.to(c_in.dtype)[:, None]
    f_path = (f_b + a_f * (f_in - f_b)).detach().requires_grad_(True)   # [n_steps+1, n_firm]
    c_path = (c_b + a_c * (c_in - c_b)).detach().requires_grad_(True)
    rows = n_steps + 1
    f_cat = inputs["firm_cat"].expand(rows, -1) if inputs["firm_cat"].dim() == 2 else inputs["firm_cat"]
    c_cat = inputs["ceo_cat"].expand(rows, -1) if inputs["ceo_cat"].dim() == 2 else inputs["ceo_cat"]
    out = model(f_path, f_cat.contiguous(), c_path, c_cat.contiguous())
    score = out[0] if isinstance(out, tuple) else out
    gf, gc = torch.autograd.grad(score.sum(), (f_path, c_path))
    firm_ig = gf.mean(dim=0, keepdim=True) * (f_in.detach() - f_b)
    ceo_ig = gc.mean(dim=0, keepdim=True) * (c_in.detach() - c_b)
    return {"firm_numeric": firm_ig.squeeze(0).cpu().numpy(), "ceo_numeric": ceo_ig.squeeze(0).cpu().numpy()}
