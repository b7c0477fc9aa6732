"""Partial dependence on the fused eval forward.

Reference ``explain.py:19-131``: ``ModelWrapper`` (sklearn-like predict over
the flat [firm num | firm cat | ceo num | ceo cat] layout) and
``explain_model_pdp`` (per feature: 50 grid values x a 1,000-row sample, 50
predict calls).  Here each feature's whole 50 x 1,000 grid is ONE batched
forward; the sample is drawn with the same global numpy RNG call, so the
curves match the reference's.  SHAP (``explain_model_shap``) stays out of
scope (the ``shap`` package is not part of this build).
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import numpy as np
import pandas as pd
import torch

from .data import DataProcessor


class ModelWrapper:
    """Reference explain.py:19-64."""

    def __init__(self, model, processor: DataProcessor):
        self.model = model
        self.processor = processor
        self.device = processor.cfg.DEVICE
        self.n_firm_num = len(processor.final_firm_numeric)
        self.n_firm_cat = len(processor.cfg.FIRM_CAT_COLS)
        self.n_ceo_num = len(processor.final_ceo_numeric)
        self.n_ceo_cat = len(processor.cfg.CEO_CAT_COLS)
        self.idx_firm_num_end = self.n_firm_num
        self.idx_firm_cat_end = self.idx_firm_num_end + self.n_firm_cat
        self.idx_ceo_num_end = self.idx_firm_cat_end + self.n_ceo_num
        self.idx_ceo_cat_end = self.idx_ceo_num_end + self.n_ceo_cat

    def predict(self, X: np.ndarray) -> np.ndarray:
        self.model.eval()
        x = torch.tensor(X, dtype=torch.float32).to(self.device)
        a, b, c = self.idx_firm_num_end, self.idx_firm_cat_end, self.idx_ceo_num_end
        with torch.no_grad():
            preds = self.model(x[:, :a], x[:, a:b].long(), x[:, b:c], x[:, c:].long())
        return preds.cpu().numpy().flatten()


def partial_dependence(wrapper: ModelWrapper, df: pd.DataFrame, features: List[str], n_grid: int = 50,
                       n_sample: int = 1000) -> Dict[str, Tuple[np.ndarray, np.ndarray]]:
    """{feature: (grid, mean prediction)} -- reference explain.py:67-118 with
    one predict call per feature."""
    d = wrapper.processor.transform(df)
    X = np.hstack([d['firm_numeric'].numpy(), d['firm_cat'].numpy(), d['ceo_numeric'].numpy(),
                   d['ceo_cat'].numpy()])
    names = wrapper.processor.get_feature_names()
    out = {}
    for name in features:
        if name not in names:
            print(f"Warning: Feature '{name}' not found in model inputs.")
            continue
        idx = names.index(name)
        vals = X[:, idx]
        grid = np.linspace(vals.min(), vals.max(), n_grid)
        sample = X[np.random.choice(X.shape[0], min(n_sample, X.shape[0]), replace=False)]
        big = np.repeat(sample[None], n_grid, axis=0)  # [grid, sample, features]
        big[:, :, idx] = grid[:, None]
        preds = wrapper.predict(big.reshape(-1, X.shape[1])).reshape(n_grid, -1)
        out[name] = (grid, preds.astype(np.float64).mean(axis=1))
    return out


def explain_model_pdp(wrapper: ModelWrapper, df: pd.DataFrame, features_to_plot: List[str]):
    """Reference explain.py:67 signature: PDP panels saved as pdp_plots.svg."""
    print("\nGenerating Partial Dependence Plots (PDP)...")
    curves = partial_dependence(wrapper, df, features_to_plot)
    if not curves:
        return curves
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, axes = plt.subplots(1, len(curves), figsize=(5 * len(curves), 4))
    axes = np.atleast_1d(axes)
    for ax, (name, (grid, y)) in zip(axes, curves.items()):
        ax.plot(grid, y, color='blue')
        ax.set_title(f"PDP: {name}")
        ax.set_xlabel("Standardized Value / Code")
        ax.set_ylabel("Avg Match Score")
        ax.grid(True, alpha=0.3)
    plt.tight_layout()
    out = wrapper.processor.cfg.OUTPUT_PATH
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, "pdp_plots.svg")
    plt.savefig(path)
    print(f"Saved PDP plots to {path}")
    plt.close(fig)
    return curves


def explain_model_shap(wrapper: ModelWrapper, df: pd.DataFrame):
    """Reference explain.py:134-170 (SHAP KernelExplainer summary plot).
    Not part of this build: the ``shap`` package is absent from the image and
    the explainer is off the training path (the reference CLI disables it)."""
    raise NotImplementedError("explain_model_shap needs the 'shap' package, which this MI355X build does not "
                              "ship; use explain_model_pdp (batched on the fused eval forward)")
