"""Interaction heatmaps on the fused eval forward.

Reference ``visualization.py:19-170`` (``plot_interaction_heatmap``) evaluates
a 50 x 50 grid (or categories) of two features around the data's baseline
(mean numeric features, modal categories) with one ``model(...)`` call and
one ``.item()`` sync per cell -- 2,500 batch-1 forwards per plot.  In eval
mode BatchNorm uses its running statistics, so every cell is independent:
here the whole grid is ONE batched forward (on a HIP device: one tt_forward
launch sequence) and one copy back.  Same grid, same baseline, same plot.
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np
import torch

from .data import DataProcessor


def _feature_info(processor: DataProcessor, name: str) -> Tuple[str, int]:
    if name in processor.final_firm_numeric:
        return 'firm_numeric', list(processor.scalers['firm'].feature_names_in_).index(name)
    if name in processor.final_ceo_numeric:
        return 'ceo_numeric', list(processor.scalers['ceo'].feature_names_in_).index(name)
    if name in processor.cfg.FIRM_CAT_COLS:
        return 'firm_cat', list(processor.cfg.FIRM_CAT_COLS).index(name)
    if name in processor.cfg.CEO_CAT_COLS:
        return 'ceo_cat', list(processor.cfg.CEO_CAT_COLS).index(name)
    raise ValueError(f"Feature {name} not supported for heatmap.")


def interaction_grid(model, processor: DataProcessor, x_feature: str, y_feature: str):
    """(x_vals, y_vals, heatmap[len(y), len(x)]) of the model's eval score
    with x_feature / y_feature swept over the reference's grid."""
    data = processor._to_tensors(processor.processed_df)
    dev = processor.cfg.DEVICE
    d = {k: data[k].to(dev) for k in ('firm_numeric', 'firm_cat', 'ceo_numeric', 'ceo_cat')}
    x_type, x_idx = _feature_info(processor, x_feature)
    y_type, y_idx = _feature_info(processor, y_feature)

    def grid(kind, idx):
        if kind in ('firm_cat', 'ceo_cat'):
            col = (processor.cfg.FIRM_CAT_COLS if kind == 'firm_cat' else processor.cfg.CEO_CAT_COLS)[idx]
            return np.arange(len(processor.encoders[col].classes_))
        return np.linspace(d[kind][:, idx].min().item(), d[kind][:, idx].max().item(), 50)

    x_vals, y_vals = grid(x_type, x_idx), grid(y_type, y_idx)
    ny, nx = len(y_vals), len(x_vals)
    base = {
        'firm_numeric': torch.mean(d['firm_numeric'], dim=0, keepdim=True),
        'ceo_numeric': torch.mean(d['ceo_numeric'], dim=0, keepdim=True),
        'firm_cat': torch.mode(d['firm_cat'].cpu(), dim=0)[0].view(1, -1).to(dev),
        'ceo_cat': torch.mode(d['ceo_cat'].cpu(), dim=0)[0].view(1, -1).to(dev),
    }
    batch = {k: v.repeat(ny * nx, 1) for k, v in base.items()}
    # row (i, j) = y_vals[i], x_vals[j]: x first, then y (reference update order)
    for kind, idx, vals, along_x in ((x_type, x_idx, x_vals, True), (y_type, y_idx, y_vals, False)):
        v = torch.as_tensor(vals, dtype=torch.float64)
        v = v.repeat(ny) if along_x else v.repeat_interleave(nx)
        if kind.endswith('cat'):
            batch[kind][:, idx] = v.to(torch.int64).to(dev)
        else:
            batch[kind][:, idx] = v.to(torch.float32).to(dev)
    model.eval()
    with torch.no_grad():
        s = model(batch['firm_numeric'], batch['firm_cat'], batch['ceo_numeric'], batch['ceo_cat'])
    return x_vals, y_vals, s.reshape(ny, nx).double().cpu().numpy()


def plot_interaction_heatmap(model, processor: DataProcessor, x_feature: str, y_feature: str, filename: str):
    """Reference visualization.py:19 signature; the grid is one batched forward."""
    if model is None or processor.processed_df is None:
        return None
    print(f"\nGenerating interaction heatmap ({x_feature} vs {y_feature})...")
    try:
        x_vals, y_vals, heatmap = interaction_grid(model, processor, x_feature, y_feature)
    except ValueError as e:
        print(f"Visualization Error: {e}")
        return None
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    x_cat = _feature_info(processor, x_feature)[0].endswith('cat')
    y_cat = _feature_info(processor, y_feature)[0].endswith('cat')
    fig, ax = plt.subplots(figsize=(10, 6))
    if x_cat or y_cat:
        im = ax.imshow(heatmap, aspect='auto', cmap='RdBu_r', origin='lower', interpolation='nearest')
        for axis, vals, cat, feat in ((ax.xaxis, x_vals, x_cat, x_feature), (ax.yaxis, y_vals, y_cat, y_feature)):
            if cat:
                axis.set_ticks(np.arange(len(vals)), [int(v) for v in vals])
                axis.set_label_text(f'{feat} (Category)')
            else:
                axis.set_ticks(np.linspace(0, len(vals) - 1, 5),
                               [f'{v:.1f}' for v in np.linspace(vals.min(), vals.max(), 5)])
                axis.set_label_text(f'{feat} (Standardized)')
    else:
        im = ax.imshow(heatmap, aspect='auto', cmap='RdBu_r', origin='lower', interpolation='bicubic',
                       extent=[x_vals.min(), x_vals.max(), y_vals.min(), y_vals.max()])
        ax.set_xlabel(f'{x_feature} (Standardized)')
        ax.set_ylabel(f'{y_feature} (Standardized)')
    plt.colorbar(im, label='Predicted Match Quality')
    ax.set_title(f'Interaction: {x_feature} vs {y_feature}')
    out = processor.cfg.OUTPUT_PATH
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, filename)
    plt.savefig(path)
    plt.close(fig)
    print(f"Saved heatmap to {path}")
    return heatmap
