"""Eval consumers on CPU: the batched interaction grid and
partial dependence equal the reference's per-cell / per-grid-value loops
(visualization.py:98-123, explain.py:102-118) restated here over the same
model; the CLI draws the reference's plots."""
import contextlib
import io
import os

import numpy as np
import torch

from conftest import PKG_PARENT
from ceo_firm_matching import CEOFirmMatcher, Config
from ceo_firm_matching.explain import ModelWrapper, partial_dependence
from ceo_firm_matching.visualization import interaction_grid
from test_host_pipeline import cli_data


def _setup():
    cfg = Config()
    cfg.DEVICE = torch.device("cpu")
    from ceo_firm_matching.data import DataProcessor
    from ceo_firm_matching.synthetic import generate_synthetic_data
    from sklearn.model_selection import train_test_split
    proc = DataProcessor(cfg)
    with contextlib.redirect_stdout(io.StringIO()):
        df = proc.prepare_features(generate_synthetic_data(400))
        tr, va = train_test_split(df, test_size=0.2, random_state=42)
        proc.fit(tr)
        train = proc.transform(tr)
        proc.transform(va)
    torch.manual_seed(3)
    model = CEOFirmMatcher(train, cfg)
    model.eval()
    for bn in (model.firm_tower[1], model.firm_tower[5], model.ceo_tower[1], model.ceo_tower[5]):
        bn.running_mean.uniform_(-0.5, 0.5)
        bn.running_var.uniform_(0.5, 2.0)
    return cfg, proc, model, va


def _loop_grid(model, proc, xf, yf):
    """The reference's cell-by-cell evaluation (visualization.py:98-123)."""
    from ceo_firm_matching.visualization import _feature_info
    d = proc._to_tensors(proc.processed_df)
    xt, xi = _feature_info(proc, xf)
    yt, yi = _feature_info(proc, yf)
    xs, ys, _ = interaction_grid(model, proc, xf, yf)
    f0 = d['firm_numeric'].mean(0, keepdim=True)
    c0 = d['ceo_numeric'].mean(0, keepdim=True)
    fc0 = torch.mode(d['firm_cat'], dim=0)[0].view(1, -1)
    cc0 = torch.mode(d['ceo_cat'], dim=0)[0].view(1, -1)
    out = np.zeros((len(ys), len(xs)))
    with torch.no_grad():
        for i, yv in enumerate(ys):
            for j, xv in enumerate(xs):
                t = {'firm_numeric': f0.clone(), 'ceo_numeric': c0.clone(), 'firm_cat': fc0.clone(),
                     'ceo_cat': cc0.clone()}
                for kind, idx, v in ((xt, xi, xv), (yt, yi, yv)):
                    t[kind][:, idx] = int(v) if kind.endswith('cat') else float(v)
                out[i, j] = model(t['firm_numeric'], t['firm_cat'], t['ceo_numeric'], t['ceo_cat']).item()
    return out


def test_interaction_grid_equals_cell_loop():
    cfg, proc, model, _ = _setup()
    for xf, yf in (('logatw', 'Age'), ('logatw', 'Output'), ('maxedu', 'rdintw')):
        _, _, got = interaction_grid(model, proc, xf, yf)
        ref = _loop_grid(model, proc, xf, yf)
        assert got.shape == ref.shape
        assert np.max(np.abs(got - ref)) <= 1e-5 * max(1.0, np.max(np.abs(ref))), (xf, yf)


def test_partial_dependence_equals_grid_loop():
    cfg, proc, model, va = _setup()
    w = ModelWrapper(model, proc)
    np.random.seed(7)
    got = partial_dependence(w, va, ['logatw', 'Age', 'Output'])
    np.random.seed(7)
    d = proc.transform(va)
    X = np.hstack([d['firm_numeric'].numpy(), d['firm_cat'].numpy(), d['ceo_numeric'].numpy(), d['ceo_cat'].numpy()])
    names = proc.get_feature_names()
    for name in ('logatw', 'Age', 'Output'):
        idx = names.index(name)
        grid = np.linspace(X[:, idx].min(), X[:, idx].max(), 50)
        sample = X[np.random.choice(X.shape[0], min(1000, X.shape[0]), replace=False)].copy()
        ref = []
        for v in grid:
            t = sample.copy()
            t[:, idx] = v
            ref.append(np.mean(w.predict(t)))
        g, y = got[name]
        assert np.array_equal(g, grid)
        assert np.max(np.abs(y - np.array(ref))) <= 1e-5 * max(1.0, np.max(np.abs(ref))), name


def test_cli_draws_reference_plots(tmp_path):
    import subprocess
    import sys
    env = dict(os.environ, PYTHONPATH=PKG_PARENT, CEO_TT_OUTPUT=str(tmp_path), HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "ceo_firm_matching.cli", "--synthetic", "--epochs", "1"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    files = sorted(os.listdir(tmp_path))
    assert "pdp_plots.svg" in files
    assert sum(f.startswith("heatmap_") for f in files) == 11
