"""Synthetic data.

* ``generate_synthetic_data(n)`` -- the reference schema generator
  (``synthetic.py:10-75``): same columns, same ``np.random.seed(42)`` draws in
  the same order, so for n <= 114,057 it returns the reference's frame.  The
  reference crashes above that (``pd.date_range`` overflows pandas' ns range,
  ``synthetic.py:43``); here the DOB calendar wraps every 114,000 days.
* ``generate_pairs(n, n_firm, n_ceo, ...)`` -- the scaled generator of the
  benchmark configs (SURVEY 8d cfg 2-4): post-StandardScaler features
  N(0,1), target N(0,1), sd ~ U(0.1, 1), weights = 1/(sd^2+1e-6), generated
  directly on the device so 10M-pair datasets never touch the host.
"""
from typing import Dict, Optional

import numpy as np
import pandas as pd
import torch

_DOB_PERIOD = 114_000


def _dob(n: int):
    base = pd.date_range(start='1950-01-01', periods=min(n, _DOB_PERIOD)).strftime('%Y-%m-%d')
    if n <= _DOB_PERIOD:
        return base
    reps = -(-n // _DOB_PERIOD)
    return np.tile(np.asarray(base), reps)[:n]


def generate_synthetic_data(n_samples: int = 1000) -> pd.DataFrame:
    """Synthetic frame with the schema the Two Towers pipeline needs."""
    np.random.seed(42)
    r = np.random
    n = n_samples
    data = {
        'gvkey': r.randint(1000, 9999, n),
        'match_exec_id': r.randint(10000, 99999, n),
        'Age': r.uniform(30, 70, n),
        'Output': r.randint(0, 2, n),
        'Throghput': r.randint(0, 2, n),
        'Peripheral': r.randint(0, 2, n),
        'Gender': r.choice(['M', 'F'], n),
        'maxedu': r.randint(1, 5, n),
        'ivy': r.randint(0, 2, n),
        'm': r.randint(0, 2, n),
        'ceo_year': r.randint(2000, 2023, n),
        'year_born': r.randint(1950, 1990, n),
        'dep_baby_ceo': r.randint(0, 2, n),
        'DOB': _dob(n),
        'ind_firms_60w': r.normal(0, 1, n),
        'non_competition_score': r.uniform(0, 1, n),
        'boardindpw': r.uniform(0, 1, n),
        'boardsizew': r.randint(5, 20, n),
        'busyw': r.randint(0, 5, n),
        'pct_blockw': r.uniform(0, 100, n),
        'logatw': r.uniform(5, 15, n),
        'exp_roa': r.normal(0.05, 0.02, n),
        'rdintw': r.uniform(0, 0.2, n),
        'capintw': r.uniform(0, 0.3, n),
        'leverage': r.uniform(0, 1, n),
        'divyieldw': r.uniform(0, 0.05, n),
        'compindustry': r.choice(['Tech', 'Finance', 'Health', 'Energy'], n),
        'ba_state': r.choice(['CA', 'NY', 'TX', 'MA'], n),
        'rd_control': r.randint(0, 2, n),
        'dpayer': r.randint(0, 2, n),
        'fiscalyear': r.randint(2000, 2023, n),
        'match_means': r.normal(0, 1, n),
        'sd_match_means': r.uniform(0.1, 1.0, n),
        'mover': r.randint(0, 2, n),
        'output_exp_dummy': r.randint(0, 2, n),
    }
    return pd.DataFrame(data)


def generate_structural_synthetic_data(n_samples: int = 2000, seed: int = 42) -> pd.DataFrame:
    """Reference synthetic.py:78-110: the base frame plus BLM posterior type
    probabilities ``prob_ceo_1..5`` / ``prob_firm_1..5`` (flat Dirichlet, drawn
    from the global numpy RNG after the base frame's draws, which reseed 42)
    and ``tenure`` = (fiscalyear - ceo_year) clipped at 0."""
    np.random.seed(seed)
    df = generate_synthetic_data(n_samples)
    ceo = np.random.dirichlet(np.ones(5), n_samples)
    for i in range(5):
        df[f'prob_ceo_{i + 1}'] = ceo[:, i]
    firm = np.random.dirichlet(np.ones(5), n_samples)
    for i in range(5):
        df[f'prob_firm_{i + 1}'] = firm[:, i]
    df['tenure'] = (df['fiscalyear'] - df['ceo_year']).clip(lower=0)
    return df


def generate_pairs(n: int, n_firm: int, n_ceo: int, seed: int = 42,
                   device: Optional[torch.device] = None, chunk: int = 1 << 22) -> Dict[str, torch.Tensor]:
    """Scaled (firm, CEO) pair dataset in the CEOFirmDataset dict layout."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    f = torch.empty(n, n_firm, device=dev)
    c = torch.empty(n, n_ceo, device=dev)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        f[s:e].normal_(generator=g)
        c[s:e].normal_(generator=g)
    target = torch.empty(n, 1, device=dev).normal_(generator=g)
    sd = torch.empty(n, 1, device=dev).uniform_(0.1, 1.0, generator=g)
    weights = 1.0 / (sd * sd + 1e-6)
    empty = torch.zeros(n, 0, dtype=torch.int64, device=dev)
    return {"firm_numeric": f, "firm_cat": empty, "ceo_numeric": c, "ceo_cat": empty.clone(),
            "target": target, "weights": weights,
            "n_firm_numeric": n_firm, "firm_cat_counts": [], "n_ceo_numeric": n_ceo, "ceo_cat_counts": []}
