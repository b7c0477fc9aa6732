import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_PARENT = os.path.join(ROOT, "ceo-recommender_amd")
for p in (ROOT, PKG_PARENT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def sub(d, prefix):
    """{'a/b/c': x} -> sub(d, 'a/b') == {'c': x}"""
    pre = prefix + "/"
    return {k[len(pre):]: v for k, v in d.items() if k.startswith(pre)}


def meta_of(g):
    return {"n_firm_numeric": int(g["meta/n_firm_numeric"]),
            "firm_cat_counts": [int(x) for x in g["meta/firm_cat_counts"]],
            "n_ceo_numeric": int(g["meta/n_ceo_numeric"]),
            "ceo_cat_counts": [int(x) for x in g["meta/ceo_cat_counts"]]}


def normwise(a, b):
    """||a-b||_inf / ||b||_inf (SURVEY 8c tolerance rule)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.max(np.abs(b)) if b.size else 0.0
    num = np.max(np.abs(a - b)) if b.size else 0.0
    return num / den if den > 0 else num


# pre-BatchNorm Linear biases: true gradient is exactly 0 (BN cancels them),
# fp32 gives ~1e-6 noise and Adam turns noise into +-lr updates -> not
# comparable across implementations.
def excluded_param(name):
    if name.startswith("base_model."):  # ContrastiveCEOFirmMatcher wraps the base model
        name = name[len("base_model."):]
    return any(name.startswith(f"{t}_tower.{i}.bias") for t in ("firm", "ceo") for i in ("0", "4"))


@pytest.fixture
def golden():
    return load_golden
