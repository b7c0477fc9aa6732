"""Pin the contrastive oracle (oracle/contrastive.py) to the reference's
own outputs (tests/golden/contrastive.npz, produced by running
contrastive.py:102-138 and :275-332 -- make_golden.py)."""
import numpy as np
import pytest
import torch

from conftest import load_golden, normwise
from oracle import contrastive as OC

CASES = ["b1", "b2", "b64", "b256", "raw256"]


@pytest.mark.parametrize("case", CASES)
def test_info_nce_matches_reference(case):
    g = load_golden("contrastive")
    f = torch.from_numpy(g[f"nce/{case}/f"]).double()
    c = torch.from_numpy(g[f"nce/{case}/c"]).double()
    loss, df, dc = OC.info_nce(f, c, 0.07)
    assert abs(float(loss) - float(g[f"nce/{case}/loss64"])) <= 1e-12 * max(1.0, abs(float(loss)))
    assert abs(float(loss) - float(g[f"nce/{case}/loss"])) <= 1e-5 * max(1.0, abs(float(loss)))
    if f.shape[0] <= 1:
        assert df is None and f"nce/{case}/df64" not in g
        return
    assert normwise(df.numpy(), g[f"nce/{case}/df64"]) < 1e-6
    assert normwise(dc.numpy(), g[f"nce/{case}/dc64"]) < 1e-6
    if f"nce/{case}/df" in g:  # the reference's own fp32 autograd
        assert normwise(df.numpy(), g[f"nce/{case}/df"]) < 1e-5
        assert normwise(dc.numpy(), g[f"nce/{case}/dc"]) < 1e-5


def test_retrieval_metrics_match_reference():
    g = load_golden("contrastive")
    fe = torch.from_numpy(g["ret/firm_emb"])
    ce = torch.from_numpy(g["ret/ceo_emb"])
    ranks = OC.retrieval_ranks(fe, ce, cap=5000)
    got = OC.retrieval_metrics(ranks)
    for k in ("recall@1", "recall@5", "recall@10", "MRR", "median_rank"):
        assert got[k] == pytest.approx(float(g[f"ret/metric/{k}"]), rel=1e-12, abs=1e-12), k


def test_mfma_order_dot_is_a_dot():
    rng = np.random.default_rng(0)
    a = rng.standard_normal((50, 256)).astype(np.float32)
    b = rng.standard_normal((50, 256)).astype(np.float32)
    ref = (a.astype(np.float64) * b).sum(1)
    assert np.max(np.abs(OC.mfma_order_dot(a, b) - ref)) < 1e-4


TRI_CASES = ["b1", "b2", "b64", "b256", "corr128", "raw96"]


@pytest.mark.parametrize("case", TRI_CASES)
def test_semi_hard_matches_reference(case):
    """oracle.semi_hard vs the reference's semi_hard_negative_mining
    (contrastive.py:141-192) in fp64 (exact selection) and fp32."""
    g = load_golden("triplet")
    f = torch.from_numpy(g[f"tri/{case}/f"])
    c = torch.from_numpy(g[f"tri/{case}/c"])
    o64 = OC.semi_hard(f.double(), c.double(), 0.2)
    assert abs(float(o64["loss"]) - float(g[f"tri/{case}/loss64"])) <= 1e-12
    if f.shape[0] <= 1:
        assert f"tri/{case}/df64" not in g
        return
    assert normwise(o64["df"].numpy(), g[f"tri/{case}/df64"]) < 1e-6
    assert normwise(o64["dc"].numpy(), g[f"tri/{case}/dc64"]) < 1e-6
    o32 = OC.semi_hard(f, c, 0.2)
    assert abs(float(o32["loss"]) - float(g[f"tri/{case}/loss"])) <= 1e-5 * max(1.0, float(g[f"tri/{case}/loss"]))
    assert normwise(o32["df"].numpy(), g[f"tri/{case}/df"]) < 1e-5
    assert normwise(o32["dc"].numpy(), g[f"tri/{case}/dc"]) < 1e-5


def test_semi_hard_cases_cover_both_branches():
    g = load_golden("triplet")
    o = OC.semi_hard(torch.from_numpy(g["tri/corr128/f"]).double(), torch.from_numpy(g["tri/corr128/c"]).double())
    assert 0 < int(o["semi"].sum()) < 128           # semi-hard picks and fallbacks
    assert 0 < int(o["active"].sum()) < 128         # active and zero-loss rows


def test_semi_hard_aten_path_matches_oracle():
    """The package's CPU (ATen) semi_hard_negative_mining == the oracle."""
    from ceo_firm_matching.contrastive import semi_hard_negative_mining
    g = load_golden("triplet")
    for case in TRI_CASES:
        f = torch.from_numpy(g[f"tri/{case}/f"])
        c = torch.from_numpy(g[f"tri/{case}/c"])
        got = semi_hard_negative_mining(f, c, 0.2)
        assert abs(float(got) - float(g[f"tri/{case}/loss"])) <= 1e-6, case
