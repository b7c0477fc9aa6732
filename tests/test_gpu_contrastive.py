"""HIP contrastive kernels (tt_nce_*, tt_retrieval_ranks) vs the reference's
golden vectors (tests/golden/contrastive.npz) and the CPU oracle
(oracle/contrastive.py).  Tolerance: normwise 1e-5 (loss: relative 1e-5)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import load_golden, normwise
from oracle import contrastive as OC

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _nce(f, c, tau=0.07):
    from ceo_firm_matching.contrastive import info_nce_loss
    f = f.clone().requires_grad_(True)
    c = c.clone().requires_grad_(True)
    loss = info_nce_loss(f, c, tau)
    if loss.requires_grad:
        loss.backward()
    return loss, f.grad, c.grad


@pytest.mark.parametrize("case", ["b1", "b2", "b64", "b256", "raw256"])
def test_info_nce_golden(case):
    dev = _dev()
    g = load_golden("contrastive")
    f = torch.from_numpy(g[f"nce/{case}/f"]).to(dev)
    c = torch.from_numpy(g[f"nce/{case}/c"]).to(dev)
    loss, df, dc = _nce(f, c)
    ref = float(g[f"nce/{case}/loss64"])
    assert abs(float(loss.detach()) - ref) <= TOL * max(1.0, abs(ref)), (float(loss.detach()), ref)
    if f.shape[0] <= 1:
        assert df is None
        return
    assert normwise(df.cpu().numpy(), g[f"nce/{case}/df64"]) < TOL
    assert normwise(dc.cpu().numpy(), g[f"nce/{case}/dc64"]) < TOL


@pytest.mark.parametrize("B,D", [(3000, 256), (1000, 100), (517, 36), (4100, 64)])
def test_info_nce_ragged_vs_oracle(B, D):
    """Partial tiles, several blocks / K splits, D not a multiple of 16."""
    dev = _dev()
    gen = torch.Generator().manual_seed(B + D)
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1)
    c = torch.nn.functional.normalize(torch.randn(B, D, generator=gen) + 0.3 * f, dim=1)
    loss, df, dc = _nce(f.to(dev), c.to(dev))
    rl, rdf, rdc = OC.info_nce(f.double(), c.double(), 0.07)
    assert abs(float(loss) - float(rl)) <= TOL * abs(float(rl))
    assert normwise(df.cpu().numpy(), rdf.numpy()) < TOL
    assert normwise(dc.cpu().numpy(), rdc.numpy()) < TOL


@pytest.mark.parametrize("B,D,W", [(2048, 128, 4), (100_000, 256, 8)])
def test_info_nce_row_shards_compose(B, D, W):
    """The sharded decomposition (row0 offsets, partial column sums, partial
    dC) reproduces the full loss on one device -- the multi-GPU algebra of
    info_nce_loss_sharded; (100k, 256, 8) is BASELINE cfg 5's production
    shape (8 ranks x 12,500 firm rows against all 100k CEO rows), checked
    against the chunked fp64 device reference."""
    from ceo_firm_matching.contrastive import _NCE
    dev = _dev()
    gen = torch.Generator().manual_seed(3)
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1).to(dev)
    c = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1).to(dev)
    m = B // W
    hs = [_NCE(f[r * m:(r + 1) * m].contiguous(), c, m, B, D, r * m, B, 0.07) for r in range(W)]
    n2 = torch.stack([h.norms() for h in hs]).max(dim=0).values
    col = sum(h.forward(n2) for h in hs)
    parts = [h.loss(col) for h in hs]
    assert sum(int(st.item()) for _, st in parts) == 0
    loss = sum(lo for lo, _ in parts)
    df, dc = None, None
    for i, h in enumerate(hs):  # each shard's E released after its backward
        g_ = h.backward()
        df = g_[0] if df is None else torch.cat([df, g_[0]])
        dc = g_[1] if dc is None else dc + g_[1]
        hs[i] = None
        del h, g_
    loss = float(loss)
    del hs
    torch.cuda.empty_cache()
    if B <= 4096:
        rl, rdf, rdc = OC.info_nce(f.cpu().double(), c.cpu().double(), 0.07)
        rdf, rdc = rdf.to(dev), rdc.to(dev)
        rl = float(rl)
    else:
        rl, rdf, rdc = _info_nce_fp64_chunked(f, c, 0.07)
    assert abs(loss - rl) <= TOL * abs(rl), (loss, rl)
    for got, ref in ((df, rdf), (dc, rdc)):
        err = float((got.double() - ref).abs().max() / ref.abs().max())
        assert err < TOL, err


def test_info_nce_robust_row_shards_compose():
    """The robust pass's sharded decomposition (per-shard row maxima, MAX of
    the column maxima, SUM of the shifted column sums, per-shard losses and
    dC) reproduces the full loss at a temperature the shared shift cannot
    serve -- the collectives info_nce_loss_sharded runs in its fallback."""
    from ceo_firm_matching.contrastive import _NCE
    dev = _dev()
    gen = torch.Generator().manual_seed(4)
    B, D, W, tau = 1536, 64, 3, 0.004
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1)
    c = torch.nn.functional.normalize(torch.randn(B, D, generator=gen) + 0.5 * f, dim=1)
    fd, cd = f.to(dev), c.to(dev)
    m = B // W
    hs = [_NCE(fd[r * m:(r + 1) * m].contiguous(), cd, m, B, D, r * m, B, tau) for r in range(W)]
    cmax = torch.stack([h.maxes() for h in hs]).max(dim=0).values
    col = sum(h.forward_lse(cmax) for h in hs)
    parts = [h.loss_lse(cmax, col) for h in hs]
    assert sum(int(st.item()) for _, st in parts) == 0
    loss = sum(lo for lo, _ in parts)
    grads = [h.backward() for h in hs]
    df = torch.cat([g_[0] for g_ in grads])
    dc = sum(g_[1] for g_ in grads)
    rl, rdf, rdc = OC.info_nce(f.double(), c.double(), tau)
    l32, df32, dc32 = OC.info_nce(f, c, tau)
    assert abs(float(loss) - float(rl)) <= max(TOL * abs(float(rl)), 10 * abs(float(l32) - float(rl)))
    for got, ref, r32 in ((df, rdf, df32), (dc, rdc, dc32)):
        assert normwise(got.cpu().numpy(), ref.numpy()) <= max(TOL, 10 * normwise(r32.double().numpy(), ref.numpy()))


def test_info_nce_one_long_row_vs_oracle():
    """One row 40x longer than the rest: the shared shift (40/tau) underflows
    every other row's sum; the robust pass returns the reference's finite
    loss and gradients (was: NotImplementedError)."""
    dev = _dev()
    gen = torch.Generator().manual_seed(1)
    f = torch.nn.functional.normalize(torch.randn(64, 32, generator=gen), dim=1)
    f[0] *= 40.0
    c = f.clone()
    loss, df, dc = _nce(f.to(dev), c.to(dev))
    rl, rdf, rdc = OC.info_nce(f.double(), c.double(), 0.07)
    l32, df32, dc32 = OC.info_nce(f, c, 0.07)
    assert abs(float(loss.detach()) - float(rl)) <= max(TOL * abs(float(rl)), 10 * abs(float(l32) - float(rl)))
    for got, ref, r32 in ((df, rdf, df32), (dc, rdc, dc32)):
        assert normwise(got.cpu().numpy(), ref.numpy()) <= max(TOL, 10 * normwise(r32.double().numpy(), ref.numpy()))


def test_retrieval_golden_metrics():
    dev = _dev()
    from ceo_firm_matching.contrastive import metrics_from_ranks, retrieval_ranks
    g = load_golden("contrastive")
    fe = torch.from_numpy(g["ret/firm_emb"]).to(dev)
    ce = torch.from_numpy(g["ret/ceo_emb"]).to(dev)
    got = metrics_from_ranks(retrieval_ranks(fe, ce))
    for k in ("recall@1", "recall@5", "recall@10", "MRR", "median_rank"):
        assert got[k] == pytest.approx(float(g[f"ret/metric/{k}"]), rel=1e-12, abs=1e-12), k


@pytest.mark.parametrize("N,D,cap", [(5000, 256, 5000), (7000, 64, None), (333, 30 + 2, None)])
def test_retrieval_ranks_vs_oracle(N, D, cap):
    dev = _dev()
    from ceo_firm_matching.contrastive import retrieval_ranks
    gen = torch.Generator().manual_seed(N)
    f = torch.nn.functional.normalize(torch.randn(N, D, generator=gen), dim=1)
    c = torch.nn.functional.normalize(torch.randn(N, D, generator=gen) + 0.5 * f, dim=1)
    got = retrieval_ranks(f.to(dev), c.to(dev), cap=cap).cpu().numpy()
    ref = OC.retrieval_ranks(f, c, cap=cap)
    # fp32 GEMM vs fp64: a pair may only swap order when the scores agree to fp32 rounding
    bad = np.nonzero(got != ref)[0]
    assert len(bad) <= max(1, len(ref) // 1000), bad[:10]
    assert np.all(np.abs(got[bad] - ref[bad]) <= 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sharded_rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching.contrastive import info_nce_loss_sharded
        dev = torch.device("cuda:0")
        gen = torch.Generator().manual_seed(9)
        B, D = 1024, 64
        f = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1)
        c = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1)
        m = B // world
        fl = f[rank * m:(rank + 1) * m].to(dev).requires_grad_(True)
        cl = c[rank * m:(rank + 1) * m].to(dev).requires_grad_(True)
        loss = info_nce_loss_sharded(fl, cl, 0.07)
        loss.backward()
        rl, rdf, rdc = OC.info_nce(f.double(), c.double(), 0.07)
        e = (abs(float(loss) - float(rl)) / abs(float(rl)),
             normwise(fl.grad.cpu().numpy(), rdf[rank * m:(rank + 1) * m].numpy()),
             normwise(cl.grad.cpu().numpy(), rdc[rank * m:(rank + 1) * m].numpy()))
        q.put((rank, max(e)))
    except Exception as ex:
        q.put((rank, repr(ex)))
        raise
    finally:
        dist.destroy_process_group()


def test_info_nce_sharded_two_ranks():
    _dev()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sharded_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=120)
    for rank, err in res:
        assert isinstance(err, float) and err < TOL, (rank, err)


def _sharded_cfg5_rank(rank, world, port, q, N, D):
    """BASELINE cfg 5 sharded across processes: rank r owns firm / CEO rows
    [r*m, (r+1)*m) and runs info_nce_loss_sharded forward + backward -- the
    all-gather of C (N x D fp32), the MAX all-reduce of the norms, the column
    sum and loss all-reduces, and the dC reduction (gloo: all-reduce + slice)
    at the production shape."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ceo_firm_matching.contrastive import info_nce_loss_sharded
        dev = torch.device("cuda:0")
        gen = torch.Generator().manual_seed(11)
        f = torch.nn.functional.normalize(torch.randn(N, D, generator=gen), dim=1)
        c = torch.nn.functional.normalize(torch.randn(N, D, generator=gen), dim=1)
        m = N // world
        fl = f[rank * m:(rank + 1) * m].to(dev).requires_grad_(True)
        cl = c[rank * m:(rank + 1) * m].to(dev).requires_grad_(True)
        del f, c
        loss = info_nce_loss_sharded(fl, cl, 0.07)
        loss.backward()
        torch.cuda.synchronize()
        q.put((rank, float(loss.detach()), fl.grad.cpu().numpy(), cl.grad.cpu().numpy()))
    except Exception as ex:
        q.put((rank, repr(ex), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_info_nce_sharded_eight_processes_cfg5():
    """cfg 5 at its production shape across 8 processes (sharing the test
    box's GPU, gloo collectives): N = 100k firms x 100k CEOs, D = 256, every
    rank's loss, dF shard and dC shard vs the fp64 chunked reference of the
    whole matrix at 1e-5 (contrastive.py:102-138)."""
    dev = _dev()
    world, N, D = 8, 100_000, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sharded_cfg5_rank, args=(r, world, port, q, N, D)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=900) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=120)
    for rank, loss, _, _ in res:
        assert isinstance(loss, float), (rank, loss)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    gen = torch.Generator().manual_seed(11)
    f = torch.nn.functional.normalize(torch.randn(N, D, generator=gen), dim=1).to(dev)
    c = torch.nn.functional.normalize(torch.randn(N, D, generator=gen), dim=1).to(dev)
    rl, rdf, rdc = _info_nce_fp64_chunked(f, c, 0.07)
    m = N // world
    df = torch.from_numpy(np.concatenate([r[2] for r in res])).to(dev)
    dc = torch.from_numpy(np.concatenate([r[3] for r in res])).to(dev)
    for rank, loss, _, _ in res:  # every rank holds the global loss
        assert abs(loss - rl) <= TOL * abs(rl), (rank, loss, rl)
    for got, ref in ((df, rdf), (dc, rdc)):
        assert got.shape == ref.shape == (world * m, D)
        err = float((got.double() - ref).abs().max() / ref.abs().max())
        assert err < TOL, err


# ---------------------------------------------------------------------------
# semi_hard_negative_mining (contrastive.py:141-192) on tt_triplet_*
# ---------------------------------------------------------------------------
AMBIG = 2e-6  # rows whose candidates sit this close to a selection boundary may
              # legitimately select differently under another summation order


def _triplet(f, c, margin=0.2):
    from ceo_firm_matching.contrastive import semi_hard_mining
    f = f.clone().requires_grad_(True)
    c = c.clone().requires_grad_(True)
    loss, hardest, row_loss = semi_hard_mining(f, c, margin)
    loss.backward()
    return loss.detach(), hardest, row_loss, f.grad, c.grad


def _grads_given(f, c, j, act):
    """closed-form grads (oracle algebra) for a given selection"""
    B = f.shape[0]
    w = act.double() / B
    df = w[:, None] * (c[j] - c)
    dc = -w[:, None] * f
    dc.index_add_(0, j, w[:, None] * f)
    return df, dc


def _check_triplet(f, c, got, margin=0.2, ref_loss=None):
    loss, hardest, row_loss, df, dc = got
    f64, c64 = f.double(), c.double()
    o = OC.semi_hard(f64, c64, margin)
    ok = (o["slack"] > AMBIG)
    hj = hardest.cpu().long()
    rl = row_loss.cpu().double()
    # unambiguous rows select exactly what the reference selects
    assert torch.equal(hj[ok], o["hardest"][ok]), int((hj[ok] != o["hardest"][ok]).sum())
    assert float((rl[ok] - o["row_loss"][ok]).abs().max()) <= 1e-5
    assert int((~ok).sum()) <= max(2, f.shape[0] // 10)  # near-ties grow with B at small D
    expect = torch.where(ok, o["row_loss"], rl).mean()
    assert abs(float(loss) - float(expect)) <= TOL * max(1.0, float(expect))
    if ref_loss is not None and bool(ok.all()):
        assert abs(float(loss) - ref_loss) <= TOL * max(1.0, abs(ref_loss))
    # backward kernel == the closed form for the selection it made
    rdf, rdc = _grads_given(f64, c64, hj, rl > 0)
    assert normwise(df.cpu().numpy(), rdf.numpy()) < TOL
    assert normwise(dc.cpu().numpy(), rdc.numpy()) < TOL


@pytest.mark.parametrize("case", ["b2", "b64", "b256", "corr128", "raw96"])
def test_semi_hard_golden(case):
    dev = _dev()
    g = load_golden("triplet")
    f = torch.from_numpy(g[f"tri/{case}/f"])
    c = torch.from_numpy(g[f"tri/{case}/c"])
    got = _triplet(f.to(dev), c.to(dev))
    _check_triplet(f, c, got, ref_loss=float(g[f"tri/{case}/loss64"]))
    o = OC.semi_hard(f.double(), c.double())
    if bool((o["slack"] > AMBIG).all()):  # then the reference's own autograd grads too
        assert normwise(got[3].cpu().numpy(), g[f"tri/{case}/df64"]) < TOL
        assert normwise(got[4].cpu().numpy(), g[f"tri/{case}/dc64"]) < TOL


def test_semi_hard_b1_is_zero():
    from ceo_firm_matching.contrastive import semi_hard_negative_mining
    dev = _dev()
    x = torch.randn(1, 32, device=dev)
    assert float(semi_hard_negative_mining(x, x)) == 0.0


@pytest.mark.parametrize("B,D,mix", [(1000, 64, 0.5), (4100, 32, 0.5), (517, 36, 0.5), (2048, 30, 0.5),
                                     (3000, 256, 0.0), (700, 128, 2.0)])
def test_semi_hard_ragged_vs_oracle(B, D, mix):
    """Partial tiles, several column blocks, D not a multiple of 4 (padded),
    both selection branches."""
    dev = _dev()
    gen = torch.Generator().manual_seed(B + D)
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1)
    c = torch.nn.functional.normalize(torch.randn(B, D, generator=gen) + mix * f, dim=1)
    got = _triplet(f.to(dev), c.to(dev))
    _check_triplet(f, c, got)


def test_semi_hard_matches_aten_reference_expression():
    """semi_hard_negative_mining on a HIP tensor == the package's ATen
    expression of the reference loop on CPU (same inputs)."""
    from ceo_firm_matching.contrastive import semi_hard_negative_mining
    dev = _dev()
    gen = torch.Generator().manual_seed(9)
    f = torch.nn.functional.normalize(torch.randn(300, 48, generator=gen), dim=1)
    c = torch.nn.functional.normalize(torch.randn(300, 48, generator=gen) + 0.4 * f, dim=1)
    a = semi_hard_negative_mining(f.to(dev), c.to(dev))
    b = semi_hard_negative_mining(f, c)
    assert abs(float(a) - float(b)) <= TOL * max(1.0, float(b))


def test_semi_hard_row_shards_compose():
    """Row shards against all CEO rows (the multi-GPU decomposition, as
    bench.py's cfg-5 leg runs it) reproduce the single-launch mining."""
    from ceo_firm_matching.contrastive import semi_hard_mining, semi_hard_mining_rows
    dev = _dev()
    gen = torch.Generator().manual_seed(21)
    B, D, W = 3000, 64, 4
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=gen), dim=1).to(dev)
    c = torch.nn.functional.normalize(torch.randn(B, D, generator=gen) + 0.5 * f.cpu(), dim=1).to(dev)
    loss, hardest, row_loss = semi_hard_mining(f, c)
    m = B // W
    parts = [semi_hard_mining_rows(f[r * m:(r + 1) * m], c, r * m, 0.2, B) for r in range(W)]
    assert torch.equal(torch.cat([p[1] for p in parts]), hardest)
    assert torch.equal(torch.cat([p[2] for p in parts]), row_loss)
    assert abs(float(sum(p[0] for p in parts)) - float(loss.detach())) <= TOL * float(loss.detach())


def _info_nce_fp64_chunked(f, c, tau, chunk=8192):
    """Symmetric InfoNCE (contrastive.py:102-138) and its gradients in fp64
    on the device, in row chunks (never the whole N x N): a plain torch
    reference for the full cfg-5 size, where the CPU oracle is too slow."""
    f, c = f.double(), c.double()
    n = f.shape[0]
    shift = 1.0 / tau  # unit rows: |S| <= 1 / tau
    rowsum = torch.empty(n, dtype=torch.float64, device=f.device)
    colsum = torch.zeros(n, dtype=torch.float64, device=f.device)
    for i0 in range(0, n, chunk):
        e = torch.exp(f[i0:i0 + chunk] @ c.T / tau - shift)
        rowsum[i0:i0 + chunk] = e.sum(1)
        colsum += e.sum(0)
    diag = (f * c).sum(1) / tau
    lse_r, lse_c = torch.log(rowsum) + shift, torch.log(colsum) + shift
    loss = 0.5 * ((lse_r - diag).mean() + (lse_c - diag).mean())
    df = torch.empty_like(f)
    dc = torch.zeros_like(c)
    for i0 in range(0, n, chunk):
        i1 = min(i0 + chunk, n)
        g = torch.exp(f[i0:i1] @ c.T / tau - shift)
        g *= (1.0 / rowsum[i0:i1])[:, None] + (1.0 / colsum)[None, :]
        df[i0:i1] = g @ c
        dc += g.T @ f[i0:i1]
        del g
    df = df / (2 * n * tau) - c / (n * tau)
    dc = dc / (2 * n * tau) - f / (n * tau)
    return float(loss), df, dc


def test_info_nce_full_cfg5_vs_fp64():
    """BASELINE cfg 5 at its full size (100k firms x 100k CEOs, D = 256, the
    bench's workload): loss and both gradients vs an fp64 device reference,
    1e-5 (loss relative, gradients normwise)."""
    dev = _dev()
    n, d, tau = 100_000, 256, 0.07
    gen = torch.Generator(device=dev).manual_seed(5)
    f = torch.nn.functional.normalize(torch.randn(n, d, device=dev, generator=gen), dim=1)
    c = torch.nn.functional.normalize(torch.randn(n, d, device=dev, generator=gen) + 0.3 * f, dim=1)
    loss, df, dc = _nce(f, c, tau)
    loss = float(loss.detach())
    torch.cuda.empty_cache()  # the similarity workspace (40 GB) before the reference's chunks
    rl, rdf, rdc = _info_nce_fp64_chunked(f, c, tau)
    assert abs(loss - rl) <= TOL * abs(rl), (loss, rl)
    for got, ref in ((df, rdf), (dc, rdc)):
        err = float((got.double() - ref).abs().max() / ref.abs().max())
        assert err < TOL, err


@pytest.mark.parametrize("kind,tau,B,D", [("norm", 0.004, 300, 64), ("norm", 0.005, 1030, 128),
                                         ("raw", 0.07, 517, 36), ("raw", 0.07, 64, 256)])
def test_info_nce_underflow_falls_back_to_robust_pass(kind, tau, B, D):
    """Inputs the shared exponent shift cannot serve (L2-normalised rows at a
    temperature far below 0.03; unnormalised projections, |f| |c| / tau in
    the hundreds): the shared-shift pass reports underflowed sums, and
    info_nce_loss recomputes with exact row / column maxima (tt_nce_maxes,
    tt_nce_forward_lse, tt_nce_loss_lse, tt_nce_backward_lse).  Loss and
    gradients vs the fp64 oracle; logits this large carry fp32 rounding of
    |s| * 2^-24 into every softmax, so the bound is 1e-5 normwise or 10x the
    fp32 oracle's own error, whichever is larger."""
    from ceo_firm_matching.contrastive import _NCE
    dev = _dev()
    gen = torch.Generator().manual_seed(B * 7 + D)
    f = torch.randn(B, D, generator=gen)
    c = torch.randn(B, D, generator=gen) + 0.5 * f
    if kind == "norm":
        f, c = torch.nn.functional.normalize(f, dim=1), torch.nn.functional.normalize(c, dim=1)
    else:
        f, c = 3.0 * f, 3.0 * c
    # the default pass does underflow on these inputs (so the fallback runs)
    fd, cd = f.to(dev).contiguous(), c.to(dev).contiguous()
    h = _NCE(fd, cd, B, B, D, 0, B, tau)
    _, status = h.loss(h.forward(h.norms()))
    assert int(status.item()) > 0
    loss, df, dc = _nce(fd, cd, tau)
    rl, rdf, rdc = OC.info_nce(f.double(), c.double(), tau)
    l32, df32, dc32 = OC.info_nce(f, c, tau)
    lerr = abs(float(loss.detach()) - float(rl))
    assert np.isfinite(float(loss.detach()))
    assert lerr <= max(TOL * abs(float(rl)), 10 * abs(float(l32) - float(rl))), (float(loss), float(rl), float(l32))
    for got, ref, r32 in ((df, rdf, df32), (dc, rdc, dc32)):
        err = normwise(got.cpu().numpy(), ref.numpy())
        err32 = normwise(r32.double().numpy(), ref.numpy())
        assert err <= max(TOL, 10 * err32), (err, err32)


def test_info_nce_float64_inputs_warn_and_return_float64():
    from ceo_firm_matching import contrastive as CT
    dev = _dev()
    gen = torch.Generator().manual_seed(11)
    f = torch.nn.functional.normalize(torch.randn(64, 32, generator=gen, dtype=torch.float64), dim=1)
    c = torch.nn.functional.normalize(torch.randn(64, 32, generator=gen, dtype=torch.float64), dim=1)
    CT._F64_WARNED = False
    with pytest.warns(RuntimeWarning, match="float64"):
        loss, df, dc = _nce(f.to(dev), c.to(dev))
    assert loss.dtype == torch.float64 and df.dtype == torch.float64
    rl, rdf, _ = OC.info_nce(f, c, 0.07)
    assert abs(float(loss.detach()) - float(rl)) <= TOL * abs(float(rl))
    assert normwise(df.cpu().numpy(), rdf.numpy()) < TOL
