"""Contrastive scoring on the HIP kernels (reference ``contrastive.py``).

SURVEY 8a rows a18/a19, BASELINE cfg 5:

* ``info_nce_loss(firm_proj, ceo_proj, temperature)`` -- same signature and
  semantics as the reference (contrastive.py:102-138): symmetric InfoNCE over
  the full B x B similarity matrix, ``B <= 1`` returns 0.  On HIP tensors the
  forward and backward run in ``libceo_tt.so`` (tt_nce_*: three fp32 MFMA
  GEMMs, the similarity matrix is never materialised as logits).
* ``info_nce_loss_sharded`` -- the same loss when the B pairs are sharded over
  the ranks of a process group (one GPU each): all-gather of the CEO rows,
  all-reduce of the column sums and of the loss, reduce-scatter of dC.
* ``retrieval_ranks`` / ``compute_retrieval_metrics`` (contrastive.py:275-332):
  rank of the true match among all candidates, recall@1/5/k, MRR, median rank.
* ``semi_hard_negative_mining`` (contrastive.py:141-192): triplet loss with
  semi-hard negatives as one fused similarity GEMM + masked-min kernel
  (tt_triplet_*) instead of a per-row Python loop.
* ``ContrastiveCEOFirmMatcher`` (contrastive.py:21-99): the reference's module
  tree (base CEOFirmMatcher + projector heads); on a HIP device the towers
  run in the fused kernels (tt_embed_forward / tt_embed_backward).
* ``train_contrastive`` (contrastive.py:197-272): combined regression +
  contrastive training loop with the reference's printed lines.

On CPU tensors every function evaluates the reference's ATen expression.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
import torch.optim as optim
from torch.utils.data import DataLoader

from . import _native as N
from .config import Config
from .model import _POISON_WS, CEOFirmMatcher

def _status_bad(status: torch.Tensor) -> bool:
    """Underflowed softmax sums in the shared-shift pass (host read)."""
    return int(status.item()) != 0


def _check_robust(status: torch.Tensor):
    bad = int(status.item())
    if bad:
        raise FloatingPointError(f"info_nce_loss: {bad} non-finite log-sum-exps (inf / nan in the projections)")


_F64_WARNED = False


def _warn_f64(*xs):
    global _F64_WARNED
    if not _F64_WARNED and any(x.dtype == torch.float64 for x in xs):
        import warnings
        warnings.warn("info_nce_loss: float64 projections are scored by the fp32-accurate HIP kernels "
                      "(results and gradients in float64, arithmetic at fp32 accuracy)", RuntimeWarning, stacklevel=3)
        _F64_WARNED = True


def _f32(x: torch.Tensor) -> torch.Tensor:
    x = x.to(torch.float32)
    return x if x.is_contiguous() else x.contiguous()


def _f32_pad4(x: torch.Tensor) -> torch.Tensor:
    """fp32, contiguous, feature dim zero-padded to a multiple of 4 (the
    GEMM core stages 4 consecutive k per load; zero columns add nothing to
    any dot product -- e.g. the default LATENT_DIM 60 gives 30-wide
    projections)."""
    x = _f32(x)
    r = (-x.shape[1]) % 4
    return F.pad(x, (0, r)) if r else x


class _NCE:
    """Host state of one forward (workspace holds E for the backward)."""

    def __init__(self, f, c, m, n, d, row0, batch, tau):
        self.L = N.lib()
        self.f, self.c, self.m, self.n, self.d = f, c, m, n, d
        self.row0, self.batch, self.tau = row0, batch, tau
        self.ws_bytes = int(self.L.tt_nce_workspace_bytes(m, n, d))
        if self.ws_bytes < 0:
            N.check(self.ws_bytes, "tt_nce_workspace_bytes")
        self.ws = torch.empty(self.ws_bytes // 4, dtype=torch.float32, device=f.device)
        if _POISON_WS:
            self.ws.fill_(float("nan"))
        self.st = N.stream_ptr(f.device)

    def norms(self):
        norm2 = torch.empty(2, dtype=torch.float32, device=self.f.device)
        N.check(self.L.tt_nce_norms(self.f.data_ptr(), self.c.data_ptr(), self.m, self.n, self.d,
                                    norm2.data_ptr(), self.st), "tt_nce_norms")
        return norm2

    def forward(self, norm2):
        col_sum = torch.empty(self.n, dtype=torch.float32, device=self.f.device)
        N.check(self.L.tt_nce_forward(self.f.data_ptr(), self.c.data_ptr(), self.m, self.n, self.d, self.row0,
                                      ctypes.c_float(self.tau), norm2.data_ptr(), self.ws.data_ptr(),
                                      self.ws_bytes, col_sum.data_ptr(), self.st), "tt_nce_forward")
        return col_sum

    def loss(self, col_sum):
        """(loss share, status): status counts underflowed softmax sums."""
        loss = torch.zeros(1, dtype=torch.float32, device=self.f.device)
        status = torch.zeros(1, dtype=torch.int32, device=self.f.device)
        N.check(self.L.tt_nce_loss(self.m, self.n, self.d, self.row0, self.batch, ctypes.c_float(self.tau),
                                   self.ws.data_ptr(), self.ws_bytes, col_sum.data_ptr(), loss.data_ptr(),
                                   status.data_ptr(), self.st), "tt_nce_loss")
        return loss, status

    # robust (two-exponent) pass: the fallback when loss() reports underflow
    def maxes(self):
        col_max = torch.empty(self.n, dtype=torch.float32, device=self.f.device)
        N.check(self.L.tt_nce_maxes(self.f.data_ptr(), self.c.data_ptr(), self.m, self.n, self.d, self.row0,
                                    ctypes.c_float(self.tau), self.ws.data_ptr(), self.ws_bytes, col_max.data_ptr(),
                                    self.st), "tt_nce_maxes")
        return col_max

    def forward_lse(self, col_max):
        col_sum = torch.empty(self.n, dtype=torch.float32, device=self.f.device)
        N.check(self.L.tt_nce_forward_lse(self.f.data_ptr(), self.c.data_ptr(), self.m, self.n, self.d, self.row0,
                                          ctypes.c_float(self.tau), col_max.data_ptr(), self.ws.data_ptr(),
                                          self.ws_bytes, col_sum.data_ptr(), self.st), "tt_nce_forward_lse")
        return col_sum

    def loss_lse(self, col_max, col_sum):
        loss = torch.zeros(1, dtype=torch.float32, device=self.f.device)
        status = torch.zeros(1, dtype=torch.int32, device=self.f.device)
        N.check(self.L.tt_nce_loss_lse(self.m, self.n, self.d, self.row0, self.batch, self.ws.data_ptr(),
                                       self.ws_bytes, col_max.data_ptr(), col_sum.data_ptr(), loss.data_ptr(),
                                       status.data_ptr(), self.st), "tt_nce_loss_lse")
        self.robust = True
        return loss, status

    def backward(self):
        df = torch.empty(self.m, self.d, dtype=torch.float32, device=self.f.device)
        dc = torch.empty(self.n, self.d, dtype=torch.float32, device=self.f.device)
        fn = self.L.tt_nce_backward_lse if getattr(self, "robust", False) else self.L.tt_nce_backward
        N.check(fn(self.f.data_ptr(), self.c.data_ptr(), self.m, self.n, self.d, self.row0,
                   self.batch, ctypes.c_float(self.tau), self.ws.data_ptr(), self.ws_bytes,
                   df.data_ptr(), dc.data_ptr(), self.st), "tt_nce_backward")
        return df, dc


class _InfoNCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, c, temperature):
        f32, c32 = _f32_pad4(f), _f32_pad4(c)
        B, d = f32.shape
        h = _NCE(f32, c32, B, B, d, 0, B, float(temperature))
        loss, status = h.loss(h.forward(h.norms()))
        if _status_bad(status):  # shared shift underflowed: exact row / column maxima
            col_max = h.maxes()
            loss, status = h.loss_lse(col_max, h.forward_lse(col_max))
            _check_robust(status)
        ctx.h = h
        ctx.dtypes = (f.dtype, c.dtype)
        ctx.d_in = f.shape[1]
        return loss.reshape(()).to(f.dtype)

    @staticmethod
    def backward(ctx, g):
        df, dc = ctx.h.backward()
        ctx.h = None  # release E
        g = g.to(torch.float32)
        d = ctx.d_in
        return (df[:, :d] * g).to(ctx.dtypes[0]), (dc[:, :d] * g).to(ctx.dtypes[1]), None


def info_nce_loss(firm_proj: torch.Tensor, ceo_proj: torch.Tensor, temperature: float = 0.07) -> torch.Tensor:
    """Symmetric InfoNCE (reference contrastive.py:102-138)."""
    B = firm_proj.size(0)
    if B <= 1:
        return torch.tensor(0.0, device=firm_proj.device)
    if firm_proj.device.type == "cuda":
        if firm_proj.shape != ceo_proj.shape:
            raise ValueError("info_nce_loss: firm_proj and ceo_proj must have the same shape")
        _warn_f64(firm_proj, ceo_proj)
        return _InfoNCEFn.apply(firm_proj, ceo_proj, temperature)
    sim_matrix = torch.mm(firm_proj, ceo_proj.t()) / temperature
    labels = torch.arange(B, device=firm_proj.device)
    return (F.cross_entropy(sim_matrix, labels) + F.cross_entropy(sim_matrix.t(), labels)) / 2


class _ShardedNCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, c, temperature, group):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        f32, c32 = _f32_pad4(f), _f32_pad4(c)
        m, d = f32.shape
        ctx.d_in = f.shape[1]
        if dist.get_backend(group) == "gloo":
            parts = [torch.empty_like(c32) for _ in range(world)]
            dist.all_gather(parts, c32, group=group)
            c_all = torch.cat(parts)
        else:
            c_all = torch.empty(world * m, d, dtype=torch.float32, device=f.device)
            dist.all_gather_into_tensor(c_all, c32, group=group)
        n = world * m
        h = _NCE(f32, c_all, m, n, d, rank * m, n, float(temperature))
        norm2 = h.norms()
        dist.all_reduce(norm2, op=dist.ReduceOp.MAX, group=group)
        col_sum = h.forward(norm2)
        dist.all_reduce(col_sum, group=group)
        loss, status = h.loss(col_sum)
        dist.all_reduce(loss, group=group)
        dist.all_reduce(status, group=group)
        if _status_bad(status):  # every rank takes the robust pass together
            col_max = h.maxes()
            dist.all_reduce(col_max, op=dist.ReduceOp.MAX, group=group)
            col_sum = h.forward_lse(col_max)
            dist.all_reduce(col_sum, group=group)
            loss, status = h.loss_lse(col_max, col_sum)
            dist.all_reduce(loss, group=group)
            dist.all_reduce(status, group=group)
            _check_robust(status)
        ctx.h, ctx.group, ctx.m = h, group, m
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        df, dc_all = ctx.h.backward()
        ctx.h = None
        group, m = ctx.group, ctx.m
        rank = dist.get_rank(group)
        if dist.get_backend(group) == "gloo":  # no reduce_scatter on gloo
            dist.all_reduce(dc_all, group=group)
            dc = dc_all[rank * m:(rank + 1) * m].contiguous()
        else:
            dc = torch.empty(m, dc_all.shape[1], dtype=torch.float32, device=dc_all.device)
            dist.reduce_scatter_tensor(dc, dc_all, group=group)
        g = g.to(torch.float32)
        d = ctx.d_in
        return df[:, :d] * g, dc[:, :d] * g, None, None


def info_nce_loss_sharded(firm_proj: torch.Tensor, ceo_proj: torch.Tensor, temperature: float = 0.07,
                          group=None) -> torch.Tensor:
    """InfoNCE over pairs sharded across the ranks of ``group`` (equal shards:
    rank r holds pairs [r*m, (r+1)*m)).  Returns the global loss on every rank;
    gradients flow to the local shards."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return info_nce_loss(firm_proj, ceo_proj, temperature)
    if firm_proj.device.type != "cuda":
        raise NotImplementedError("info_nce_loss_sharded runs on the HIP kernels (one GPU per rank)")
    return _ShardedNCEFn.apply(firm_proj, ceo_proj, temperature, group)


# --------------------------------------------------------------------------
# triplet loss with semi-hard negative mining
# --------------------------------------------------------------------------
class _SemiHardFn(torch.autograd.Function):
    """One fused similarity GEMM + masked-min epilogue (tt_triplet_forward);
    the backward touches only the mined rows (tt_triplet_backward)."""

    @staticmethod
    def forward(ctx, f, c, margin):
        f32, c32 = _f32_pad4(f), _f32_pad4(c)
        B, d = f32.shape
        L = N.lib()
        wsb = int(L.tt_triplet_workspace_bytes(B, B, d))
        if wsb < 0:
            N.check(wsb, "tt_triplet_workspace_bytes")
        ws = torch.empty(wsb // 4, dtype=torch.float32, device=f.device)
        if _POISON_WS:
            ws.fill_(float("nan"))
        hardest = torch.empty(B, dtype=torch.int32, device=f.device)
        row_loss = torch.empty(B, dtype=torch.float32, device=f.device)
        loss = torch.zeros(1, dtype=torch.float32, device=f.device)
        st = N.stream_ptr(f.device)
        N.check(L.tt_triplet_forward(f32.data_ptr(), c32.data_ptr(), B, B, d, 0, ctypes.c_float(margin), B,
                                     ws.data_ptr(), wsb, hardest.data_ptr(), row_loss.data_ptr(),
                                     loss.data_ptr(), st), "tt_triplet_forward")
        ctx.save_for_backward(f32, c32, hardest, row_loss)
        ctx.meta = (f.dtype, c.dtype, f.shape[1])
        ctx.mark_non_differentiable(hardest, row_loss)
        return loss.reshape(()).to(f.dtype), hardest, row_loss

    @staticmethod
    def backward(ctx, g, _gh, _gr):
        f32, c32, hardest, row_loss = ctx.saved_tensors
        B, d = f32.shape
        g = g.to(torch.float32).reshape(1).contiguous()
        df = torch.empty_like(f32)
        dc = torch.empty_like(c32)
        N.check(N.lib().tt_triplet_backward(f32.data_ptr(), c32.data_ptr(), B, B, d, 0, B, hardest.data_ptr(),
                                            row_loss.data_ptr(), g.data_ptr(), df.data_ptr(), dc.data_ptr(),
                                            N.stream_ptr(f32.device)), "tt_triplet_backward")
        fd, cd, d_in = ctx.meta
        return df[:, :d_in].to(fd), dc[:, :d_in].to(cd), None


def semi_hard_mining_rows(f: torch.Tensor, c: torch.Tensor, row0: int = 0, margin: float = 0.2,
                          batch: Optional[int] = None):
    """Forward mining for a row shard (no autograd): firm rows f [m, D] are
    global rows row0.., ``c`` holds every CEO row [n, D].  Returns this
    shard's loss share (sum of its row losses / batch), the hardest column
    and the loss of each row."""
    m, n = f.shape[0], c.shape[0]
    if row0 < 0 or row0 + m > n:
        raise ValueError("semi_hard_mining_rows: firm rows must map onto ceo rows row0..row0+m")
    f32, c32 = _f32_pad4(f), _f32_pad4(c)
    d = f32.shape[1]
    L = N.lib()
    wsb = int(L.tt_triplet_workspace_bytes(m, n, d))
    if wsb < 0:
        N.check(wsb, "tt_triplet_workspace_bytes")
    ws = torch.empty(wsb // 4, dtype=torch.float32, device=f.device)
    hardest = torch.empty(m, dtype=torch.int32, device=f.device)
    row_loss = torch.empty(m, dtype=torch.float32, device=f.device)
    loss = torch.zeros(1, dtype=torch.float32, device=f.device)
    N.check(L.tt_triplet_forward(f32.data_ptr(), c32.data_ptr(), m, n, d, int(row0), ctypes.c_float(margin),
                                 int(batch if batch is not None else n), ws.data_ptr(), wsb, hardest.data_ptr(),
                                 row_loss.data_ptr(), loss.data_ptr(), N.stream_ptr(f.device)), "tt_triplet_forward")
    return loss.reshape(()), hardest, row_loss


def semi_hard_mining(firm_proj: torch.Tensor, ceo_proj: torch.Tensor, margin: float = 0.2):
    """(loss, hardest column per row, per-row loss) on the HIP kernels."""
    if firm_proj.device.type != "cuda":
        raise NotImplementedError("semi_hard_mining runs on the HIP kernels")
    if firm_proj.shape != ceo_proj.shape or firm_proj.dim() != 2:
        raise ValueError("semi_hard_negative_mining: firm_proj and ceo_proj must be [B, D] of the same shape")
    return _SemiHardFn.apply(firm_proj, ceo_proj, float(margin))


def semi_hard_negative_mining(firm_proj: torch.Tensor, ceo_proj: torch.Tensor, margin: float = 0.2) -> torch.Tensor:
    """Triplet loss with semi-hard negative mining (reference
    contrastive.py:141-192).  dist = 1 - F C^T; per anchor firm i the
    smallest negative distance in (pos_i, pos_i + margin), else the smallest
    negative overall; loss = mean_i relu(pos_i - hardest_i + margin).
    On HIP tensors: one fused GEMM + masked-min kernel instead of the
    reference's per-row Python loop (ties resolve to the lowest column)."""
    B = firm_proj.size(0)
    if B <= 1:
        return torch.tensor(0.0, device=firm_proj.device)
    if firm_proj.device.type == "cuda":
        return semi_hard_mining(firm_proj, ceo_proj, margin)[0]
    dist_matrix = 1 - torch.mm(firm_proj, ceo_proj.t())
    pos = torch.diagonal(dist_matrix)
    eye = torch.eye(B, dtype=torch.bool, device=firm_proj.device)
    neg = dist_matrix.masked_fill(eye, float("inf"))
    semi = (neg > pos[:, None]) & (neg < (pos + margin)[:, None])
    semi_min = neg.masked_fill(~semi, float("inf")).min(dim=1).values
    hardest = torch.where(semi.any(dim=1), semi_min, neg.min(dim=1).values)
    return F.relu(pos - hardest + margin).mean()


# --------------------------------------------------------------------------
# retrieval
# --------------------------------------------------------------------------
def retrieval_ranks_rows(f: torch.Tensor, c: torch.Tensor, row0: int = 0) -> torch.Tensor:
    """1-based rank of the true match (ceo row row0 + i) of each firm row i
    among all rows of ``c`` (a row shard of firms against every CEO)."""
    m, n = f.shape[0], c.shape[0]
    if row0 < 0 or row0 + m > n:
        raise ValueError("retrieval_ranks_rows: firm rows must map onto ceo rows row0..row0+m")
    if f.device.type != "cuda":
        sim = f.double() @ c.double().t()
        idx = torch.arange(m)
        d = sim[idx, row0 + idx]
        gt = sim > d[:, None]
        gt[idx, row0 + idx] = False
        return gt.sum(dim=1).to(torch.int32) + 1
    f32, c32 = _f32_pad4(f), _f32_pad4(c)
    L = N.lib()
    wsb = int(L.tt_rank_workspace_bytes(m))
    if wsb < 0:
        N.check(wsb, "tt_rank_workspace_bytes")
    ws = torch.empty(wsb // 4, dtype=torch.float32, device=f.device)
    ranks = torch.empty(m, dtype=torch.int32, device=f.device)
    N.check(L.tt_retrieval_ranks(f32.data_ptr(), c32.data_ptr(), m, n, f32.shape[1], row0, ws.data_ptr(), wsb,
                                 ranks.data_ptr(), N.stream_ptr(f.device)), "tt_retrieval_ranks")
    return ranks


def retrieval_ranks(firm_emb: torch.Tensor, ceo_emb: torch.Tensor, cap: Optional[int] = 5000) -> torch.Tensor:
    """Ranks over the first N = min(rows, cap) pairs, as the reference
    (contrastive.py:306-322); ``cap=None`` ranks all pairs."""
    N_ = firm_emb.size(0) if cap is None else min(firm_emb.size(0), cap)
    return retrieval_ranks_rows(firm_emb[:N_], ceo_emb[:N_], 0)


def metrics_from_ranks(ranks: torch.Tensor, top_k: int = 10) -> Dict[str, float]:
    r = ranks.detach().cpu().numpy().astype(np.float64)
    return {
        'recall@1': float(np.mean(r <= 1)),
        'recall@5': float(np.mean(r <= 5)),
        'recall@10': float(np.mean(r <= top_k)),
        'MRR': float(np.mean(1.0 / r)),
        'median_rank': float(np.median(r)),
    }


def compute_retrieval_metrics(model, data_dict: Dict, config: Config, top_k: int = 10,
                              cap: Optional[int] = 5000) -> Dict[str, float]:
    """Reference contrastive.py:275-332 (``cap=None``: no 5000-row cap)."""
    model.eval()
    with torch.no_grad():
        dev = config.DEVICE
        fe, ce = model.get_embeddings(data_dict['firm_numeric'].to(dev), data_dict['firm_cat'].to(dev),
                                      data_dict['ceo_numeric'].to(dev), data_dict['ceo_cat'].to(dev))
        ranks = retrieval_ranks(fe, ce, cap=cap)
    return metrics_from_ranks(ranks, top_k)


# --------------------------------------------------------------------------
# module tree of the reference (contrastive.py:21-99)
# --------------------------------------------------------------------------
class ContrastiveCEOFirmMatcher(nn.Module):
    def __init__(self, metadata: Dict[str, int], config: Config):
        super().__init__()
        self.base_model = CEOFirmMatcher(metadata, config)
        self.config = config
        D = config.LATENT_DIM
        self.firm_projector = nn.Sequential(nn.Linear(D, D), nn.ReLU(), nn.Linear(D, D // 2))
        self.ceo_projector = nn.Sequential(nn.Linear(D, D), nn.ReLU(), nn.Linear(D, D // 2))

    def get_embeddings(self, f_numeric, f_cat, c_numeric, c_cat):
        """L2-normalised tower outputs (contrastive.py:52-72); the towers run
        in the fused HIP kernels on a HIP device (tt_embed_forward)."""
        u, v = self.base_model.tower_embeddings(f_numeric, f_cat, c_numeric, c_cat)
        return F.normalize(u, dim=1), F.normalize(v, dim=1)

    def forward(self, f_numeric, f_cat, c_numeric, c_cat):
        u, v = self.get_embeddings(f_numeric, f_cat, c_numeric, c_cat)
        match_score = (u * v).sum(dim=1, keepdim=True) * self.base_model.logit_scale.exp()
        return match_score, F.normalize(self.firm_projector(u), dim=1), F.normalize(self.ceo_projector(v), dim=1)


# --------------------------------------------------------------------------
# combined regression + contrastive training (contrastive.py:197-272)
# --------------------------------------------------------------------------
def train_contrastive(train_loader: DataLoader, val_loader: DataLoader, metadata: Dict[str, int], config: Config,
                      contrastive_weight: float = 0.3, temperature: float = 0.07,
                      use_triplet: bool = False) -> ContrastiveCEOFirmMatcher:
    """Train the two-tower model on (1 - a) * weighted MSE + a * InfoNCE (or
    semi-hard triplet) loss -- reference contrastive.py:197-272, same
    signature, same prints, same batch order (the loader is iterated as is).

    On a HIP device the towers run forward and backward in the fused kernels
    (one autograd node for both encoders), InfoNCE / triplet mining in the
    similarity kernels; the projector heads, the match score and Adam are
    ATen ops.  Loss totals stay on the device until an epoch is printed
    (the reference syncs three times per step with ``.item()``)."""
    model = ContrastiveCEOFirmMatcher(metadata, config).to(config.DEVICE)
    optimizer = optim.Adam(model.parameters(), lr=config.LEARNING_RATE)

    print(f"Training Contrastive Two-Tower on {config.DEVICE}")
    print(f"  Contrastive weight: {contrastive_weight}")
    print(f"  Temperature: {temperature}")
    print(f"  Loss type: {'Triplet' if use_triplet else 'InfoNCE'}")

    dev = torch.device(config.DEVICE)
    for epoch in range(config.EPOCHS):
        model.train()
        totals = torch.zeros(3, dtype=torch.float64, device=dev)  # loss, mse, cl
        n_batches = 0
        for batch in train_loader:
            batch = {k: v.to(dev) for k, v in batch.items()}
            optimizer.zero_grad()
            match_score, firm_proj, ceo_proj = model(batch['firm_numeric'], batch['firm_cat'],
                                                     batch['ceo_numeric'], batch['ceo_cat'])
            mse_loss = (batch['weights'] * (match_score - batch['target']) ** 2).mean()
            if use_triplet:
                cl_loss = semi_hard_negative_mining(firm_proj, ceo_proj)
            else:
                cl_loss = info_nce_loss(firm_proj, ceo_proj, temperature)
            loss = (1 - contrastive_weight) * mse_loss + contrastive_weight * cl_loss
            loss.backward()
            optimizer.step()
            totals += torch.stack([loss.detach(), mse_loss.detach(), cl_loss.detach().to(mse_loss.dtype)]).double()
            n_batches += 1
        if epoch % 5 == 0:
            avg_loss, avg_mse, avg_cl = (totals / max(n_batches, 1)).tolist()
            print(f"  Epoch {epoch}: Loss={avg_loss:.4f} (MSE={avg_mse:.4f}, CL={avg_cl:.4f})")
    return model
