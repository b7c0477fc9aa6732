"""CEOFirmMatcher -- the two-tower model, MI355X-native.

Drop-in for the reference ``ceo_firm_matching/model.py:14-89``:
* the same ``nn.Module`` surface: ``CEOFirmMatcher(metadata, config)``,
  ``forward(f_numeric, f_cat, c_numeric, c_cat) -> [B, 1]``, attributes
  ``firm_embeddings``/``ceo_embeddings`` (ModuleList), ``firm_tower``/
  ``ceo_tower`` (indexable ``nn.Sequential``, callable on their own) and
  ``logit_scale``; identical ``state_dict`` keys; modules are created in the
  reference order, so ``torch.manual_seed(s)`` gives identical initial weights.
* On a HIP device the whole forward (embedding gather, both towers, L2
  normalisation, scaled cosine) and its backward run in the fused kernels of
  ``libceo_tt.so`` (one autograd node).  Parameters and BatchNorm buffers are
  re-pointed into one flat fp32 arena (views; ``state_dict``/optimizers keep
  working) laid out as ``tt_param_offsets`` says.
* On CPU tensors the module evaluates the same algorithm with ATen ops (there
  is no HIP kernel to call); this is the reference's own CPU behaviour and is
  never used for a tensor on a HIP device: a missing extension raises.
"""
from __future__ import annotations

import os
import warnings
import weakref
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from . import _native as N
from .config import Config

TOWERS = ("firm", "ceo")


class _Arena:
    """Flat device storage the kernels address (params / BN buffers / counters)."""

    def __init__(self, desc, params, buffers, nbt, views):
        self.desc = desc
        self.params = params
        self.buffers = buffers
        self.nbt = nbt
        self.views = views  # list of (tensor-getter, data_ptr) to validate binding


class CEOFirmMatcher(nn.Module):
    """Two-tower network: firm / CEO encoders + scaled cosine similarity."""

    def __init__(self, metadata: Dict[str, int], config: Config):
        super().__init__()
        large = config.EMBEDDING_DIM_LARGE
        medium = config.EMBEDDING_DIM_MEDIUM
        p = float(getattr(config, "DROPOUT_P", 0.1))
        # construction order == reference (model.py:24-65): same RNG draws
        self.firm_embeddings = nn.ModuleList([nn.Embedding(n, large) for n in metadata['firm_cat_counts']])
        self.ceo_embeddings = nn.ModuleList([nn.Embedding(n, medium) for n in metadata['ceo_cat_counts']])
        firm_in = metadata['n_firm_numeric'] + len(metadata['firm_cat_counts']) * large
        ceo_in = metadata['n_ceo_numeric'] + len(metadata['ceo_cat_counts']) * medium
        self.firm_tower = self._tower(firm_in, config.LATENT_DIM, p)
        self.ceo_tower = self._tower(ceo_in, config.LATENT_DIM, p)
        self.logit_scale = nn.Parameter(torch.ones([]) * np.log(1 / 0.07))

        self._geom = dict(n_num=(int(metadata['n_firm_numeric']), int(metadata['n_ceo_numeric'])),
                          cat_counts=(list(metadata['firm_cat_counts']), list(metadata['ceo_cat_counts'])),
                          emb_dim=(large, medium), latent=int(config.LATENT_DIM))
        self._arena: Optional[_Arena] = None
        self._stream_step = 0
        self._aten_warned = False
        # deterministic reductions (TT_FLAG_DETERMINISTIC): None follows
        # torch.use_deterministic_algorithms / CEO_TT_DETERMINISTIC
        self.deterministic: Optional[bool] = None
        # a FusedTrainer whose last step deferred the late half of its
        # reduction (TT_FLAG_DEFER_LATE): its flush, run before anything reads
        # the parameters (forward, tower_embeddings, state_dict)
        self._pending_flush = None

    def sync_trainer(self):
        """Finish a deferred optimizer step of the training engine, if any.
        engine.FusedTrainer registers its bound ``flush`` here only while a
        late half is pending (a strong reference: a trainer dropped with a
        pending step stays alive until the step is finished here, never losing
        it) and clears it once the late half has run."""
        fn = self._pending_flush
        if fn is not None:
            fn()
            self._pending_flush = None

    def __getstate__(self):
        """copy.deepcopy / pickle / torch.save of the module: finish a pending
        deferred step first, and leave out the engine's handles (the weak
        trainer reference, the ctypes arena descriptor) -- the copy binds its
        own arena on first use on a HIP device."""
        self.sync_trainer()
        state = self.__dict__.copy()
        state["_pending_flush"] = None
        state["_arena"] = None
        return state

    def state_dict(self, *args, **kwargs):
        self.sync_trainer()
        return super().state_dict(*args, **kwargs)

    def is_deterministic(self) -> bool:
        return N.deterministic_default() if self.deterministic is None else bool(self.deterministic)

    @staticmethod
    def _tower(d_in: int, latent: int, p: float) -> nn.Sequential:
        return nn.Sequential(
            nn.Linear(d_in, 64), nn.BatchNorm1d(64), nn.ReLU(), nn.Dropout(p),
            nn.Linear(64, 32), nn.BatchNorm1d(32), nn.ReLU(), nn.Dropout(p),
            nn.Linear(32, latent))

    # ------------------------------------------------------------------ helpers
    def dropout_p(self) -> float:
        ps = {float(t[i].p) for t in (self.firm_tower, self.ceo_tower) for i in (3, 7)}
        if len(ps) != 1:
            raise NotImplementedError("the fused kernels need one dropout probability for all four Dropout layers")
        return ps.pop()

    def bn_config(self):
        bns = [t[i] for t in (self.firm_tower, self.ceo_tower) for i in (1, 5)]
        eps = {float(b.eps) for b in bns}
        mom = {float(b.momentum) for b in bns}
        if len(eps) != 1 or len(mom) != 1 or None in mom:
            raise NotImplementedError("the fused kernels need one BatchNorm eps/momentum")
        return eps.pop(), mom.pop()

    def tt_desc(self) -> N.TTModelDesc:
        g = self._geom
        eps, mom = self.bn_config()
        return N.make_desc(g["n_num"], g["cat_counts"], g["emb_dim"], g["latent"],
                           dropout_p=self.dropout_p(), bn_eps=eps, bn_momentum=mom)

    def _named_slots(self, offs):
        """(name, tensor, float offset) for every parameter in arena order."""
        out = []
        for t, tw in enumerate(TOWERS):
            embs = self.firm_embeddings if t == 0 else self.ceo_embeddings
            for j, e in enumerate(embs):
                out.append((f"{tw}_embeddings.{j}.weight", e.weight, offs[t * N.TT_MAX_CAT + j]))
        for t, tw in enumerate(TOWERS):
            tower = self.firm_tower if t == 0 else self.ceo_tower
            for s, nm in enumerate(N.SLOT_NAMES):
                idx, attr = nm.split(".")
                out.append((f"{tw}_tower.{nm}", getattr(tower[int(idx)], attr),
                            offs[2 * N.TT_MAX_CAT + t * N.TT_SLOTS_PER_TOWER + s]))
        out.append(("logit_scale", self.logit_scale, offs[-1]))
        return out

    def _bn_modules(self):
        return [self.firm_tower[1], self.firm_tower[5], self.ceo_tower[1], self.ceo_tower[5]]

    def bind_arena(self) -> _Arena:
        """Re-point parameters / BN buffers into flat device arenas (idempotent)."""
        a = self._arena
        if a is not None and all(get().data_ptr() == p for get, p in a.views):
            return a
        desc = self.tt_desc()
        dev = self.logit_scale.device
        offs = N.param_offsets(desc)
        n = N.param_count(desc)
        params = torch.empty(n, dtype=torch.float32, device=dev)
        views = []
        for name, prm, off in self._named_slots(offs):
            k = prm.numel()
            v = params[off:off + k].view_as(prm)
            v.copy_(prm.detach())
            prm.data = v
            views.append(((lambda p=prm: p), v.data_ptr()))
        bns = self._bn_modules()
        buffers = torch.empty(2 * (2 * 64 + 2 * 32), dtype=torch.float32, device=dev)
        nbt = torch.empty(4, dtype=torch.int64, device=dev)
        off = 0
        for i, bn in enumerate(bns):
            H = bn.num_features
            for attr in ("running_mean", "running_var"):
                v = buffers[off:off + H]
                v.copy_(getattr(bn, attr).detach().to(torch.float32))
                setattr(bn, attr, v)
                views.append(((lambda b=bn, a_=attr: getattr(b, a_)), v.data_ptr()))
                off += H
            v = nbt[i]
            v.copy_(bn.num_batches_tracked.detach())
            bn.num_batches_tracked = v
            views.append(((lambda b=bn: b.num_batches_tracked), v.data_ptr()))
        self._arena = _Arena(desc, params, buffers, nbt, views)
        return self._arena

    def next_dropout_stream(self):
        """(seed, step) of the counter-RNG stream for one train-mode forward.
        The seed follows torch.cuda's (torch.manual_seed) without a sync and
        without consuming the CPU generator."""
        self._stream_step += 1
        return int(torch.cuda.initial_seed()) & ((1 << 63) - 1), self._stream_step

    # ------------------------------------------------------------------ forward
    def forward(self, f_numeric, f_cat, c_numeric, c_cat):
        self.sync_trainer()
        if f_numeric.device.type == "cuda":
            return _fused_forward(self, f_numeric, f_cat, c_numeric, c_cat)
        return self._aten_forward(f_numeric, f_cat, c_numeric, c_cat)

    def tower_embeddings(self, f_numeric, f_cat, c_numeric, c_cat):
        """(U, V): the raw firm / CEO tower outputs (model.py:69-77, before the
        L2 normalisation) -- the encoder half that contrastive.py:52-72
        get_embeddings builds on.  One fused autograd node on a HIP device."""
        self.sync_trainer()
        if f_numeric.device.type == "cuda":
            return _fused_embeddings(self, f_numeric, f_cat, c_numeric, c_cat)
        f = torch.cat([f_numeric] + [e(f_cat[:, i]) for i, e in enumerate(self.firm_embeddings)], dim=1)
        c = torch.cat([c_numeric] + [e(c_cat[:, i]) for i, e in enumerate(self.ceo_embeddings)], dim=1)
        return self.firm_tower(f), self.ceo_tower(c)

    def _aten_forward(self, f_numeric, f_cat, c_numeric, c_cat):
        """CPU evaluation of model.py:67-89 with ATen ops (no HIP device)."""
        if not self._aten_warned:
            warnings.warn("CEOFirmMatcher on CPU tensors: evaluating with ATen ops; the fused HIP "
                          "kernels run only for tensors on a HIP device", RuntimeWarning, stacklevel=3)
            self._aten_warned = True
        f = torch.cat([f_numeric] + [e(f_cat[:, i]) for i, e in enumerate(self.firm_embeddings)], dim=1)
        c = torch.cat([c_numeric] + [e(c_cat[:, i]) for i, e in enumerate(self.ceo_embeddings)], dim=1)
        u = self.firm_tower(f)
        v = self.ceo_tower(c)
        u = u / u.norm(dim=1, keepdim=True)
        v = v / v.norm(dim=1, keepdim=True)
        return (u * v).sum(dim=1, keepdim=True) * self.logit_scale.exp()


_POISON_WS = bool(os.environ.get("CEO_TT_POISON_WS"))  # diagnostic: NaN-fill workspaces


def _as_f32(x, dev):
    x = x.to(device=dev, dtype=torch.float32)
    return x if x.is_contiguous() else x.contiguous()


def _as_i64(x, dev):
    if x is None:
        return None
    x = x.to(device=dev, dtype=torch.int64)
    return x if x.is_contiguous() else x.contiguous()


class _FusedTwoTower(torch.autograd.Function):
    """One autograd node for the whole CEOFirmMatcher forward (HIP kernels)."""

    @staticmethod
    def forward(ctx, model, f_num, f_cat, c_num, c_cat, *params):
        arena = model._arena
        L = N.lib()
        B = f_num.shape[0]
        train = bool(model.training)
        desc = N.set_deterministic(arena.desc, model.is_deterministic())
        ws_bytes = N.workspace_bytes(desc, max(B, 1))
        ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=f_num.device)
        if _POISON_WS:  # diagnostic: surface reads of workspace the kernels never wrote
            ws.fill_(float("nan"))
        score = torch.empty(B, dtype=torch.float32, device=f_num.device)
        seed, step = model.next_dropout_stream() if train else (0, 0)
        batch = N.make_batch(f_num, f_cat, c_num, c_cat, n_rows=B)
        rc = L.tt_forward(desc, arena.params.data_ptr(), arena.buffers.data_ptr(), arena.nbt.data_ptr(),
                          batch, int(train), seed, step, ws.data_ptr(), ws_bytes, score.data_ptr(),
                          N.stream_ptr(f_num.device))
        N.check(rc, "tt_forward", B, 64)
        ctx.model = model
        ctx.train = train
        ctx.det = model.is_deterministic()
        ctx.seed, ctx.step = seed, step
        ctx.ws, ctx.ws_bytes = ws, ws_bytes
        ctx.n_params = len(params)
        ctx.save_for_backward(f_num, f_cat, c_num, c_cat)
        return score.view(B, 1)

    @staticmethod
    def backward(ctx, dscore):
        # train- or eval-mode backward (eval: BatchNorm as the affine map of the
        # running statistics, no dropout -- what autograd of model.py:67-89
        # gives after model.eval()), with the numeric inputs' gradients when
        # they require grad (run_deep_extensions.py:564-590 integrated gradients)
        f_num, f_cat, c_num, c_cat = ctx.saved_tensors
        model = ctx.model
        arena = model._arena
        B = f_num.shape[0]
        grad = torch.empty_like(arena.params)
        ds = dscore.reshape(-1).to(torch.float32).contiguous()
        dxf, dxc = _input_grad_buffers(ctx, f_num, c_num)
        batch = N.make_batch(f_num, f_cat, c_num, c_cat, n_rows=B)
        N.set_deterministic(arena.desc, ctx.det)
        rc = N.lib().tt_backward_ex(arena.desc, arena.params.data_ptr(), arena.buffers.data_ptr(), batch,
                                    ds.data_ptr(), int(ctx.train), ctx.seed, ctx.step, ctx.ws.data_ptr(),
                                    ctx.ws_bytes, grad.data_ptr(), N.ptr(dxf), N.ptr(dxc),
                                    N.stream_ptr(f_num.device))
        N.check(rc, "tt_backward_ex", B, 64)
        offs = N.param_offsets(arena.desc)
        grads = [grad[off:off + p.numel()].view_as(p) for _, p, off in model._named_slots(offs)]
        return (None, dxf, None, dxc, None, *grads)


class _FusedTowerEmbeddings(torch.autograd.Function):
    """Raw tower outputs (U, V) of both towers as one autograd node
    (tt_embed_forward / tt_embed_backward): the encoder half of the model for
    callers that score embeddings themselves (contrastive.py:52-99)."""

    @staticmethod
    def forward(ctx, model, f_num, f_cat, c_num, c_cat, *params):
        arena = model._arena
        B = f_num.shape[0]
        D = arena.desc.latent
        train = bool(model.training)
        ctx.det = model.is_deterministic()
        N.set_deterministic(arena.desc, ctx.det)
        ws_bytes = N.workspace_bytes(arena.desc, max(B, 1))
        ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=f_num.device)
        if _POISON_WS:
            ws.fill_(float("nan"))
        emb = torch.empty(2, B, D, dtype=torch.float32, device=f_num.device)
        seed, step = model.next_dropout_stream() if train else (0, 0)
        batch = N.make_batch(f_num, f_cat, c_num, c_cat, n_rows=B)
        rc = N.lib().tt_embed_forward(arena.desc, arena.params.data_ptr(), arena.buffers.data_ptr(),
                                      arena.nbt.data_ptr(), batch, int(train), seed, step, ws.data_ptr(), ws_bytes,
                                      emb.data_ptr(), N.stream_ptr(f_num.device))
        N.check(rc, "tt_embed_forward", B, 64)
        ctx.model, ctx.train, ctx.seed, ctx.step = model, train, seed, step
        ctx.ws, ctx.ws_bytes = ws, ws_bytes
        ctx.save_for_backward(f_num, f_cat, c_num, c_cat)
        return emb[0], emb[1]

    @staticmethod
    def backward(ctx, du, dv):
        f_num, f_cat, c_num, c_cat = ctx.saved_tensors
        model = ctx.model
        arena = model._arena
        B = f_num.shape[0]
        D = arena.desc.latent
        demb = torch.zeros(2, B, D, dtype=torch.float32, device=f_num.device)
        if du is not None:
            demb[0].copy_(du)
        if dv is not None:
            demb[1].copy_(dv)
        grad = torch.empty_like(arena.params)
        dxf, dxc = _input_grad_buffers(ctx, f_num, c_num)
        batch = N.make_batch(f_num, f_cat, c_num, c_cat, n_rows=B)
        N.set_deterministic(arena.desc, ctx.det)
        rc = N.lib().tt_embed_backward_ex(arena.desc, arena.params.data_ptr(), arena.buffers.data_ptr(), batch,
                                          demb.data_ptr(), int(ctx.train), ctx.seed, ctx.step, ctx.ws.data_ptr(),
                                          ctx.ws_bytes, grad.data_ptr(), N.ptr(dxf), N.ptr(dxc),
                                          N.stream_ptr(f_num.device))
        N.check(rc, "tt_embed_backward_ex", B, 64)
        offs = N.param_offsets(arena.desc)
        grads = [grad[off:off + p.numel()].view_as(p) for _, p, off in model._named_slots(offs)]
        return (None, dxf, None, dxc, None, *grads)


def _input_grad_buffers(ctx, f_num, c_num):
    """dL/d(numeric input) outputs of the backward, for the inputs that
    require grad (autograd marks them in ctx.needs_input_grad: forward's
    arguments are (model, f_num, f_cat, c_num, c_cat, *params))."""
    out = []
    for i, x in ((1, f_num), (3, c_num)):
        want = ctx.needs_input_grad[i] and x.dim() == 2 and x.shape[1] > 0
        out.append(torch.empty(x.shape[0], x.shape[1], dtype=torch.float32, device=x.device) if want else None)
    return out




_CHECKED_CODES: Dict[tuple, "weakref.ref"] = {}


def check_category_codes(cat: Optional[torch.Tensor], counts, what: str):
    """Raise IndexError when a categorical code is outside its embedding table,
    as the reference's nn.Embedding does (model.py:69,74); the fused kernels
    would otherwise clamp it.  Only towers with categorical columns pay
    anything: a host tensor is checked on the host (no device sync); a device
    tensor costs one reduction + host read the first time it is seen, then
    never again while its storage and version counter are unchanged (batch-1
    eval loops over one resident tensor do not sync per forward)."""
    if not counts or cat is None or cat.numel() == 0:
        return
    k = len(counts)
    if cat.device.type == "cpu":
        c = cat[:, :k].numpy()
        if bool(((c < 0) | (c >= np.asarray(counts, dtype=np.int64)[None, :])).any()):
            raise IndexError(f"{what}: category code out of range of its embedding table")
        return
    # the cache holds a weak reference to the checked tensor itself: a new
    # tensor that reuses a freed one's storage never matches
    key = (cat.data_ptr(), cat._version, tuple(cat.shape), tuple(cat.stride()), tuple(counts))
    ref = _CHECKED_CODES.get(key)
    if ref is not None and ref() is cat:
        return
    hi = torch.tensor(counts, device=cat.device, dtype=cat.dtype)
    if bool(((cat[:, :k] < 0) | (cat[:, :k] >= hi)).any()):
        raise IndexError(f"{what}: category code out of range of its embedding table")
    if len(_CHECKED_CODES) > 256:
        _CHECKED_CODES.clear()
    _CHECKED_CODES[key] = weakref.ref(cat)


def _fused_inputs(model: CEOFirmMatcher, f_numeric, f_cat, c_numeric, c_cat):
    dev = f_numeric.device
    if model.logit_scale.device != dev:
        raise RuntimeError(f"CEOFirmMatcher parameters are on {model.logit_scale.device}, inputs on {dev}")
    model.bind_arena()
    g = model._geom
    f_cat_in, c_cat_in = f_cat, c_cat
    # host-side code check before the upload (no device sync)
    for cat, counts, what in ((f_cat, g["cat_counts"][0], "firm_cat"), (c_cat, g["cat_counts"][1], "ceo_cat")):
        if cat is not None and cat.device.type == "cpu" and cat.dim() == 2:
            check_category_codes(cat.long(), counts, what)
    f_num = _as_f32(f_numeric, dev)
    c_num = _as_f32(c_numeric, dev)
    f_cat = _as_i64(f_cat, dev)
    c_cat = _as_i64(c_cat, dev)
    for t, (num, cat) in enumerate(((f_num, f_cat), (c_num, c_cat))):
        if num.dim() != 2 or num.shape[1] != g["n_num"][t]:
            raise RuntimeError(f"tower {TOWERS[t]}: expected [B, {g['n_num'][t]}] numeric input, got {tuple(num.shape)}")
        if len(g["cat_counts"][t]) and (cat is None or cat.dim() != 2 or cat.shape[1] < len(g["cat_counts"][t])):
            raise RuntimeError(f"tower {TOWERS[t]}: expected [B, {len(g['cat_counts'][t])}] categorical input")
    if f_num.shape[0] != c_num.shape[0]:
        raise RuntimeError("firm and CEO batches differ in size")
    for raw, cat, counts, what in ((f_cat_in, f_cat, g["cat_counts"][0], "firm_cat"),
                                   (c_cat_in, c_cat, g["cat_counts"][1], "ceo_cat")):
        if raw is None or raw.device.type != "cpu":  # host tensors were checked before the upload
            check_category_codes(cat, counts, what)
    params = [p for _, p, _ in model._named_slots(N.param_offsets(model._arena.desc))]
    return f_num, f_cat, c_num, c_cat, params


def _fused_forward(model: CEOFirmMatcher, f_numeric, f_cat, c_numeric, c_cat):
    f_num, f_cat, c_num, c_cat, params = _fused_inputs(model, f_numeric, f_cat, c_numeric, c_cat)
    return _FusedTwoTower.apply(model, f_num, f_cat, c_num, c_cat, *params)


def _fused_embeddings(model: CEOFirmMatcher, f_numeric, f_cat, c_numeric, c_cat):
    f_num, f_cat, c_num, c_cat, params = _fused_inputs(model, f_numeric, f_cat, c_numeric, c_cat)
    return _FusedTowerEmbeddings.apply(model, f_num, f_cat, c_num, c_cat, *params)
