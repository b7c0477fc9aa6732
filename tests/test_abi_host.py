"""Host-side checks of the C-ABI boundary (no GPU needed).

* libceo_tt.so loads and exports every entry point include/ceo_tt.h declares;
* the ABI version and the constants of the header match the ctypes mirror;
* the parameter arena layout (tt_param_offsets) is the module's parameter
  set, 16-byte aligned and non-overlapping, for the golden geometries;
* argument errors are reported on the host before anything is enqueued
  (null pointers, unsupported shapes, short workspace, train-mode B < 2 ->
  the same ValueError text as torch's BatchNorm).
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden, meta_of
from ceo_firm_matching import CEOFirmMatcher, Config
from ceo_firm_matching import _native as N

HEADER = os.path.join(ROOT, "include", "ceo_tt.h")


def header_text():
    with open(HEADER) as f:
        return f.read()


def header_functions():
    txt = re.sub(r"/\*.*?\*/", "", header_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|void)\s+(tt_\w+)\s*\(", txt, flags=re.M)))


def header_define(name):
    m = re.search(rf"#define\s+{name}\s+\(?(-?\d+)\)?", header_text())
    assert m, name
    return int(m.group(1))


def test_library_exports_every_header_symbol():
    L = N.lib()
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(L, n), f"libceo_tt.so does not export {n}"
    assert set(N.EXPORTED) <= set(names)


def test_header_constants_match_binding():
    assert N.lib().tt_abi_version() == header_define("TT_ABI_VERSION") == N.TT_ABI_VERSION
    assert header_define("TT_MAX_CAT") == N.TT_MAX_CAT
    for k in ("TT_OK", "TT_ERR_ARG", "TT_ERR_BATCH_TOO_SMALL", "TT_ERR_UNSUPPORTED", "TT_ERR_WORKSPACE"):
        assert header_define(k) == getattr(N, k), k


def test_struct_sizes_match_header_layout():
    # tt_model_desc: 7 int32 + 32 int32 + 3 floats + flags; tt_batch: 11 8-byte fields
    assert ctypes.sizeof(N.TTModelDesc) == 4 * (7 + 2 * N.TT_MAX_CAT + 3 + 1)
    assert header_define("TT_FLAG_DETERMINISTIC") == N.TT_FLAG_DETERMINISTIC
    assert ctypes.sizeof(N.TTBatch) == 8 * 15
    assert ctypes.sizeof(N.TTAdamHP) == 32


def _model(case):
    g = load_golden(case)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DEVICE = torch.device("cpu")
    torch.manual_seed(0)
    return CEOFirmMatcher(meta_of(g), cfg)


@pytest.mark.parametrize("case", ["meta_test", "cfg2", "cfg3"])
def test_param_arena_layout(case):
    m = _model(case)
    desc = m.tt_desc()
    n = N.param_count(desc)
    offs = N.param_offsets(desc)
    slots = m._named_slots(offs)
    names = [s[0] for s in slots]
    assert sorted(names) == sorted(k for k, _ in m.named_parameters())
    spans = sorted((off, off + p.numel(), name) for name, p, off in slots)
    for (a0, a1, na), (b0, b1, nb) in zip(spans, spans[1:]):
        assert a1 <= b0, f"{na} overlaps {nb}"
    assert all(off % 4 == 0 for off, _, _ in spans), "parameters must start 16-byte aligned"
    assert spans[-1][1] <= n < spans[-1][1] + 4 * len(spans)
    # the arena binding keeps every value and is seen through state_dict
    before = {k: v.clone() for k, v in m.state_dict().items()}
    arena = m.bind_arena()
    assert arena.params.numel() == n
    after = m.state_dict()
    assert before.keys() == after.keys()
    for k in before:
        assert torch.equal(before[k], after[k]), k
    for name, p, off in m._named_slots(offs):
        assert p.data_ptr() == arena.params.data_ptr() + 4 * off, name
    assert N.lib().tt_buffer_count(ctypes.byref(desc)) == arena.buffers.numel()


def test_workspace_bytes_grow_with_batch():
    desc = _model("cfg3").tt_desc()
    w = [N.workspace_bytes(desc, b) for b in (1, 128, 4096, 16384, 65536)]
    assert all(x > 0 and x % 256 == 0 for x in w)
    assert w == sorted(w) and w[-1] > w[0]
    with pytest.raises(ValueError):
        N.workspace_bytes(desc, 0)


def test_step_plan_tiles():
    """tt_step_plan (host only): the folded five-kernel step from B = 4096
    (numeric-only towers), k_top_pair from B = 4096 on 32-row blocks below
    8192, the six-kernel step below 4096 (and for towers with embeddings),
    and the other tower kernels' row tiles (32 below the folded path when the
    build enables it: TT_FWD32_MAX_B / TT_BWD32_MAX_B)."""
    desc = _model("cfg3").tt_desc()
    big = N.step_plan(desc, 16384)
    assert big["folded_bn0_backward"] and big["kernels"] == 5 and big["mid_rows"] == 128
    assert big["top_pair"] and big["train_top_rows"] == 64 and big["fwd_rows"] == 64
    mid = N.step_plan(desc, 6000)
    assert mid["folded_bn0_backward"] and mid["kernels"] == 5 and mid["mid_rows"] == 128
    assert mid["top_pair"] and mid["train_top_rows"] == 32
    low = N.step_plan(desc, 3000)
    assert not low["folded_bn0_backward"] and low["kernels"] == 6 and not low["top_pair"]
    assert low["fwd_rows"] in (32, 64) and low["mid_rows"] in (32, 64)
    emb = N.step_plan(_model("meta_test").tt_desc(), 6000)  # embeddings: never folded
    assert not emb["folded_bn0_backward"] and emb["kernels"] == 6 and emb["train_top_rows"] == 32
    small = N.step_plan(desc, 1000)
    assert not small["top_pair"] and small["train_top_rows"] == small["top_rows"] == 64
    # the workspace covers the doubled tile count of the 32-row kernels
    assert N.workspace_bytes(desc, 8191) >= N.workspace_bytes(desc, 4096)


def _fake(n=1 << 20):
    """A host buffer standing in for device pointers: argument errors are
    decided before anything dereferences or enqueues."""
    return np.zeros(n, dtype=np.float32)


def _batch(desc, n_rows):
    buf = _fake()
    b = N.TTBatch()
    for t in range(2):
        b.num[t] = buf.ctypes.data
        b.num_ld[t] = desc.n_num[t]
        if desc.n_cat[t]:
            b.cat[t] = buf.ctypes.data
            b.cat_ld[t] = desc.n_cat[t]
    b.target = buf.ctypes.data
    b.weight = buf.ctypes.data
    b.n_rows = n_rows
    return b, buf


def test_host_argument_errors():
    L = N.lib()
    m = _model("meta_test")
    desc = m.tt_desc()
    b, keep = _batch(desc, 64)
    pbuf = _fake()
    p = pbuf.ctypes.data
    ws_ok = N.workspace_bytes(desc, 64)
    fwd = lambda d, bb, train, ws_bytes, params=p: L.tt_forward(  # noqa: E731
        ctypes.byref(d), params, p, p, ctypes.byref(bb), train, 0, 1, p, ws_bytes, p, None)
    # null parameter pointer
    assert fwd(desc, b, 0, ws_ok, params=None) == N.TT_ERR_ARG
    # workspace too small
    assert fwd(desc, b, 0, ws_ok - 4) == N.TT_ERR_WORKSPACE
    # train-mode batch of one row (BatchNorm), both for forward and the fused step
    b1, keep1 = _batch(desc, 1)
    assert fwd(desc, b1, 1, ws_ok) == N.TT_ERR_BATCH_TOO_SMALL
    hp = N.adam_hp(4e-4)
    rc = L.tt_train_step(ctypes.byref(desc), p, p, p, ctypes.byref(b1), ctypes.byref(hp), 0, p, p, ws_ok,
                         p, p, p, 1, None)
    assert rc == N.TT_ERR_BATCH_TOO_SMALL
    with pytest.raises(ValueError, match="Expected more than 1 value per channel when training"):
        N.check(rc, "tt_train_step", 1, 64)
    # unsupported geometry: LATENT_DIM beyond the fused top kernel
    big = N.make_desc(desc.n_num, [[], []], desc.emb_dim, 1024)  # LATENT <= 512 (generic top, tt_topgen.hip)
    bb, keep2 = _batch(big, 64)
    assert fwd(big, bb, 0, 1 << 40) == N.TT_ERR_UNSUPPORTED
    # invalid descriptor (dropout p = 1, more categorical columns than supported)
    bad = N.make_desc(desc.n_num, [[], []], desc.emb_dim, 64, dropout_p=1.0)
    assert L.tt_param_count(ctypes.byref(bad)) == N.TT_ERR_ARG
    with pytest.raises(NotImplementedError):
        N.make_desc((1, 1), [[2] * 17, []], (4, 4), 8)
    # cosine kernels: null pointers
    assert L.tt_cosine_forward(None, p, 8, 16, p, p, None) == N.TT_ERR_ARG
    assert L.tt_adam_apply(p, p, p, p, 10, ctypes.byref(hp), None, 0, None) == N.TT_ERR_ARG
    # tt_train_steps cannot carry a deferred chain (the host's pending record
    # is needed between steps): refused before anything is enqueued
    cyc, keep3 = _batch(desc, 64)
    cyc.cycle = 4
    for fl in (N.TT_FLAG_DEFER_LATE, N.TT_FLAG_LATE_PENDING):
        desc.flags |= fl
        rc = L.tt_train_steps(ctypes.byref(desc), p, p, p, ctypes.byref(cyc), ctypes.byref(hp), 0, p, p, ws_ok,
                              p, p, p, 3, None)
        desc.flags &= ~fl
        assert rc == N.TT_ERR_UNSUPPORTED, fl


def test_product_path_refuses_without_extension(monkeypatch):
    """A missing extension fails loudly (no CPU fallback on a HIP device)."""
    monkeypatch.setattr(N, "_LIB", None)
    monkeypatch.setattr(N, "LIB_PATH", os.path.join(ROOT, "does-not-exist", "libceo_tt.so"))
    with pytest.raises(N.NativeLibraryError, match="HIP extension not built"):
        N.lib()


def test_contrastive_host_argument_errors():
    L = N.lib()
    buf = _fake()
    p = buf.ctypes.data
    assert L.tt_nce_workspace_bytes(0, 10, 16) == N.TT_ERR_ARG
    assert L.tt_nce_workspace_bytes(10, 10, 6) == N.TT_ERR_ARG  # d % 4
    ws = L.tt_nce_workspace_bytes(100, 100, 32)
    assert ws >= 4 * 100 * 100
    # 100k x 100k at D=256: E (40 GB) dominates; fits one MI355X (288 GB)
    big = L.tt_nce_workspace_bytes(100_000, 100_000, 256)
    assert 4 * 100_000 ** 2 <= big < 45 * 2 ** 30
    # row shard outside the CEO range / short workspace / bad temperature
    assert L.tt_nce_forward(p, p, 60, 100, 32, 50, ctypes.c_float(0.07), p, p, ws, p, None) == N.TT_ERR_ARG
    assert L.tt_nce_forward(p, p, 100, 100, 32, 0, ctypes.c_float(0.07), p, p, ws - 4, p, None) == N.TT_ERR_WORKSPACE
    assert L.tt_nce_forward(p, p, 100, 100, 32, 0, ctypes.c_float(0.0), p, p, ws, p, None) == N.TT_ERR_ARG
    assert L.tt_nce_loss(100, 100, 32, 0, 1, ctypes.c_float(0.07), p, ws, p, p, None, None) == N.TT_ERR_ARG
    assert L.tt_nce_backward(p, None, 100, 100, 32, 0, 100, ctypes.c_float(0.07), p, ws, p, p, None) == N.TT_ERR_ARG
    assert L.tt_rank_workspace_bytes(0) == N.TT_ERR_ARG
    rb = L.tt_rank_workspace_bytes(100)
    assert L.tt_retrieval_ranks(p, p, 100, 100, 32, 0, p, rb - 4, p, None) == N.TT_ERR_WORKSPACE


def test_contrastive_cpu_path_matches_oracle():
    """CPU tensors evaluate the reference expression (no HIP device)."""
    from oracle import contrastive as OC
    from ceo_firm_matching.contrastive import info_nce_loss, metrics_from_ranks, retrieval_ranks
    g = load_golden("contrastive")
    f = torch.from_numpy(g["nce/b64/f"])
    c = torch.from_numpy(g["nce/b64/c"])
    assert abs(float(info_nce_loss(f, c)) - float(g["nce/b64/loss"])) < 1e-5
    assert float(info_nce_loss(f[:1], c[:1])) == 0.0
    fe = torch.from_numpy(g["ret/firm_emb"])
    ce = torch.from_numpy(g["ret/ceo_emb"])
    got = metrics_from_ranks(retrieval_ranks(fe, ce))
    assert got == OC.retrieval_metrics(OC.retrieval_ranks(fe, ce))


def test_embedding_mining_exchange_host_argument_errors():
    """tt_embed_*, tt_triplet_*, tt_ar_*: argument errors decided on the host,
    before any HIP call (fake host pointers stand in for device memory)."""
    L = N.lib()
    m = _model("meta_test")
    desc = m.tt_desc()
    b, keep = _batch(desc, 64)
    buf = _fake()
    p = buf.ctypes.data
    ws_ok = N.workspace_bytes(desc, 64)
    # embeddings: missing output / upstream gradient, short workspace, B = 1 in train mode
    assert L.tt_embed_forward(ctypes.byref(desc), p, p, p, ctypes.byref(b), 1, 0, 1, p, ws_ok, None, None) \
        == N.TT_ERR_ARG
    assert L.tt_embed_forward(ctypes.byref(desc), p, p, p, ctypes.byref(b), 1, 0, 1, p, ws_ok - 4, p, None) \
        == N.TT_ERR_WORKSPACE
    b1, keep1 = _batch(desc, 1)
    assert L.tt_embed_forward(ctypes.byref(desc), p, p, p, ctypes.byref(b1), 1, 0, 1, p, ws_ok, p, None) \
        == N.TT_ERR_BATCH_TOO_SMALL
    assert L.tt_embed_backward(ctypes.byref(desc), p, ctypes.byref(b), None, 0, 1, p, ws_ok, p, None) == N.TT_ERR_ARG
    # semi-hard mining: sizes, d % 4, batch < 2, short workspace, null outputs
    assert L.tt_triplet_workspace_bytes(0, 10, 16) == N.TT_ERR_ARG
    assert L.tt_triplet_workspace_bytes(10, 10, 30) == N.TT_ERR_ARG
    tw = L.tt_triplet_workspace_bytes(100, 100, 32)
    assert tw > 0
    assert L.tt_triplet_forward(p, p, 100, 100, 32, 0, ctypes.c_float(0.2), 1, p, tw, p, p, p, None) == N.TT_ERR_ARG
    assert L.tt_triplet_forward(p, p, 100, 100, 32, 0, ctypes.c_float(0.2), 100, p, tw - 4, p, p, p, None) \
        == N.TT_ERR_WORKSPACE
    assert L.tt_triplet_forward(p, p, 100, 100, 32, 0, ctypes.c_float(0.2), 100, p, tw, None, p, p, None) \
        == N.TT_ERR_ARG
    assert L.tt_triplet_backward(p, p, 100, 100, 32, 0, 100, p, p, None, p, p, None) == N.TT_ERR_ARG
    # peer exchange: sizes, rank / world, missing error word, Adam without state
    assert L.tt_ar_region_bytes(0) == N.TT_ERR_ARG
    assert L.tt_ar_region_bytes(21313) >= 2 * 21313 * 4
    peers = N.TTArPeers()
    for q in range(2):
        peers.region[q] = p
    hp = N.adam_hp(4e-4)
    run = lambda rank, world, n, err, params=None, step=1: L.tt_ar_allreduce_adam(  # noqa: E731
        ctypes.byref(peers), rank, world, n, p, p, params, p, p, ctypes.byref(hp), None, step, err, 0, None)
    assert run(0, 0, 100, p) == N.TT_ERR_ARG
    assert run(2, 2, 100, p) == N.TT_ERR_ARG
    assert run(0, N.TT_AR_MAX_RANKS + 1, 100, p) == N.TT_ERR_ARG
    assert run(0, 2, 100, None) == N.TT_ERR_ARG
    assert run(0, 3, 100, p) == N.TT_ERR_ARG          # region of rank 2 missing
    assert run(0, 2, 100, p, step=0) == N.TT_ERR_ARG  # no device state: host epochs start at 1
    # protocol field (ABI 6): unknown values refused; push above 8 ranks unsupported
    peers.protocol = 7
    assert run(0, 2, 100, p) == N.TT_ERR_ARG
    peers.protocol = N.TT_AR_PUSH
    for q in range(9):
        peers.region[q] = p
    assert run(0, 9, 100, p) == N.TT_ERR_UNSUPPORTED
    peers.protocol = N.TT_AR_PULL
    assert (header_define("TT_AR_PULL"), header_define("TT_AR_PUSH")) == (N.TT_AR_PULL, N.TT_AR_PUSH)
