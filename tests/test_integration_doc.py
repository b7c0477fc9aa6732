"""INTEGRATION.md's ctypes stub is code a maintainer pastes into the
reference: execute it as written.

* CPU: every ```python block of section B runs against libceo_tt.so (loads,
  binds, and its own asserts tie each ctypes struct to the library's
  ``tt_struct_size``); the stub's structs have the binding's fields;
* GPU: the stub's ``train_step`` (the replacement of training.py:44-55)
  gives bitwise the parameters, Adam moments and BN buffers of
  ``FusedTrainer.step`` in deterministic mode over three steps.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden, meta_of, sub

DOC = os.path.join(ROOT, "INTEGRATION.md")


def stub_blocks():
    txt = open(DOC).read()
    sec = txt[txt.index("## B."):txt.index("## Data-parallel launch")]
    return re.findall(r"```python\n(.*?)```", sec, flags=re.S)


def load_stub():
    from ceo_firm_matching import _native as N
    os.environ["CEO_TT_LIB"] = N.LIB_PATH
    ns = {}
    for code in stub_blocks():
        exec(compile(code, DOC, "exec"), ns)  # noqa: S102 -- the document's own code
    return ns


def test_stub_blocks_execute_and_match_the_library():
    from ceo_firm_matching import _native as N
    blocks = stub_blocks()
    assert len(blocks) >= 3
    ns = load_stub()
    L = N.lib()
    for which, name in ((N.TT_STRUCT_MODEL_DESC, "TTModelDesc"), (N.TT_STRUCT_BATCH, "TTBatch"),
                        (N.TT_STRUCT_ADAM_HP, "TTAdamHP")):
        st = ns[name]
        assert ctypes.sizeof(st) == L.tt_struct_size(which), name
        mine = getattr(N, name)
        assert [f[0] for f in st._fields_] == [f[0] for f in mine._fields_], name
        for (fn, _), (fm, _) in zip(st._fields_, mine._fields_):
            assert getattr(st, fn).offset == getattr(mine, fm).offset, (name, fn)
    assert L.tt_struct_size(99) == -1
    assert callable(ns["train_step"]) and callable(ns["backward_ex"]) and callable(ns["semi_hard_loss"])
    # the DataLoader-order stub is torch's randperm under the sampler's seed
    for n, seed in ((0, 1), (1000, 5), (100_003, 2 ** 45 + 3)):
        g = torch.Generator()
        g.manual_seed(seed)
        assert torch.equal(ns["epoch_order"](n, seed), torch.randperm(n, generator=g)), (n, seed)


@pytest.mark.gpu
def test_stub_train_step_bitwise_equals_fused_trainer():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.engine import FusedTrainer
    ns = load_stub()
    dev = torch.device("cuda:0")
    g = load_golden("cfg2")
    meta = meta_of(g)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = 0.1
    cfg.DEVICE = dev
    init = {k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()}
    B, K = 512, 3
    rng = np.random.default_rng(11)
    data = {
        "firm_numeric": torch.from_numpy(rng.standard_normal((K * B, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.zeros(K * B, 0, dtype=torch.int64),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((K * B, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.zeros(K * B, 0, dtype=torch.int64),
        "target": torch.from_numpy(rng.standard_normal((K * B,)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (K * B,)).astype(np.float32)),
    }
    d = {k: v.to(dev) for k, v in data.items()}
    seed = 99

    # (a) the package's trainer, deterministic reductions
    m1 = CEOFirmMatcher(meta, cfg)
    m1.load_state_dict(init)
    m1 = m1.to(dev)
    tr = FusedTrainer(m1, lr=4e-4, max_batch=B, seed=seed, deterministic=True)
    tr.set_data(d)
    for k in range(K):
        tr.step(None, k * B, B)
    torch.cuda.synchronize()

    # (b) the INTEGRATION.md stub on a second copy of the same model
    m2 = CEOFirmMatcher(meta, cfg)
    m2.load_state_dict(init)
    m2 = m2.to(dev)
    arena = m2.bind_arena()
    desc = ns["TTModelDesc"]()
    ctypes.memmove(ctypes.addressof(desc), ctypes.addressof(arena.desc), ctypes.sizeof(desc))
    desc.flags |= N.TT_FLAG_DETERMINISTIC
    hp = ns["TTAdamHP"](4e-4, 0.9, 0.999, 1e-8)
    n = arena.params.numel()
    grad, mom, vel = (torch.zeros(n, device=dev) for _ in range(3))
    state = torch.zeros(4, dtype=torch.int64, device=dev)
    ws = torch.zeros(N.workspace_bytes(arena.desc, B) // 4, device=dev)
    for k in range(K):
        b = ns["TTBatch"]()
        b.num[0], b.num_ld[0] = d["firm_numeric"].data_ptr(), d["firm_numeric"].stride(0)
        b.num[1], b.num_ld[1] = d["ceo_numeric"].data_ptr(), d["ceo_numeric"].stride(0)
        b.target, b.weight = d["target"].data_ptr(), d["weights"].data_ptr()
        b.row0, b.n_rows = k * B, B
        ns["train_step"](desc, arena, b, hp, seed, state, ws, grad, mom, vel)
    torch.cuda.synchronize()
    assert int(state[0]) == K
    for a_, b_ in ((tr.arena.params, arena.params), (tr.exp_avg, mom), (tr.exp_avg_sq, vel),
                   (tr.arena.buffers, arena.buffers), (tr.arena.nbt, arena.nbt)):
        assert torch.equal(a_, b_)
