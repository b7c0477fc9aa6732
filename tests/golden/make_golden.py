"""Generate the golden parity vectors from the REAL reference implementation.

Run once in the build container (the only place ``/root/reference`` exists):

    python tests/golden/make_golden.py

It imports the reference package read-only (``shap``/``seaborn`` are stubbed:
neither is on the hot path -- SURVEY.md 8c), runs ``CEOFirmMatcher`` /
weighted MSE / ``torch.optim.Adam`` / ``train_model`` exactly as the
reference does, and writes small ``.npz`` fixtures (inputs + expected
outputs) next to this script.  Nothing here ships in the product, and no test
imports the reference at run time: the tests read only the ``.npz`` files.

Fixtures:
  * ``<case>.npz`` for case in {meta_test, cfg2, cfg3}:
      init params/buffers, eval forward, train forward + grads with p = 0,
      the same with injected dropout masks (p = 0.1), fp64 grads (truth),
      params after 1 and 5 Adam steps (p = 0, fixed batch sequence).
  * ``ddp.npz``: per-shard local-BN grads averaged over G in {2, 4, 8}
      shards + one Adam step (DistributedDataParallel semantics).
  * ``cli.npz``: the default CLI pipeline (cli.py:29-59) with dropout
      disabled and EPOCHS=6 under torch.manual_seed(1234): the transformed
      train tensors, printed loss lines and final state_dict.
  * ``contrastive.npz``: ``info_nce_loss``
      (contrastive.py:102-138) loss + autograd dF/dC for normalised and
      un-normalised inputs, B in {1, 2, 64, 256}; ``get_embeddings`` +
      ``compute_retrieval_metrics`` (contrastive.py:52-72, 275-332) of a
      small ContrastiveCEOFirmMatcher (the embeddings are stored too).

  * ``triplet.npz``: ``semi_hard_negative_mining`` (contrastive.py:141-192)
      loss + autograd dF/dC (fp32 and fp64) for B in {1, 2, 64, 96, 128, 256}.

  * ``contrastive_train.npz``: ``train_contrastive`` (contrastive.py:197-272),
      InfoNCE and triplet: one-step grads and a 2-epoch run (prints, final state).

  * ``ig.npz``: eval-mode backward with input gradients -- the reference's
      ``integrated_gradients`` (run_deep_extensions.py:550-603) and one
      eval-mode weighted-MSE backward (parameter + numeric-input grads).

    python tests/golden/make_golden.py [contrastive|triplet|contrastive_train|synthetic|ig]   # only that fixture
"""
import contextlib
import io
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

for _m in ("shap", "seaborn"):
    sys.modules.setdefault(_m, types.ModuleType(_m))
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

import ceo_firm_matching as ref  # noqa: E402
from ceo_firm_matching.model import CEOFirmMatcher  # noqa: E402

torch.set_num_threads(8)

META_TEST = {"n_firm_numeric": 12, "firm_cat_counts": [4, 4, 2, 2],
             "n_ceo_numeric": 2, "ceo_cat_counts": [2, 4, 2, 2, 2, 2, 2]}

CASES = {
    # name: (metadata, latent, batch)
    "meta_test": (META_TEST, 60, 32),
    "cfg2": ({"n_firm_numeric": 32, "firm_cat_counts": [], "n_ceo_numeric": 32,
              "ceo_cat_counts": []}, 64, 256),
    "cfg3": ({"n_firm_numeric": 64, "firm_cat_counts": [], "n_ceo_numeric": 64,
              "ceo_cat_counts": []}, 128, 512),
}


class MaskDropout(torch.nn.Module):
    """Dropout with an injected keep-mask, computed like ATen's dropout:
    noise = mask.div_(1 - p); out = x * noise."""

    def __init__(self, p):
        super().__init__()
        self.p = p
        self.mask = None

    def forward(self, x):
        if not self.training or self.mask is None:
            return x
        noise = self.mask.to(x.dtype).div_(1 - self.p)
        return x * noise


def make_config(latent):
    cfg = ref.Config()
    cfg.LATENT_DIM = latent
    return cfg


def make_batch(meta, B, rng):
    kf, kc = len(meta["firm_cat_counts"]), len(meta["ceo_cat_counts"])
    b = {
        "firm_numeric": rng.standard_normal((B, meta["n_firm_numeric"])).astype(np.float32),
        "firm_cat": np.stack([rng.integers(0, n, B) for n in meta["firm_cat_counts"]], 1).astype(np.int64)
        if kf else np.zeros((B, 0), np.int64),
        "ceo_numeric": rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32),
        "ceo_cat": np.stack([rng.integers(0, n, B) for n in meta["ceo_cat_counts"]], 1).astype(np.int64)
        if kc else np.zeros((B, 0), np.int64),
        "target": rng.standard_normal((B, 1)).astype(np.float32),
    }
    sd = rng.uniform(0.1, 1.0, (B, 1))
    b["weights"] = (1.0 / (sd ** 2 + 1e-6)).astype(np.float32)
    return b


def tt(b, dtype=torch.float32):
    out = {}
    for k, v in b.items():
        t = torch.from_numpy(np.ascontiguousarray(v))
        out[k] = t.to(dtype) if t.is_floating_point() else t
    return out


def set_dropout(model, p=None, masks=None):
    """p: replace every nn.Dropout's p; masks: {(tower, layer): mask} ->
    swap the Dropout modules for MaskDropout with that mask."""
    for ti, tower in enumerate((model.firm_tower, model.ceo_tower)):
        for li, idx in enumerate((3, 7)):
            if masks is not None:
                md = MaskDropout(0.1)
                md.mask = masks[(ti, li)]
                tower[idx] = md
            elif p is not None:
                tower[idx].p = p


def run_forward_backward(model, batch):
    model.train()
    model.zero_grad(set_to_none=True)
    preds = model(batch["firm_numeric"], batch["firm_cat"], batch["ceo_numeric"], batch["ceo_cat"])
    loss = (batch["weights"] * (preds - batch["target"]) ** 2).mean()
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    return preds.detach().clone(), loss.detach().clone(), grads


def put(out, prefix, d):
    for k, v in d.items():
        out[f"{prefix}/{k}"] = v.detach().cpu().clone().numpy() if torch.is_tensor(v) else np.array(v, copy=True)


def gen_case(name, meta, latent, B):
    rng = np.random.default_rng({"meta_test": 1, "cfg2": 2, "cfg3": 3}[name])
    cfg = make_config(latent)
    torch.manual_seed(0)
    model = CEOFirmMatcher(meta, cfg)
    init_sd = {k: v.clone() for k, v in model.state_dict().items()}
    out = {"meta/n_firm_numeric": meta["n_firm_numeric"], "meta/n_ceo_numeric": meta["n_ceo_numeric"],
           "meta/firm_cat_counts": np.array(meta["firm_cat_counts"], np.int64),
           "meta/ceo_cat_counts": np.array(meta["ceo_cat_counts"], np.int64),
           "meta/latent": latent}
    put(out, "init", init_sd)
    batch_np = make_batch(meta, B, rng)
    put(out, "batch", batch_np)
    batch = tt(batch_np)

    # eval forward (BN running stats: perturb them so eval is non-trivial)
    with torch.no_grad():
        for tower in (model.firm_tower, model.ceo_tower):
            for idx in (1, 5):
                bn = tower[idx]
                bn.running_mean.copy_(torch.from_numpy(rng.normal(0, 0.3, bn.running_mean.shape).astype(np.float32)))
                bn.running_var.copy_(torch.from_numpy(rng.uniform(0.5, 2.0, bn.running_var.shape).astype(np.float32)))
    put(out, "eval_buffers", {k: v for k, v in model.state_dict().items() if "running" in k})
    model.eval()
    with torch.no_grad():
        out["eval/score"] = model(batch["firm_numeric"], batch["firm_cat"], batch["ceo_numeric"], batch["ceo_cat"]).numpy()
    model.load_state_dict(init_sd)

    # train, p = 0
    set_dropout(model, p=0.0)
    preds, loss, grads = run_forward_backward(model, batch)
    out["train_p0/score"] = preds.numpy()
    out["train_p0/loss"] = loss.numpy()
    put(out, "train_p0/grad", grads)
    put(out, "train_p0/buffers", {k: v for k, v in model.state_dict().items() if "running" in k or "num_batches" in k})

    # fp64 truth for the same step
    m64 = CEOFirmMatcher(meta, cfg).double()
    m64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in init_sd.items()})
    set_dropout(m64, p=0.0)
    preds64, loss64, grads64 = run_forward_backward(m64, tt(batch_np, torch.float64))
    out["train_p0_f64/score"] = preds64.numpy()
    out["train_p0_f64/loss"] = loss64.numpy()
    put(out, "train_p0_f64/grad", grads64)

    # injected dropout masks, p = 0.1
    model.load_state_dict(init_sd)
    masks = {}
    for ti in range(2):
        for li, H in enumerate((64, 32)):
            masks[(ti, li)] = torch.from_numpy((rng.random((B, H)) >= 0.1).astype(np.float32))
            out[f"mask/{ti}_{li}"] = masks[(ti, li)].numpy().astype(np.uint8)
    set_dropout(model, masks=masks)
    preds, loss, grads = run_forward_backward(model, batch)
    out["train_mask/score"] = preds.numpy()
    out["train_mask/loss"] = loss.numpy()
    put(out, "train_mask/grad", grads)

    # k-step Adam, p = 0, a fixed sequence of 5 batches
    torch.manual_seed(0)
    model = CEOFirmMatcher(meta, cfg)
    model.load_state_dict(init_sd)
    set_dropout(model, p=0.0)
    opt = torch.optim.Adam(model.parameters(), lr=cfg.LEARNING_RATE)
    losses = []
    for k in range(5):
        bnp = make_batch(meta, B, rng)
        put(out, f"steps/batch{k}", bnp)
        b = tt(bnp)
        model.train()
        opt.zero_grad()
        preds = model(b["firm_numeric"], b["firm_cat"], b["ceo_numeric"], b["ceo_cat"])
        loss = (b["weights"] * (preds - b["target"]) ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(loss.item())
        if k in (0, 4):
            put(out, f"steps/after{k + 1}", model.state_dict())
    out["steps/losses"] = np.array(losses)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(f"wrote {name}.npz ({len(out)} arrays)")


def gen_ddp():
    meta, latent = CASES["cfg2"][0], 64
    cfg = make_config(latent)
    rng = np.random.default_rng(7)
    torch.manual_seed(0)
    base = CEOFirmMatcher(meta, cfg)
    init_sd = {k: v.clone() for k, v in base.state_dict().items()}
    out = {}
    put(out, "init", init_sd)
    for G in (2, 4, 8):
        Bl = 64
        shards = [make_batch(meta, Bl, rng) for _ in range(G)]
        acc = None
        for s, bnp in enumerate(shards):
            put(out, f"G{G}/shard{s}", bnp)
            m = CEOFirmMatcher(meta, cfg)
            m.load_state_dict(init_sd)
            set_dropout(m, p=0.0)
            _, _, grads = run_forward_backward(m, tt(bnp))
            if acc is None:
                acc = {k: v.clone() for k, v in grads.items()}
            else:
                for k in acc:
                    acc[k] += grads[k]
        avg = {k: v / G for k, v in acc.items()}
        put(out, f"G{G}/avg_grad", avg)
        m = CEOFirmMatcher(meta, cfg)
        m.load_state_dict(init_sd)
        opt = torch.optim.Adam(m.parameters(), lr=cfg.LEARNING_RATE)
        for n, p in m.named_parameters():
            p.grad = avg[n].clone()
        opt.step()
        put(out, f"G{G}/after_step", {n: p.detach() for n, p in m.named_parameters()})
    np.savez_compressed(os.path.join(HERE, "ddp.npz"), **out)
    print("wrote ddp.npz")


def gen_cli():
    """cli.py:29-59 with EPOCHS=6 and dropout disabled (p=0)."""
    from sklearn.model_selection import train_test_split
    from torch.utils.data import DataLoader
    from ceo_firm_matching.data import DataProcessor, CEOFirmDataset
    from ceo_firm_matching.synthetic import generate_synthetic_data
    from ceo_firm_matching.training import train_model

    orig_dropout = torch.nn.Dropout.__init__

    def no_dropout(self, p=0.5, inplace=False):
        orig_dropout(self, 0.0, inplace)

    cfg = ref.Config()
    cfg.EPOCHS = 6
    cfg.DEVICE = torch.device("cpu")
    processor = DataProcessor(cfg)
    raw = generate_synthetic_data(1000)
    df = processor.prepare_features(raw)
    train_df, val_df = train_test_split(df, test_size=0.2, random_state=42)
    processor.fit(train_df)
    train_data = processor.transform(train_df)
    val_data = processor.transform(val_df)
    out = {}
    for k in ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target", "weights"):
        out[f"train/{k}"] = train_data[k].numpy()
        out[f"val/{k}"] = val_data[k].numpy()
    out["meta/firm_cat_counts"] = np.array(train_data["firm_cat_counts"], np.int64)
    out["meta/ceo_cat_counts"] = np.array(train_data["ceo_cat_counts"], np.int64)
    out["meta/n_firm_numeric"] = train_data["n_firm_numeric"]
    out["meta/n_ceo_numeric"] = train_data["n_ceo_numeric"]
    torch.nn.Dropout.__init__ = no_dropout
    try:
        torch.manual_seed(1234)
        train_loader = DataLoader(CEOFirmDataset(train_data), batch_size=256, shuffle=True)
        val_loader = DataLoader(CEOFirmDataset(val_data), batch_size=256, shuffle=False)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            model = train_model(train_loader, val_loader, train_data, cfg)
    finally:
        torch.nn.Dropout.__init__ = orig_dropout
    lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("Epoch")]
    out["printed"] = np.array(lines)
    put(out, "final", model.state_dict())
    np.savez_compressed(os.path.join(HERE, "cli.npz"), **out)
    print("wrote cli.npz:", lines)


def gen_contrastive():
    from ceo_firm_matching.contrastive import (ContrastiveCEOFirmMatcher, compute_retrieval_metrics,
                                               info_nce_loss)
    out = {}
    g = torch.Generator().manual_seed(5)
    cases = {"b1": (1, 32, True), "b2": (2, 32, True), "b64": (64, 32, True),
             "b256": (256, 256, True), "raw256": (256, 256, False)}
    for name, (B, D, norm) in cases.items():
        f = torch.randn(B, D, generator=g)
        c = torch.randn(B, D, generator=g)
        if norm:
            f = torch.nn.functional.normalize(f, dim=1)
            c = torch.nn.functional.normalize(c, dim=1)
        else:
            f, c = 0.1 * f, 0.1 * c
        f.requires_grad_(True)
        c.requires_grad_(True)
        loss = info_nce_loss(f, c, 0.07)
        out[f"nce/{name}/f"] = f.detach().numpy().copy()
        out[f"nce/{name}/c"] = c.detach().numpy().copy()
        out[f"nce/{name}/loss"] = np.float32(loss.item())
        if loss.requires_grad and B <= 64:
            loss.backward()
            out[f"nce/{name}/df"] = f.grad.numpy().copy()
            out[f"nce/{name}/dc"] = c.grad.numpy().copy()
        # fp64 truth for the tolerance check
        f64 = f.detach().double().requires_grad_(True)
        c64 = c.detach().double().requires_grad_(True)
        l64 = info_nce_loss(f64, c64, 0.07)
        out[f"nce/{name}/loss64"] = np.float64(l64.item())
        if l64.requires_grad:
            l64.backward()
            # fp64 truth, stored rounded to fp32 (6e-8 relative: far below 1e-5)
            out[f"nce/{name}/df64"] = f64.grad.numpy().astype(np.float32)
            out[f"nce/{name}/dc64"] = c64.grad.numpy().astype(np.float32)
    # retrieval metrics of a small contrastive model (meta_test geometry)
    cfg = make_config(32)
    cfg.DEVICE = torch.device("cpu")
    torch.manual_seed(11)
    model = ContrastiveCEOFirmMatcher(META_TEST, cfg)
    rng = np.random.default_rng(11)
    N = 300
    bnp = make_batch(META_TEST, N, rng)
    dd = {k: torch.from_numpy(v) for k, v in bnp.items()}
    metrics = compute_retrieval_metrics(model, dd, cfg)
    model.eval()
    with torch.no_grad():
        fe, ce = model.get_embeddings(dd["firm_numeric"], dd["firm_cat"], dd["ceo_numeric"], dd["ceo_cat"])
    out["ret/firm_emb"] = fe.numpy().copy()
    out["ret/ceo_emb"] = ce.numpy().copy()
    for k, v in metrics.items():
        out[f"ret/metric/{k}"] = np.float64(v)
    np.savez_compressed(os.path.join(HERE, "contrastive.npz"), **out)
    print("wrote contrastive.npz:", {k: out[f"nce/{k}/loss"] for k in cases}, metrics)


def gen_triplet():
    """``semi_hard_negative_mining`` (contrastive.py:141-192): loss and
    autograd dF/dC of the reference's per-row loop, fp32 and fp64, for
    normalised / correlated / un-normalised pairs (B = 1 returns 0)."""
    from ceo_firm_matching.contrastive import semi_hard_negative_mining
    out = {}
    g = torch.Generator().manual_seed(7)
    nrm = torch.nn.functional.normalize
    cases = {"b1": (1, 32, "norm"), "b2": (2, 32, "norm"), "b64": (64, 32, "norm"),
             "b256": (256, 64, "norm"), "corr128": (128, 32, "corr"), "raw96": (96, 30, "raw")}
    for name, (B, D, kind) in cases.items():
        f = torch.randn(B, D, generator=g)
        c = torch.randn(B, D, generator=g)
        if kind == "norm":
            f, c = nrm(f, dim=1), nrm(c, dim=1)
        elif kind == "corr":  # positives close: a mix of semi-hard and fallback rows
            f = nrm(f, dim=1)
            c = nrm(f + 0.35 * c, dim=1)
        else:
            f, c = 0.3 * f, 0.3 * c
        for tag, dt in (("", torch.float32), ("64", torch.float64)):
            fx = f.to(dt).clone().requires_grad_(True)
            cx = c.to(dt).clone().requires_grad_(True)
            loss = semi_hard_negative_mining(fx, cx, margin=0.2)
            out[f"tri/{name}/loss{tag}"] = np.float64(loss.item())
            if loss.requires_grad:
                loss.backward()
                out[f"tri/{name}/df{tag}"] = fx.grad.numpy().astype(np.float32)
                out[f"tri/{name}/dc{tag}"] = cx.grad.numpy().astype(np.float32)
        out[f"tri/{name}/f"] = f.numpy().copy()
        out[f"tri/{name}/c"] = c.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "triplet.npz"), **out)
    print("wrote triplet.npz:", {k: out[f"tri/{k}/loss"] for k in cases})


def gen_contrastive_train():
    """``train_contrastive`` (contrastive.py:197-272) on the CLI fixture's
    train split (cli.npz), default Config (LATENT 60 -> 30-wide projections),
    dropout disabled, batch 128 (6 full + 1 partial batch), InfoNCE and
    triplet: (a) one step from the seeded init -- losses and every
    parameter's grad; (b) EPOCHS=2 of the real loop -- printed lines and the
    final state_dict."""
    from torch.utils.data import DataLoader
    from ceo_firm_matching.contrastive import (ContrastiveCEOFirmMatcher, info_nce_loss,
                                               semi_hard_negative_mining, train_contrastive)
    from ceo_firm_matching.data import CEOFirmDataset
    cli = np.load(os.path.join(HERE, "cli.npz"), allow_pickle=False)
    data = {k: torch.from_numpy(cli[f"train/{k}"]) for k in
            ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target", "weights")}
    meta = {"n_firm_numeric": int(cli["meta/n_firm_numeric"]), "firm_cat_counts": list(cli["meta/firm_cat_counts"]),
            "n_ceo_numeric": int(cli["meta/n_ceo_numeric"]), "ceo_cat_counts": list(cli["meta/ceo_cat_counts"])}
    data.update(meta)
    orig_dropout = torch.nn.Dropout.__init__

    def no_dropout(self, p=0.5, inplace=False):
        orig_dropout(self, 0.0, inplace)

    out = {}
    torch.nn.Dropout.__init__ = no_dropout
    try:
        for trip in (False, True):
            tag = "tri" if trip else "nce"
            cfg = ref.Config()
            cfg.EPOCHS = 2
            cfg.DEVICE = torch.device("cpu")
            # (a) one step
            torch.manual_seed(77)
            m = ContrastiveCEOFirmMatcher(meta, cfg)
            put(out, f"{tag}/init", m.state_dict())
            m.train()
            b = {k: data[k][:128] for k in ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target", "weights")}
            ms, fp, cp = m(b["firm_numeric"], b["firm_cat"], b["ceo_numeric"], b["ceo_cat"])
            mse = (b["weights"] * (ms - b["target"]) ** 2).mean()
            cl = semi_hard_negative_mining(fp, cp) if trip else info_nce_loss(fp, cp, 0.07)
            loss = 0.7 * mse + 0.3 * cl
            loss.backward()
            out[f"{tag}/step/mse"] = np.float64(mse.item())
            out[f"{tag}/step/cl"] = np.float64(cl.item())
            out[f"{tag}/step/loss"] = np.float64(loss.item())
            out[f"{tag}/step/match_score"] = ms.detach().numpy().copy()
            out[f"{tag}/step/firm_proj"] = fp.detach().numpy().copy()
            put(out, f"{tag}/grad", {n: p.grad for n, p in m.named_parameters()})
            # (b) the loop
            torch.manual_seed(77)
            tl = DataLoader(CEOFirmDataset(data), batch_size=128, shuffle=True)
            vl = DataLoader(CEOFirmDataset(data), batch_size=128, shuffle=False)
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                model = train_contrastive(tl, vl, meta, cfg, contrastive_weight=0.3, temperature=0.07,
                                          use_triplet=trip)
            out[f"{tag}/printed"] = np.array(buf.getvalue().splitlines())
            put(out, f"{tag}/final", model.state_dict())
    finally:
        torch.nn.Dropout.__init__ = orig_dropout
    np.savez_compressed(os.path.join(HERE, "contrastive_train.npz"), **out)
    print("wrote contrastive_train.npz:", list(out["nce/printed"]), list(out["tri/printed"]))


def gen_synthetic():
    """``synthetic.npz``: numeric columns of generate_synthetic_data(300) and
    generate_structural_synthetic_data(300, seed=7) (synthetic.py:10-110)."""
    from ceo_firm_matching.synthetic import generate_structural_synthetic_data, generate_synthetic_data
    out = {}
    base = generate_synthetic_data(300)
    for k in ("gvkey", "Age", "maxedu", "ind_firms_60w", "logatw", "match_means", "sd_match_means", "fiscalyear"):
        out[f"base/{k}"] = base[k].to_numpy()
    out["base/compindustry"] = base["compindustry"].to_numpy().astype("U8")
    st = generate_structural_synthetic_data(300, seed=7)
    for k in [f"prob_ceo_{i}" for i in range(1, 6)] + [f"prob_firm_{i}" for i in range(1, 6)] + ["tenure"]:
        out[f"structural/{k}"] = st[k].to_numpy()
    np.savez_compressed(os.path.join(HERE, "synthetic.npz"), **out)


def gen_ig():
    """Eval-mode backward with input gradients (SURVEY 8a a12 in eval mode):
    the reference's own integrated_gradients (run_deep_extensions.py:550-603:
    model.eval(), requires_grad_ on the numeric inputs, score.backward(),
    f_num.grad) on one input row, plus one eval-mode weighted-MSE backward of
    a batch (parameter and input gradients), fp32 and fp64, for the
    meta_test (embeddings) and cfg2 geometries."""
    sys.path.insert(0, REF)
    import run_deep_extensions as rde
    out = {}
    for name in ("meta_test", "cfg2"):
        meta, latent, _ = CASES[name]
        rng = np.random.default_rng(11)
        cfg = make_config(latent)
        torch.manual_seed(0)
        model = CEOFirmMatcher(meta, cfg)
        with torch.no_grad():
            for tower in (model.firm_tower, model.ceo_tower):
                for idx in (1, 5):
                    bn = tower[idx]
                    bn.running_mean.copy_(torch.from_numpy(rng.normal(0, 0.3, bn.running_mean.shape)
                                                           .astype(np.float32)))
                    bn.running_var.copy_(torch.from_numpy(rng.uniform(0.5, 2.0, bn.running_var.shape)
                                                          .astype(np.float32)))
        sd = {k: v.clone() for k, v in model.state_dict().items()}
        put(out, f"{name}/state", sd)
        out[f"{name}/latent"] = latent
        bnp = make_batch(meta, 32, rng)
        put(out, f"{name}/batch", bnp)
        base = {"firm_numeric": np.zeros((1, meta["n_firm_numeric"]), np.float32),
                "ceo_numeric": np.zeros((1, meta["n_ceo_numeric"]), np.float32)}
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            m = CEOFirmMatcher(meta, cfg).to(dt)
            m.load_state_dict({k: (v.to(dt) if v.is_floating_point() else v) for k, v in sd.items()})
            b = tt(bnp, dt)
            m.eval()
            f_num = b["firm_numeric"].clone().requires_grad_(True)
            c_num = b["ceo_numeric"].clone().requires_grad_(True)
            s = m(f_num, b["firm_cat"], c_num, b["ceo_cat"])
            loss = (b["weights"] * (s - b["target"]) ** 2).mean()
            loss.backward()
            out[f"{name}/{tag}/score"] = s.detach().numpy()
            out[f"{name}/{tag}/loss"] = loss.detach().numpy()
            out[f"{name}/{tag}/dx_firm"] = f_num.grad.numpy()
            out[f"{name}/{tag}/dx_ceo"] = c_num.grad.numpy()
            put(out, f"{name}/{tag}/grad", {n: p.grad for n, p in m.named_parameters()})
            inputs = {k: b[k][:1] for k in ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat")}
            bl = {k: torch.from_numpy(v).to(dt) for k, v in base.items()}
            ig = rde.integrated_gradients(m, inputs, bl, n_steps=8)
            out[f"{name}/{tag}/ig_firm"] = np.asarray(ig["firm_numeric"])
            out[f"{name}/{tag}/ig_ceo"] = np.asarray(ig["ceo_numeric"])
    np.savez_compressed(os.path.join(HERE, "ig.npz"), **out)
    print("wrote ig.npz")


if __name__ == "__main__":
    if sys.argv[1:] == ["ig"]:
        gen_ig()
        sys.exit(0)
    if sys.argv[1:] == ["synthetic"]:
        gen_synthetic()
        sys.exit(0)
    if sys.argv[1:] == ["contrastive_train"]:
        gen_contrastive_train()
        sys.exit(0)
    if sys.argv[1:] == ["contrastive"]:
        gen_contrastive()
        sys.exit(0)
    if sys.argv[1:] == ["triplet"]:
        gen_triplet()
        sys.exit(0)
    for name, (meta, latent, B) in CASES.items():
        gen_case(name, meta, latent, B)
    gen_ddp()
    gen_cli()
    gen_contrastive()
    gen_triplet()
    gen_contrastive_train()
    gen_synthetic()
    gen_ig()
