"""Run-to-run determinism probe of the fused forward/backward at a ragged
large batch: the same inputs N times in one process; reports, per parameter,
the max deviation of each run's gradient from the first run's (fp32 atomics
make ~1e-7 relative expected; anything near 1e-3 is a bug)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden, meta_of, sub  # noqa: E402
from ceo_firm_matching import CEOFirmMatcher, Config  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 12
g = load_golden("cfg3")
meta = meta_of(g)
cfg = Config()
cfg.LATENT_DIM = int(g["meta/latent"])
cfg.DROPOUT_P = 0.1
cfg.DEVICE = torch.device("cuda")
dev = torch.device("cuda:0")
rng = np.random.default_rng(B)
fn = torch.from_numpy(rng.standard_normal((B, meta["n_firm_numeric"])).astype(np.float32)).to(dev)
cn = torch.from_numpy(rng.standard_normal((B, meta["n_ceo_numeric"])).astype(np.float32)).to(dev)
fc = torch.zeros((B, 0), dtype=torch.int64, device=dev)
cc = torch.zeros((B, 0), dtype=torch.int64, device=dev)
tg = torch.from_numpy(rng.standard_normal((B, 1)).astype(np.float32)).to(dev)
wt = torch.from_numpy(rng.uniform(1, 10, (B, 1)).astype(np.float32)).to(dev)
ref = None
worst = {}
for k in range(runs):
    torch.manual_seed(1234)
    m = CEOFirmMatcher(meta, cfg)
    m.load_state_dict({kk: torch.from_numpy(np.asarray(v)) for kk, v in sub(g, "init").items()})
    m = m.to(dev)
    m.train()
    m._stream_step = 0
    s = m(fn, fc, cn, cc)
    loss = (wt * (s - tg) ** 2).mean()
    loss.backward()
    grads = {n: p.grad.detach().double().cpu().numpy() for n, p in m.named_parameters()}
    if ref is None:
        ref = grads
        continue
    for n, v in grads.items():
        d = float(np.max(np.abs(v - ref[n])) / max(np.max(np.abs(ref[n])), 1e-30))
        worst[n] = max(worst.get(n, 0.0), d)
        if d > 1e-4:
            bad = np.argwhere(np.abs(v - ref[n]) > 1e-4 * np.max(np.abs(ref[n])))
            print(f"run {k}: {n} normwise dev {d:.3g} at {len(bad)} elements, first {bad[:4].tolist()}")
for n, d in worst.items():
    print(f"{n:28s} max normwise dev over runs {d:.3g}")
