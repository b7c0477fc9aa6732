"""Step-by-step check of the tower-embedding entry points (prints after each sync)."""
import sys
import time
sys.path.insert(0, "ceo-recommender_amd")
sys.path.insert(0, "tests")
import torch
from ceo_firm_matching import CEOFirmMatcher, Config
from test_contrastive_train import _data, KEYS

dev = torch.device("cuda:0")
data, meta = _data()
cfg = Config(); cfg.DROPOUT_P = 0.0; cfg.DEVICE = dev
torch.manual_seed(5)
m = CEOFirmMatcher(meta, cfg).to(dev)
xb = [data[k][:128].to(dev) for k in KEYS[:4]]
torch.cuda.synchronize(); print("setup ok", flush=True)
t = time.time()
s = m(*xb); torch.cuda.synchronize(); print("score fwd ok", time.time() - t, flush=True)
u, v = m.tower_embeddings(*xb); torch.cuda.synchronize(); print("embed fwd ok", time.time() - t, u.shape, flush=True)
print(float(u.abs().sum()), float(v.abs().sum()), flush=True)
(u.sum() + v.sum()).backward(); torch.cuda.synchronize(); print("embed bwd ok", flush=True)
