"""Dev: the stamps.py eager step loop on the production library (for rocprof)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ceo-recommender_amd")]
import torch
from bench import CONFIGS
from ceo_firm_matching import CEOFirmMatcher, Config
from ceo_firm_matching.engine import FusedTrainer
from ceo_firm_matching.synthetic import generate_pairs
dev = torch.device("cuda", 0)
n_total, nf, nc, D, B = CONFIGS["cfg3"]
n = min(n_total, int(os.environ.get("STAMPS_ROWS", 2_000_000)))
data = generate_pairs(n, nf, nc, seed=42, device=dev)
meta = {k: data[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
cfg = Config(); cfg.LATENT_DIM = D; cfg.DEVICE = dev
torch.manual_seed(42)
model = CEOFirmMatcher(meta, cfg).to(dev)
tr = FusedTrainer(model, max_batch=B, seed=42)
tr.set_data(data)
rows = torch.randperm(n, device=dev)
for _ in range(30):
    tr.step_cycle(rows, B, n // B)
torch.cuda.synchronize()
print("done")
