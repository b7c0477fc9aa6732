"""Dev check: per-step loss of the fused engine vs the CPU loop on the CLI data."""
import sys, os, contextlib, io
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ceo-recommender_amd"), os.path.join(ROOT, "tests")]
import torch
from torch.utils.data import DataLoader
from ceo_firm_matching import Config, CEOFirmMatcher
from ceo_firm_matching.data import CEOFirmDataset
from ceo_firm_matching.engine import FusedTrainer
from ceo_firm_matching.training import sampler_batches
from test_host_pipeline import cli_data

cfg = Config(); cfg.DROPOUT_P = 0.0; cfg.DEVICE = torch.device("cpu")
train, val = cli_data(cfg)
torch.manual_seed(1234)
m_cpu = CEOFirmMatcher(train, cfg)
m_gpu = CEOFirmMatcher(train, cfg); m_gpu.load_state_dict(m_cpu.state_dict()); m_gpu = m_gpu.cuda()
loader = DataLoader(CEOFirmDataset(train), batch_size=256, shuffle=True)
batches = sampler_batches(loader)
opt = torch.optim.Adam(m_cpu.parameters(), lr=cfg.LEARNING_RATE)
tr = FusedTrainer(m_gpu, lr=cfg.LEARNING_RATE, max_batch=256, seed=0)
data = {k: train[k] for k in ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target", "weights")}
tr.set_data(data)
rows = torch.tensor([i for b in batches for i in b]).cuda()
off = 0
import warnings; warnings.simplefilter("ignore")
for b in batches:
    idx = torch.tensor(b)
    bt = {k: v[idx] for k, v in data.items()}
    m_cpu.train()
    opt.zero_grad()
    p = m_cpu(bt["firm_numeric"], bt["firm_cat"], bt["ceo_numeric"], bt["ceo_cat"])
    loss = (bt["weights"] * (p - bt["target"]) ** 2).mean()
    loss.backward(); opt.step()
    tr.step(rows, off, len(b)); off += len(b)
    lg = tr.pop_loss_sum()
    print(f"B={len(b)} cpu loss {loss.item():.6f} gpu loss {lg:.6f}")
    for (k, a), (_, g) in zip(m_cpu.state_dict().items(), m_gpu.state_dict().items()):
        d = (a.float() - g.detach().cpu().float()).abs().max().item()
        s = a.float().abs().max().item()
        if d > 1e-4 * max(s, 1e-6):
            print("   ", k, d, s)
