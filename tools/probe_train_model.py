"""Throughput of the user-facing entry point train_model (training.py) on a
cfg-3-shaped synthetic dataset: wall time per epoch and per step, split into
the host's batch-order construction and the fused steps.

usage: python tools/probe_train_model.py [n_pairs] [epochs]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ceo-recommender_amd"))

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from ceo_firm_matching import Config, training  # noqa: E402
from ceo_firm_matching.data import CEOFirmDataset  # noqa: E402
from ceo_firm_matching.synthetic import generate_pairs  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    d = generate_pairs(n, 64, 64, seed=3)
    meta = {k: d[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    ds = CEOFirmDataset({k: d[k] for k in ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target",
                                           "weights")})
    cfg = Config()
    cfg.LATENT_DIM = 128
    cfg.DEVICE = torch.device("cuda")
    bs = 16384
    steps = -(-n // bs)
    t_order = []
    orig = training.sampler_batches

    def timed_order(loader):
        t0 = time.perf_counter()
        out = orig(loader)
        t_order.append(time.perf_counter() - t0)
        return out

    training.sampler_batches = timed_order  # the fallback path only (epoch_order covers DataLoader(shuffle))
    res = {}
    for e in (1, 1, epochs):  # the first call pays one-time costs (module load, allocations)
        cfg.EPOCHS = e
        torch.manual_seed(0)
        loader = DataLoader(ds, batch_size=bs, shuffle=True)
        t_order.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        training.train_model(loader, None, meta, cfg)
        torch.cuda.synchronize()
        res[e] = (time.perf_counter() - t0, sum(t_order))
    dt = res[epochs][0] - res[1][0]
    do = res[epochs][1] - res[1][1]
    ep = epochs - 1
    print(f"train_model: {n} pairs, bs {bs}, {steps} steps/epoch: {1e3 * dt / ep:.1f} ms/epoch "
          f"({1e6 * dt / (ep * steps):.1f} us/step, {n * ep / dt / 1e6:.1f} M pairs/s); "
          f"list-based batch order {1e3 * do / ep:.1f} ms/epoch")


if __name__ == "__main__":
    main()
