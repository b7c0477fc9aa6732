"""Run-to-run check of train_contrastive on the GPU: the 2-epoch loop of
tests/test_contrastive_train.py three times, per-parameter normwise error
vs the reference fixture and between runs."""
import sys
sys.path.insert(0, "ceo-recommender_amd")
sys.path.insert(0, "tests")
import numpy as np
import torch
from conftest import load_golden, normwise, sub, excluded_param
from test_contrastive_train import _run_loop

trip = len(sys.argv) > 1 and sys.argv[1] == "tri"
g = load_golden("contrastive_train")
tag = "tri" if trip else "nce"
ref = sub(g, f"{tag}/final")
runs = []
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    model, lines, cfg = _run_loop(torch.device("cuda"), trip)
    sd = {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}
    runs.append(sd)
    errs = {k: normwise(sd[k], ref[k]) for k in ref if sd[k].dtype.kind == "f" and not excluded_param(k)
            and not k.endswith("running_mean")}
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:6]
    print(f"run {it}: {lines[-1]}", flush=True)
    print("   vs ref worst:", [(k, f"{v:.2e}") for k, v in worst], flush=True)
for it in range(1, len(runs)):
    d = {k: normwise(runs[it][k], runs[0][k]) for k in ref if runs[0][k].dtype.kind == "f"}
    worst = sorted(d.items(), key=lambda kv: -kv[1])[:6]
    print(f"run {it} vs run 0:", [(k, f"{v:.2e}") for k, v in worst], flush=True)
