"""Where a stale HIP error comes from at the start of a process: the
first trainer of a fresh process failed its first step with "HIP error 1"
while every later one passed (a refused hipFuncSetAttribute in the
library's one-time LDS setup, left as the thread's last error; fixed in
set_lds_attrs).  Reads (and clears) hipGetLastError after each stage of
building the first trainer and taking its first steps."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ceo-recommender_amd"))

B = 16384
# the HIP runtime this process already uses (torch's bundled copy, which the
# library binds to by soname): a bare "libamdhip64.so" could load a second one
_tl = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
hip = ctypes.CDLL(_tl if os.path.exists(_tl) else "libamdhip64.so")
hip.hipGetLastError.restype = ctypes.c_int


def last(tag):
    print(f"{tag}: hipGetLastError={hip.hipGetLastError()}", flush=True)


def main():
    last("start")
    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    last("torch init")
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching.engine import FusedTrainer
    from conftest import load_golden, meta_of, sub
    import numpy as np
    g = load_golden("cfg3")
    meta = meta_of(g)
    cfg = Config()
    cfg.LATENT_DIM = int(g["meta/latent"])
    cfg.DROPOUT_P = 0.0
    cfg.DEVICE = torch.device("cuda:0")
    m = CEOFirmMatcher(meta, cfg)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sub(g, "init").items()})
    last("model cpu")
    m = m.to("cuda:0")
    torch.cuda.synchronize()
    last("model to gpu")
    tr = FusedTrainer(m, lr=4e-4, max_batch=B, seed=77, deterministic=False)
    torch.cuda.synchronize()
    last("trainer")
    n = 8 * B
    rng = np.random.default_rng(11)
    data = {
        "firm_numeric": torch.from_numpy(rng.standard_normal((n, meta["n_firm_numeric"])).astype(np.float32)),
        "firm_cat": torch.zeros(n, 0, dtype=torch.int64),
        "ceo_numeric": torch.from_numpy(rng.standard_normal((n, meta["n_ceo_numeric"])).astype(np.float32)),
        "ceo_cat": torch.zeros(n, 0, dtype=torch.int64),
        "target": torch.from_numpy(rng.standard_normal((n, 1)).astype(np.float32)),
        "weights": torch.from_numpy(rng.uniform(1, 10, (n, 1)).astype(np.float32)),
    }
    tr.set_data({k: v.to("cuda:0") for k, v in data.items()})
    torch.cuda.synchronize()
    last("set_data")
    rows = torch.randperm(n, device="cuda:0", generator=torch.Generator(device="cuda:0").manual_seed(3))
    torch.cuda.synchronize()
    last("randperm")
    tr.step(rows, 0, B)
    torch.cuda.synchronize()
    last("host step")
    tr.step_cycle(rows, B, 4)
    torch.cuda.synchronize()
    last("cycle step")
    print("done", flush=True)


if __name__ == "__main__":
    main()
