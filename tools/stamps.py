"""Per-phase timing of the fused step from the -DTT_STAMPS diagnostic build.

    CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so python tools/stamps.py [cfg3|cfg2]

Each kernel block records s_memrealtime (100 MHz, chip-wide) at its phase
boundaries (TT_STAMP(kernel, slot) in the sources).  Reported per kernel:
block start skew, and per phase the median / p90 duration over blocks, all in
microseconds.  Diagnostic only: the stamps forbid overlaps the real kernels
have, so read shares, not absolute kernel times.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402

# kernel id 4: k_bwd_first on the six-kernel path; on the folded path (no
# k_bwd_first) k_bwd_mid_fold stamps its wave 7 there (id 3 is its wave 0)
NAMES = ["k_l0_fwd", "k_l4_fwd", "k_top", "k_bwd_mid", "k_bwd_first|mid_fold w7", "k_reduce_adam",
         "sub6", "sub7"]  # sub6 / sub7: TT_SUBSTAMPS builds (finer stamps inside one kernel)


def main():
    cfgname = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.engine import FusedTrainer
    from ceo_firm_matching.synthetic import generate_pairs
    L = N.lib()
    L.tt_debug_set_stamps.restype = ctypes.c_int32
    L.tt_debug_set_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_total, nf, nc, D, B = CONFIGS[cfgname]
    n = min(n_total, int(os.environ.get("STAMPS_ROWS", 2_000_000)))
    data = generate_pairs(n, nf, nc, seed=42, device=dev)
    meta = {k: data[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    cfg = Config()
    cfg.LATENT_DIM = D
    cfg.DEVICE = dev
    torch.manual_seed(42)
    model = CEOFirmMatcher(meta, cfg).to(dev)
    tr = FusedTrainer(model, max_batch=B, seed=42)
    tr.set_data(data)
    rows = torch.randperm(n, device=dev)
    nb = n // B
    buf = torch.zeros(8 * 2048 * 8, dtype=torch.int64, device=dev)
    for _ in range(5):
        tr.step_cycle(rows, B, nb)
    torch.cuda.synchronize()
    N.check(L.tt_debug_set_stamps(buf.data_ptr()), "set_stamps")
    res = {}
    for it in range(5):
        buf.zero_()
        tr.step_cycle(rows, B, nb)
        torch.cuda.synchronize()
        st = buf.view(8, 2048, 8).cpu().numpy().astype(np.float64) / 100.0  # -> us
        res[it] = st
    N.check(L.tt_debug_set_stamps(None), "set_stamps")
    st = res[4]
    glob0 = min(st[k][st[k][:, 0] > 0, 0].min() for k in range(8) if (st[k][:, 0] > 0).any())
    for k, name in enumerate(NAMES):
        s = st[k]
        m = s[:, 0] > 0
        if not m.any():
            continue
        s = s[m]
        nslots = int((s > 0).all(axis=0).sum())
        t0 = s[:, 0].min()
        tend = s[:, nslots - 1].max()
        print(f"{name:14s} blocks={m.sum():4d} start@{t0 - glob0:8.2f}us span={tend - t0:7.2f}us "
              f"start-skew p50={np.median(s[:, 0] - t0):6.2f} max={np.max(s[:, 0] - t0):6.2f}")
        for j in range(1, nslots):
            d = s[:, j] - s[:, j - 1]
            print(f"    phase {j - 1}->{j}: p50={np.median(d):7.2f}  p90={np.percentile(d, 90):7.2f}  "
                  f"max={d.max():7.2f}")
        life = s[:, nslots - 1] - s[:, 0]
        print(f"    block life: p50={np.median(life):7.2f} max={life.max():7.2f}")
        if os.environ.get("STAMPS_BLOCKS") and name == "k_reduce_adam":
            # block life / end time by block index (element-space order of make_red)
            idx = np.nonzero(m)[0]
            for lo in range(0, len(idx), 16):
                sl = slice(lo, lo + 16)
                ph = " ".join(f"ph{j - 1}={np.median(s[sl, j] - s[sl, j - 1]):5.2f}" for j in range(1, nslots))
                print(f"      blocks {idx[sl][0]:4d}-{idx[sl][-1]:4d}: life p50={np.median(life[sl]):5.2f} "
                      f"max={life[sl].max():5.2f} end max={(s[sl, nslots - 1] - t0).max():5.2f}  {ph}")


if __name__ == "__main__":
    main()
