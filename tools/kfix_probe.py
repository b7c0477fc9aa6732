"""Fixed cost of bench.py's timed region at the driver's K = 20: the same
cfg-3 steps replayed from hipGraphs split in different chunk lists, each
timed region measured REPS times, interleaved.  CEO_PROBE_SPIN=1 sets
hipDeviceScheduleSpin before the HIP context exists (host sync by spinning).

usage: python tools/kfix_probe.py [K] [REPS]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))
sys.path.insert(0, ROOT)

if os.environ.get("CEO_PROBE_SPIN"):
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)))

import torch  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from bench import CONFIGS
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching.engine import FusedTrainer
    from ceo_firm_matching.synthetic import generate_pairs
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n_total, nf, nc, D, B = CONFIGS["cfg3"]
    data = generate_pairs(n_total, nf, nc, seed=42, device=dev)
    meta = {k: data[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    cfg = Config()
    cfg.LATENT_DIM = D
    cfg.DEVICE = dev
    torch.manual_seed(42)
    model = CEOFirmMatcher(meta, cfg).to(dev)
    tr = FusedTrainer(model, lr=cfg.LEARNING_RATE, max_batch=B, seed=42)
    tr.set_data(data)
    nb = n_total // B
    rows = torch.randperm(n_total, device=dev, generator=torch.Generator(device=dev).manual_seed(1000))
    step = lambda: tr.step_cycle(rows, B, nb)  # noqa: E731
    for _ in range(5):
        step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graphs = {}

    def graph_of(n):
        if n not in graphs:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    step()
            g.replay()
            torch.cuda.synchronize()
            graphs[n] = g
        return graphs[n]
    spec = os.environ.get("CEO_PROBE_VARIANTS")  # e.g. "10+10,4+4+4+4+4"
    if spec:
        variants = {v: [int(x) for x in v.split("+")] for v in spec.split(",")}
    else:
        variants = {"10+10": [10, 10], "20": [20], "2+18": [2, 18], "1+19": [1, 19], "4+16": [4, 16],
                    "5x4": [4] * 5, "2+9+9": [2, 9, 9]}
    variants = {k: v for k, v in variants.items() if sum(v) == K} or {str(K): [K]}
    for v in variants.values():
        for n in v:
            graph_of(n)
    res = {k: [] for k in variants}
    host = {k: [] for k in variants}  # host time of the first replay() call
    for _ in range(reps):
        for name, v in variants.items():
            gs = [graphs[n] for n in v]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, g in enumerate(gs):
                g.replay()
                if i == 0:
                    host[name].append(1e6 * (time.perf_counter() - t0))
            torch.cuda.synchronize()
            res[name].append(1e6 * (time.perf_counter() - t0))
    # long runs (400 steps) for the per-step rate at several chunk sizes
    rates = {}
    for c in (2, 4, 5, 8, 16):
        g = graph_of(c)
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(400 // c):
                g.replay()
            torch.cuda.synchronize()
            v = 1e6 * (time.perf_counter() - t0) / (400 // c * c)
            best = v if best is None else min(best, v)
        rates[c] = round(best, 2)
    print("400-step rate by chunk (us/step, best of 3):", rates)
    per = rates[16]
    for name, v in res.items():
        v = sorted(v)
        med = v[len(v) // 2]
        print(f"K={K} chunks {name:7s}: median {med:8.1f} us total = {med / K:6.2f} us/step "
              f"(min {v[0]:.1f}, p90 {v[int(0.9 * len(v))]:.1f}); fixed vs 400-step rate {per:.2f} us/step: "
              f"{med - K * per:.1f} us; first replay() host call {sorted(host[name])[len(v) // 2]:.1f} us")


if __name__ == "__main__":
    main()
