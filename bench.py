"""Benchmark: CEOFirmMatcher training pairs/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3|cfg2]

``--gpus N`` with N > 1 runs N ranks: under ``torch.distributed.run`` (the
driver's form) WORLD_SIZE must equal N (else exit 2); started directly, this
process spawns the N ranks itself (one child per GPU, before any GPU call)
and exits with their status.  CEO_BENCH_SHARE_GPU=1 puts every rank on GPU 0
over gloo (a rehearsal on a one-GPU box).

A "step" is one fused training step (forward, weighted MSE, backward, Adam;
all-reduce of the gradient when N > 1) over one batch of synthetic pairs that
are already resident in HBM.  Warmup: the W steps, the graph capture, then
untimed replays of the captured graph (``config.warm_replayed_steps``, 200 by
default, ~10 ms: the MI355X reaches its steady kernel speed only after that
much sustained load) right before the timed region; the timed region is
exactly K full steps.  Default workload = BASELINE cfg 3 per GPU
(10M pairs, 64x64 features, LATENT 128, batch 16384 per GPU) -- cfg 4 when run
on N GPUs (weak scaling: every rank trains its own 16384-pair batches from its
own shard of ceil(10M/N) pairs, one flat-gradient all-reduce over RCCL per
step).  Prints ONE JSON line on rank 0.

Extra legs (rank 0, N=1 only for the CPU baseline):
* roofline : per-kernel HIP-event timing of K more steps on the launch stream
  (events stamped by each kernel's dispatch via hipExtLaunchKernelGGL);
  the dominant kernel's algorithmic FLOP/s (or bytes/s) vs the MI355X peak;
  HBM traffic from the committed rocprofv3 PMC summary when present.
* cosine_roofline : the standalone fused L2-norm + cosine + weighted-MSE
  fwd/bwd kernel over 4M pairs at D=128 (HBM-bound; BASELINE metric part 2).
* cpu_baseline : the CPU oracle (oracle/two_tower.py, the reference algorithm
  restated in torch CPU ops) timed on this host, reference loop (per-sample
  Dataset + DataLoader(shuffle=True)) on a 524,288-pair sample.
"""
import argparse
import gc
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (pairs, n_firm, n_ceo, latent, batch per GPU)
    "cfg2": (1_000_000, 32, 32, 64, 4096),
    "cfg3": (10_000_000, 64, 64, 128, 16384),
}
ACHIEVABLE_HBM_GBS = 6300.0  # MI355X_MICROARCH.md: float4 copy, 79 % of spec
PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3     # dense fp32 (vector == MFMA f32) spec
# dense bf16 MFMA (v_mfma_f32_16x16x32_bf16: 16K flop / 16 cyc / SIMD, 1024 SIMDs,
# 2.4 GHz) over the 6 plane products of the bf16x3 split = the fp32-equivalent
# ceiling of the contrastive GEMM core
PEAK_BF16X3_TFLOPS = round(2516.6 / 6, 1)
# event slots of tt_train_step_ev (slot 4 stays unrecorded when the BN0
# backward is folded into k_bwd_mid: tt_step_plan)
KERNELS = ("k_l0_fwd", "k_l4_fwd", "k_top", "k_bwd_mid", "k_bwd_first", "k_reduce_adam")


def flops_per_pair(nf, nc, D):
    """Reference-algorithmic FLOPs of one training pair: the
    Linear layers of both towers, forward + backward (dW for every layer, dX
    for layers 4 and 8; dX of layer 0 is not needed without embeddings),
    2 FLOPs per multiply-add.  cfg 3: 106,496; cfg 2: 65,536."""
    per = lambda n_in: 2 * (2 * n_in * 64 + 3 * 64 * 32 + 3 * 32 * D)  # noqa: E731
    return per(nf) + per(nc)


def compulsory_bytes_per_pair(nf, nc, n_params, B):
    """SURVEY 8d compulsory HBM bytes per pair: the pair's inputs (features,
    target, weight) + the optimizer's 28 B/param/step spread over the batch.
    cfg 3: 520 + 36 = 556 B."""
    return 4 * (nf + nc + 2) + 28 * n_params / B


def kernel_work(nf, nc, D, B, n_params, plan):
    """Reference-algorithmic FLOPs and HBM bytes per launch of each step
    kernel (both towers; FLOPs count 2 per multiply-add; bytes = compulsory
    activation / input / partial-slab traffic, fp32).  plan: tt_step_plan.
    FLOPs are the reference's work, not the kernels': the folded BN0
    backward's P = dY0^T X' and Q = Zh0^T X' products stand for
    the reference's ONE dW0 = dZ0^T X, so k_bwd_mid_fold is charged dW4 +
    dA0 + dW0 (cfg 3: 537 MFLOP), not the 805 MFLOP it issues."""
    f = 4
    kp = lambda n: -(-n // 16) * 16  # noqa: E731
    tiles = lambda rows: -(-B // rows)  # noqa: E731
    t64, ttop, tmid = tiles(64), tiles(plan["top_rows"]), tiles(plan["mid_rows"])
    fold = plan["folded_bn0_backward"]
    fl = {
        "k_l0_fwd": 2 * B * 64 * (nf + nc),
        "k_l4_fwd": 2 * 2 * B * 32 * 64,
        "k_top": 2 * (3 * B * D * 32) * 2,          # U,V fwd + dW8 + dA1, both towers
        "k_bwd_mid": 2 * 2 * (2 * B * 32 * 64)      # dW4 + dA0
                     + (2 * B * 64 * (nf + nc) if fold else 0),  # dW0 (folded: P, Q combine to it)
        "k_bwd_first": 0 if fold else 2 * B * 64 * (nf + nc),    # dW0
        "k_reduce_adam": 0,
    }
    w0_slab = (2 * 64 * (kp(nf) + kp(nc))) if fold else (64 * (nf + nc) + 128)  # P | Q, or dW0 | db0
    by = {
        "k_l0_fwd": B * (nf + nc) * f + 2 * B * 64 * f,
        "k_l4_fwd": 2 * B * 64 * f + 2 * B * 32 * f,
        "k_top": 2 * B * 32 * f + 2 * B * f + 2 * B * 32 * f + ttop * 2 * (D * 32 + D) * f,
        "k_bwd_mid": (2 * B * 32 * f * 2 + 2 * B * 64 * f + tmid * 2 * (32 * 64 + 32) * f
                      + ((B * (nf + nc) * f + tmid * w0_slab * f) if fold else 2 * B * 64 * f)),
        "k_bwd_first": 0 if fold else 2 * B * 64 * f * 2 + B * (nf + nc) * f + t64 * w0_slab * f,
        "k_reduce_adam": (ttop * 2 * (D * 32 + D) + tmid * 2 * (32 * 64 + 32)
                          + (tmid if fold else t64) * w0_slab) * f + 7 * n_params * f,
    }
    return fl, by


def _pmc_kernels():
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return {}
    try:
        with open(p) as fh:
            return json.load(fh).get("kernels", {})
    except Exception:
        return {}


def pmc_traffic_stale():
    """Whether profiles/pmc_traffic.json was measured on another build than
    the library this process loaded (its library_sha256 stamp, written by
    tools/pmc_traffic.py; a summary without a stamp counts as stale)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as fh:
            stamp = json.load(fh).get("library_sha256")
        import hashlib
        from ceo_firm_matching import _native as N
        with open(N.LIB_PATH, "rb") as fh:
            return stamp != hashlib.sha256(fh.read()).hexdigest()
    except Exception:
        return True


def load_pmc_traffic(name):
    """HBM bytes per launch from a committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json written by tools/pmc_traffic.py), or None."""
    return _pmc_kernels().get(name, {}).get("hbm_bytes_per_launch")


def pmc_bytes_per_step(names):
    """Sum of the PMC bytes per launch of the step's kernels (None if any is missing)."""
    k = _pmc_kernels()
    vals = [k.get(n, {}).get("hbm_bytes_per_launch") for n in names]
    return None if not vals or any(v is None for v in vals) else float(sum(vals))


def _finite(v):
    """JSON-safe copy of a timing record: inf (a form not measured) -> None."""
    if isinstance(v, dict):
        return {k: _finite(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_finite(x) for x in v]
    return None if isinstance(v, float) and not math.isfinite(v) else v


def usable_cores():
    """CPUs this process may actually run on: the cgroup CPU quota when one
    is set (the GPU box gives each GPU a 16-CPU share of a 256-CPU host),
    else the affinity mask.  os.cpu_count() counts the whole host."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except Exception:
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_baseline(nf, nc, D, B):
    """Time the CPU oracle on a bounded sample of the same workload."""
    from oracle import two_tower as O
    usable, affinity, quota = usable_cores()
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = usable if quota else (env_threads or usable)
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    n = 524_288
    g = torch.Generator().manual_seed(42)
    data = {
        "firm_numeric": torch.randn(n, nf, generator=g), "ceo_numeric": torch.randn(n, nc, generator=g),
        "firm_cat": torch.zeros(n, 0, dtype=torch.int64), "ceo_cat": torch.zeros(n, 0, dtype=torch.int64),
        "target": torch.randn(n, 1, generator=g),
    }
    sd = torch.rand(n, 1, generator=g) * 0.9 + 0.1
    data["weights"] = 1.0 / (sd * sd + 1e-6)
    meta = {"n_firm_numeric": nf, "firm_cat_counts": [], "n_ceo_numeric": nc, "ceo_cat_counts": []}
    torch.manual_seed(42)
    P = O.init_params_like_reference(meta, D)
    buf = O.fresh_buffers()
    opt = O.Adam(P, lr=4e-4)
    loader = torch.utils.data.DataLoader(O.PairDataset(data), batch_size=B, shuffle=True)
    t0 = time.perf_counter()
    pairs, _, buf = O.cpu_train_epoch(P, buf, opt, loader, p=0.1)
    t_loop = time.perf_counter() - t0
    batches = [{k: v[i:i + B] for k, v in data.items()} for i in range(0, n, B)]
    t0 = time.perf_counter()
    pairs2, _, _ = O.cpu_train_epoch(P, buf, opt, batches, p=0.1)
    t_comp = time.perf_counter() - t0
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
    except Exception:
        pass
    torch.set_num_threads(prev_threads)
    return {"value": round(pairs / t_loop, 1), "unit": "pairs/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} pairs ({nf}x{nc} feats, D={D}, bs={B}, p=0.1), 1 epoch, oracle reference loop "
                      f"(per-sample Dataset + DataLoader(shuffle=True)) in {t_loop:.1f}s",
            "compute_only_pairs_per_s": round(pairs2 / t_comp, 1),
            "cores_basis": ("cgroup CPU quota" if quota else
                            ("OMP_NUM_THREADS: this GPU's CPU share on the pool's box" if env_threads
                             else "sched affinity")),
            "cgroup_quota_cpus": quota, "affinity_cpus": affinity,
            "os_cpu_count": os.cpu_count(), "cpu_model": cpu_model}


def cosine_roofline(dev, D=128, n=1 << 22, reps=20):
    from ceo_firm_matching import _native as N
    L = N.lib()
    g = torch.Generator(device=dev).manual_seed(7)
    u = torch.randn(n, D, device=dev, generator=g)
    v = torch.randn(n, D, device=dev, generator=g)
    t = torch.randn(n, device=dev, generator=g)
    w = torch.rand(n, device=dev, generator=g) + 1
    ls = torch.full((1,), math.log(1 / 0.07), device=dev)
    score = torch.empty(n, device=dev)
    du, dv = torch.empty_like(u), torch.empty_like(v)
    acc = torch.zeros(2, device=dev)
    st = N.stream_ptr(dev)

    def run():
        N.check(L.tt_cosine_mse_fwd_bwd(u.data_ptr(), v.data_ptr(), t.data_ptr(), w.data_ptr(), n, D,
                                        ls.data_ptr(), ctypes.c_float(1.0 / n), score.data_ptr(), du.data_ptr(),
                                        dv.data_ptr(), acc.data_ptr(), acc.data_ptr() + 4, st), "cosine")
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    byts = 4 * (4 * D + 3) * n
    gbs = byts / (ms * 1e-3) / 1e9
    # measured stream ceiling on the same box: the extension's 16-B vector
    # copy (tt_stream_copy) over a 2 GiB buffer, read + write bytes / time --
    # the practical HBM rate next to the spec (torch's copy_ is a blit that
    # runs below it)
    src = torch.ones(1 << 29, device=dev)
    dst = torch.empty_like(src)
    nbytes = src.numel() * 4

    def copy():
        N.check(L.tt_stream_copy(src.data_ptr(), dst.data_ptr(), nbytes, st), "tt_stream_copy")
    for _ in range(3):
        copy()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        copy()
    e1.record()
    torch.cuda.synchronize()
    stream = 2 * nbytes / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9
    assert bool((dst[::4096] == 1).all())
    e0.record()
    for _ in range(10):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    blit = 2 * nbytes / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9
    del src, dst
    return {"kernel": "k_cosine<2,true>", "pairs": n, "D": D, "bytes_per_pair": 4 * (4 * D + 3),
            "avg_us": round(ms * 1e3, 2), "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "stream_peak_measured": round(stream, 1),
            "stream_peak_kernel": "tt_stream_copy (16-B vector loads/stores, 2 GiB)",
            "frac_of_measured_stream": round(gbs / stream, 4), "torch_copy_gbs": round(blit, 1),
            "achievable_hbm_guide": ACHIEVABLE_HBM_GBS, "frac_of_achievable": round(gbs / ACHIEVABLE_HBM_GBS, 4),
            "pairs_per_s": round(n / (ms * 1e-3), 1)}


def side_config_leg(dev, name, steps=200, warmup=20):
    """Single-GPU pairs/s of another BASELINE config (graph-replayed fused
    steps over its own synthetic dataset) -- reported beside the headline
    workload, not as `value`."""
    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching.engine import FusedTrainer
    from ceo_firm_matching.synthetic import generate_pairs
    n_total, nf, nc, D, B = CONFIGS[name]
    data = generate_pairs(n_total, nf, nc, seed=42, device=dev)
    meta = {k: data[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    cfg = Config()
    cfg.LATENT_DIM = D
    cfg.DEVICE = dev
    torch.manual_seed(42)
    model = CEOFirmMatcher(meta, cfg).to(dev)
    tr = FusedTrainer(model, lr=cfg.LEARNING_RATE, max_batch=B, seed=42)
    tr.set_data(data)
    n_batches = n_total // B
    rows = torch.randperm(n_total, device=dev, generator=torch.Generator(device=dev).manual_seed(1000))
    for _ in range(warmup):
        tr.step_cycle(rows, B, n_batches)
    chunk = 10
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            tr.step_cycle(rows, B, n_batches)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(chunk):
            tr.step_cycle(rows, B, n_batches)
    late_after = tr.deferral_state()
    for _ in range(max(1, int(os.environ.get("CEO_BENCH_WARM_STEPS", "200")) // chunk)):
        graph.replay()  # warm replays: the steady kernel speed (main(), warm_replayed_steps)
    tr.flush()  # the warm replays' last late half: outside the timed region
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // chunk):
        graph.replay()
    tr.after_replay(late_after)
    tr.flush()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    n = (steps // chunk) * chunk
    out = {"workload": f"{name}: {n_total} pairs, {nf}x{nc} feats, LATENT={D}, bs={B}, 1 GPU, hipGraph",
           "value": round(n * B / t, 1), "unit": "pairs/s", "ms_per_step": round(1e3 * t / n, 4)}
    del graph, tr, model, data, rows
    torch.cuda.empty_cache()
    return out


def train_entry_leg(dev, name, timed_epochs=8, repeats=3):
    """The north-star entry point itself: ``training.train_model`` (alias
    ``train``, reference training.py:36-57) on a ``CEOFirmDataset`` behind a
    ``DataLoader(shuffle=True)`` of the headline config -- model build, the
    loader's exact batch order (the sampler's torch.randperm, built on worker
    threads), hipGraph-replayed fused steps, the reference's prints.  Steady
    rate = (T(2 + k epochs) - T(2 epochs)) / k epochs after one warm call:
    the per-call setup (model, upload of the dataset to HBM, trainer), the
    eager first epoch and the second epoch's hipGraph capture cancel, as
    compilation does in SURVEY 8d's steady state.  Each T is the fastest of
    ``repeats`` calls and k = 8: the setup's run-to-run spread (~10 ms, a
    third of an epoch) divided by k = 2 made single differences swing by
    +-20 % per step."""
    import contextlib
    from torch.utils.data import DataLoader
    from ceo_firm_matching import Config, training
    from ceo_firm_matching.data import CEOFirmDataset
    from ceo_firm_matching.engine import DATA_KEYS
    from ceo_firm_matching.synthetic import generate_pairs
    n_total, nf, nc, D, B = CONFIGS[name]
    d = generate_pairs(n_total, nf, nc, seed=3, device=dev)
    meta = {k: d[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    ds = CEOFirmDataset({k: d[k].cpu() for k in DATA_KEYS})  # a user's dataset: host tensors
    del d
    torch.cuda.empty_cache()
    cfg = Config()
    cfg.LATENT_DIM = D
    cfg.DEVICE = dev

    def run(epochs):
        cfg.EPOCHS = epochs
        torch.manual_seed(0)
        loader = DataLoader(ds, batch_size=B, shuffle=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(sys.stderr):  # the reference's prints
            m = training.train_model(loader, None, meta, cfg)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        del m
        return t
    run(2)
    t1 = min(run(2) for _ in range(repeats))
    tk = min(run(2 + timed_epochs) for _ in range(repeats))
    per_epoch = (tk - t1) / timed_epochs
    # one epoch's batch order on one host thread (the RandomSampler's
    # torch.randperm: sequential), the work train_model's order threads overlap
    g = torch.Generator()
    g.manual_seed(1)
    t0 = time.perf_counter()
    ref = torch.randperm(n_total, generator=g)
    t_perm = time.perf_counter() - t0
    t0 = time.perf_counter()
    mine = training.host_randperm(n_total, 1)  # what train_model's order threads run (tt_randperm)
    t_native = time.perf_counter() - t0
    assert torch.equal(mine, ref)
    steps = -(-n_total // B)
    return {"workload": f"{name}: train_model(DataLoader(CEOFirmDataset, batch_size={B}, shuffle=True)), "
                        f"{n_total} pairs, 1 GPU",
            "train_entry_pairs_per_s": round(n_total / per_epoch, 1), "ms_per_epoch": round(1e3 * per_epoch, 2),
            "us_per_step": round(1e6 * per_epoch / steps, 2), "steps_per_epoch": steps,
            "timed_epochs": timed_epochs, "repeats_min_of": repeats, "setup_plus_two_epochs_s": round(t1, 3),
            "host_permutation_ms_per_epoch_one_thread": {"torch.randperm": round(1e3 * t_perm, 2),
                                                         "tt_randperm": round(1e3 * t_native, 2)},
            "order_threads": training._order_ahead()}


def contrastive_cpu(D=256, B=4096):
    """CPU oracle InfoNCE fwd+bwd (the reference's info_nce_loss algebra) at
    B=4096, extrapolated to N x N pairs (work grows as B^2)."""
    from oracle import contrastive as OC
    g = torch.Generator().manual_seed(0)
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=g), dim=1)
    c = torch.nn.functional.normalize(torch.randn(B, D, generator=g), dim=1)
    OC.info_nce(f, c, 0.07)
    t0 = time.perf_counter()
    OC.info_nce(f, c, 0.07)
    t = time.perf_counter() - t0
    return {"sample": f"oracle info_nce fwd+bwd at B={B}, D={D}, fp32, {torch.get_num_threads()} threads",
            "seconds": round(t, 4), "scored_pairs_per_s": round(B * B / t, 1), "kind": "port",
            "cores": torch.get_num_threads()}


def contrastive_leg(dev, pg, world, rank, N=100_000, D=256, reps=3, cpu=False):
    """BASELINE cfg 5: symmetric InfoNCE fwd+bwd over the full N x N scoring
    matrix (N firms x N CEOs, D=256, L2-normalised synthetic embeddings),
    pairs sharded over the ranks (RCCL all-gather / all-reduce /
    reduce-scatter), plus retrieval ranks of every firm among all N CEOs."""
    from ceo_firm_matching.contrastive import (info_nce_loss, info_nce_loss_sharded, retrieval_ranks_rows,
                                               semi_hard_mining_rows)
    m = N // world
    g = torch.Generator(device=dev).manual_seed(500 + rank)
    f = torch.nn.functional.normalize(torch.randn(m, D, device=dev, generator=g), dim=1).requires_grad_(True)
    c = torch.nn.functional.normalize(torch.randn(m, D, device=dev, generator=g), dim=1).requires_grad_(True)

    def step():
        f.grad = None
        c.grad = None
        loss = info_nce_loss_sharded(f, c, 0.07, group=pg) if pg is not None else info_nce_loss(f, c, 0.07)
        loss.backward()
        return loss

    step()
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        loss = step()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    # retrieval ranks of this rank's firms against all CEOs
    with torch.no_grad():
        if pg is not None:
            c_all = torch.empty(N, D, device=dev)
            dist.all_gather_into_tensor(c_all, c.detach())
        else:
            c_all = c.detach()
        retrieval_ranks_rows(f.detach(), c_all, rank * m)
        torch.cuda.synchronize()
        if pg is not None:
            dist.barrier()
        t1 = time.perf_counter()
        for _ in range(reps):
            ranks = retrieval_ranks_rows(f.detach(), c_all, rank * m)
        torch.cuda.synchronize()
        tr = (time.perf_counter() - t1) / reps
        # semi-hard negative mining (contrastive.py:141-192) of this rank's
        # firms against all CEOs: the similarity GEMM + masked-min epilogue
        semi_hard_mining_rows(f.detach(), c_all, rank * m, 0.2, N)
        torch.cuda.synchronize()
        if pg is not None:
            dist.barrier()
        t2 = time.perf_counter()
        for _ in range(reps):
            tri_loss, _, _ = semi_hard_mining_rows(f.detach(), c_all, rank * m, 0.2, N)
        torch.cuda.synchronize()
        tm = (time.perf_counter() - t2) / reps
        if pg is not None:
            dist.all_reduce(tri_loss)
    if pg is not None:
        tt = torch.tensor([t, tr, tm], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t, tr, tm = tt.tolist()
    flops = 3 * 2.0 * N * N * D  # S, dF, dC GEMMs
    return {"workload": f"cfg5: InfoNCE fwd+bwd, {N} firms x {N} CEOs, D={D}, tau=0.07, fp32, "
                        f"pairs sharded over {world} GPU(s)",
            "ms_per_step": round(t * 1e3, 3), "scored_pairs_per_s": round(N * N / t, 1),
            "achieved_tflops": round(flops / t / 1e12, 2), "peak_tflops": round(PEAK_BF16X3_TFLOPS * world, 1),
            "peak_basis": "bf16 MFMA dense peak / 6 (bf16x3 split, 6 plane products per fp32 product)",
            "frac": round(flops / t / 1e12 / (PEAK_BF16X3_TFLOPS * world), 4), "bound": "mfma",
            "loss": round(float(loss.detach()), 6),
            "retrieval_ranks_ms": round(tr * 1e3, 3), "ranks_median": float(ranks.float().median()),
            "semi_hard_mining_ms": round(tm * 1e3, 3), "semi_hard_loss": round(float(tri_loss), 6),
            "semi_hard_tflops": round(2.0 * N * N * D / tm / 1e12, 2),
            "cpu_baseline": contrastive_cpu(D) if cpu else None}


def _guard_stdout():
    """Route everything native libraries print to stdout (RCCL prints its
    version banner there at communicator init) to stderr, and return a
    writer for the ONE JSON result line on the real stdout."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(os.dup(2), "w")
    out = os.fdopen(real, "w")

    def emit(line):
        out.write(line + "\n")
        out.flush()
    return emit


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """``--gpus N`` (N > 1) without a launcher: start one child process per
    GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous on 127.0.0.1), as
    ``torch.distributed.run --nproc-per-node N`` would, and return the exit
    status (the first failing child's, 0 when all succeed).  Called before
    anything touches the GPU: this process only waits.  Rank 0's JSON line
    reaches stdout through the inherited descriptor."""
    import subprocess
    share = bool(os.environ.get("CEO_BENCH_SHARE_GPU"))
    n_dev = torch.cuda.device_count()  # counts devices without initialising HIP
    if not share and n_dev < n:
        print(f"bench: --gpus {n} but {n_dev} GPU(s) visible (CEO_BENCH_SHARE_GPU=1 runs every rank on "
              f"GPU 0 as a rehearsal)", file=sys.stderr)
        return 2
    env = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=os.environ.get("MASTER_PORT") or str(_free_port()))
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r))))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                for q in pending:  # a failed rank strands the others in a collective
                    q.kill()
        time.sleep(0.05)
    return rc


def main():
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    n_req = pre.parse_known_args()[0].gpus
    if "WORLD_SIZE" not in os.environ and n_req > 1:
        sys.exit(launch_ranks(n_req))
    if n_req != int(os.environ.get("WORLD_SIZE", "1")):
        print(f"bench: --gpus {n_req} does not match WORLD_SIZE={os.environ.get('WORLD_SIZE')}", file=sys.stderr)
        sys.exit(2)
    emit = _guard_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true", help="launch every step eagerly")
    ap.add_argument("--launch", choices=("graph", "steps"), default=os.environ.get("CEO_BENCH_LAUNCH", "graph"),
                    help="single GPU: hipGraph replay of captured steps, or all K steps issued by one "
                         "tt_train_steps call (C++ launch loop, no graph)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip roofline / cosine legs")
    ap.add_argument("--no-contrastive", action="store_true", help="skip the cfg-5 contrastive leg")
    ap.add_argument("--no-train-entry", action="store_true",
                    help="skip the training.train_model (DataLoader entry point) leg")
    ap.add_argument("--no-side-config", action="store_true",
                    help="skip the other single-GPU config (PMC passes: counters of the headline config only)")
    ap.add_argument("--dp", action="store_true",
                    help="data-parallel step (all-reduce + Adam) even at world size 1 (tests the N>1 path)")
    ap.add_argument("--defer", action="store_true",
                    help="single GPU: the late half of each step's gradient reduction runs inside the next "
                         "step's first kernel (TT_FLAG_DEFER_LATE; default: the whole reduction in each step's "
                         "last kernel)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("CEO_BENCH_SHARE_GPU"):  # rehearsal: every rank on GPU 0 (one-GPU box)
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1 or args.dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        # CEO_BENCH_BACKEND=gloo: rehearsal of the N > 1 flow on a one-GPU box
        # (RCCL refuses two ranks on one device); gloo steps run eagerly.
        backend = os.environ.get("CEO_BENCH_BACKEND", "gloo" if os.environ.get("CEO_BENCH_SHARE_GPU") else "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        pg = dist.group.WORLD

    from ceo_firm_matching import CEOFirmMatcher, Config
    from ceo_firm_matching import _native as N
    from ceo_firm_matching.engine import FusedTrainer
    from ceo_firm_matching.synthetic import generate_pairs

    n_total, nf, nc, D, B = CONFIGS[args.config]
    shard = -(-n_total // world)
    data = generate_pairs(shard, nf, nc, seed=42 + rank, device=dev)
    meta = {k: data[k] for k in ("n_firm_numeric", "firm_cat_counts", "n_ceo_numeric", "ceo_cat_counts")}
    cfg = Config()
    cfg.LATENT_DIM = D
    cfg.DEVICE = dev
    if os.environ.get("CEO_BENCH_DROPOUT"):  # diagnostic: the dropout-mask cost (the workload is p = 0.1)
        cfg.DROPOUT_P = float(os.environ["CEO_BENCH_DROPOUT"])
    torch.manual_seed(42)  # identical init on every rank (DDP broadcast semantics)
    model = CEOFirmMatcher(meta, cfg).to(dev)
    tr = FusedTrainer(model, lr=cfg.LEARNING_RATE, max_batch=B, seed=42, process_group=pg,
                      defer_late=(pg is None and args.defer))
    tr.set_data(data)
    n_batches = shard // B
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    rows = torch.randperm(shard, device=dev, generator=gen)
    if os.environ.get("CEO_BENCH_SEQ_ROWS"):  # diagnostic: in-order rows (gather locality probe)
        rows = torch.arange(shard, device=dev)
    if os.environ.get("CEO_BENCH_SORT_BATCHES"):  # diagnostic: each batch's rows in index order
        nb = n_batches * B
        rows[:nb] = rows[:nb].view(n_batches, B).sort(dim=1).values.reshape(-1)

    # hipGraph replay of whole steps at every world size: the RCCL all-reduce
    # of the data-parallel step is captured with the kernels (no host work
    # per step); --no-graph launches every step eagerly.
    c_steps = args.launch == "steps" and pg is None and not args.no_graph
    use_graph = not args.no_graph and not c_steps and (pg is None or dist.get_backend(pg) == "nccl" or
                                                       tr.peer is not None)
    step_fn = lambda: tr.step_cycle(rows, B, n_batches)  # noqa: E731
    branch = os.environ.get("CEO_BENCH_BRANCH")
    if branch:
        # diagnostic (review r05 item 1): the price of a parallel branch in the
        # captured graph -- forked before each step, joined after it, on a
        # second stream; "empty": one tiny kernel (the fork / join edges alone),
        # "gather": the next batch's X rows of both towers gathered into a
        # contiguous staging tile (the branch's real work)
        side = torch.cuda.Stream()
        tiny = torch.zeros(64, device=dev)
        stage = [torch.empty(B, tr.data[k].shape[1], device=dev) for k in ("firm_numeric", "ceo_numeric")]
        nxt = rows[B:2 * B]

        def step_fn():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                if branch == "gather":
                    for k, st in zip(("firm_numeric", "ceo_numeric"), stage):
                        torch.index_select(tr.data[k], 0, nxt, out=st)
                else:
                    tiny.add_(1.0)
            tr.step_cycle(rows, B, n_batches)
            cur.wait_stream(side)
    for _ in range(args.warmup):
        step_fn()
    torch.cuda.synchronize()

    # chunks of 16 steps (measured: 10 -> 16 takes 0.8 us off a step, 20 /
    # 25 / 40 add 0.3-1.1 us), the remainder of K in a second, shorter graph.
    # The driver's K = 20 stays two graphs of 10: round 5, five interleaved
    # runs of the driver's command per chunk size, 53.7-53.9 us per step
    # against 54.7-55.0 (4-step graphs) and 54.3-54.7 (5-step graphs)
    graph, graph_rem, chunk = None, None, 1
    warm_steps = int(os.environ.get("CEO_BENCH_WARM_STEPS", "200"))  # replayed steps before the clock (below)
    warm_replayed = 0
    if use_graph:
        # K split into equal graphs of at most 16 steps (the driver's K = 20:
        # two of 10 -- four interleaved rounds: 56.0-56.4 us per step against
        # 56.5-57.1 for one graph of 20 and 57.1 for 16 + 4; graphs of 4-5
        # steps 56.8-57.5)
        cmax = int(os.environ.get("CEO_BENCH_CHUNK_MAX", "16"))
        n_graphs = -(-args.steps // cmax)
        chunk = -(-args.steps // n_graphs)
        rem = args.steps % chunk
        ok = 1
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    step_fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):  # recorded only: nothing executes during capture
                for _ in range(chunk):
                    step_fn()
            if rem:
                graph_rem = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph_rem):
                    for _ in range(rem):
                        step_fn()
        except Exception as e:  # capture unsupported here: every rank falls back to eager steps
            print(f"bench: graph capture failed ({e!r}); eager steps", file=sys.stderr)
            ok, graph, graph_rem = 0, None, None
        if pg is not None:  # all ranks replay, or none does
            flag = torch.tensor([ok], device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 0:
                graph, graph_rem = None, None
        if graph is not None:
            # warm the replayed path itself, right before the clock starts:
            # MI355X needs ~10 ms of sustained load before its kernels run at
            # their steady-state speed (round 5, the driver's K = 20 / W = 5:
            # 52.5-52.7 us per step after one warm replay, 52.2-53.0 after 5,
            # 50.2-50.8 after 20 -- the K = 400 steady state is 50.5; eager
            # warmup steps before the capture do not carry over the capture's
            # idle host time).  A fixed replay count, the same on every rank
            # (a data-parallel replay waits for its peers); reported in config
            warm_rounds = max(1, -(-warm_steps // chunk))
            for _ in range(warm_rounds):
                graph.replay()
                if graph_rem is not None:
                    graph_rem.replay()
            warm_replayed = warm_rounds * (chunk + (rem if graph_rem is not None else 0))
        torch.cuda.synchronize()
        if pg is not None:
            dist.barrier()
        if graph is None:
            chunk = 1
    late_after = tr.deferral_state()  # what each captured graph's last step leaves pending

    tr.pop_loss_sum(read=False)
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    # roctx range around the timed region, opened before t0 and
    # closed after the clock stops: no host call inside the region but the
    # replays themselves (the per-step ranges are the C-ABI's own, eager steps)
    region = N.trace_range(f"bench timed region: {args.steps} steps, rank {rank}")
    region.__enter__()
    t0 = time.perf_counter()
    if graph is not None:  # exactly K steps: K // chunk full chunks + the remainder graph
        for _ in range(args.steps // chunk):
            graph.replay()
        if graph_rem is not None:
            graph_rem.replay()
    elif c_steps:  # exactly K steps launched by one tt_train_steps call
        tr.step_cycle_n(rows, B, n_batches, args.steps)
    else:
        for _ in range(args.steps):
            step_fn()
    if graph is not None:
        tr.after_replay(late_after)  # the replays ran outside step(): the last one's late half is pending
    tr.flush()  # the last step's deferred late half: inside the timed region (K whole steps)
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    region.__exit__(None, None, None)
    if pg is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    loss = tr.pop_loss_sum() / args.steps  # also raises if the peer exchange failed
    pairs = args.steps * B * world
    value = pairs / elapsed
    det_ms = None
    if world == 1 and graph is not None and not args.no_extras:
        # the same step in deterministic-reduction mode (TT_FLAG_DETERMINISTIC:
        # slots + in-order folds instead of float atomics): its cost, reported
        # beside the headline (which runs the default atomic mode)
        tr.deterministic = True
        g_det = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step_fn()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g_det):
            for _ in range(chunk):
                step_fn()
        g_det.replay()
        torch.cuda.synchronize()
        reps = max(1, args.steps // chunk)
        t1 = time.perf_counter()
        for _ in range(reps):
            g_det.replay()
        torch.cuda.synchronize()
        det_ms = 1e3 * (time.perf_counter() - t1) / (reps * chunk)
        tr.deterministic = None
        N.set_deterministic(tr.desc, tr.is_deterministic())  # the event pass below calls the C-ABI directly
        del g_det
        tr.pop_loss_sum(read=False)

    result = {
        "metric": "training pairs/sec (fused fwd+bwd+Adam, CEOFirmMatcher two-tower)",
        "value": round(value, 1), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (N(0,1) features/target, sd~U(0.1,1), w=1/(sd^2+1e-6); random-init weights, "
                "seed 42), resident in HBM",
        "config": {"workload": f"{args.config}: {n_total} pairs ({shard}/GPU), {nf}x{nc} feats, LATENT={D}, "
                               f"bs={B}/GPU, dropout 0.1, Adam lr 4e-4",
                   "global_batch": B * world, "parallelism": f"dp{world}" if pg is not None else "single",
                   "graph": bool(graph is not None), "graph_chunk": chunk,
                   "warm_replayed_steps": warm_replayed,  # untimed graph replays after the W warmup steps
                   "launch": "tt_train_steps" if c_steps else ("hipgraph" if graph is not None else "eager"),
                   "late_half": "deferred into the next step's k_l0_fwd" if tr.defer_late and not c_steps
                                else "in k_reduce_adam",
                   "grad_exchange": ("peer-memory one-shot inside k_reduce_adam (+ Adam)" if tr.fused_exchange
                                     else "peer-memory one-shot + fused Adam" if getattr(tr, "peer", None) is not None
                                     else ("rccl all-reduce" if pg is not None and dist.get_backend(pg) == "nccl"
                                           else ("gloo all-reduce" if pg is not None else "none"))),
                   "exchange_vs_collective_us": (getattr(getattr(tr, "peer", None), "timing_us", None)),
                   # (in-reduction exchange, reduce -> exchange + Adam): device us per step, MAX over
                   # ranks, measured on the first data-parallel step; the faster form is used
                   "fused_vs_two_launch_us": _finite(getattr(tr, "fused_vs_two_launch_us", None)),
                   # every exchange form the validation timed (MAX over ranks; inf: not
                   # bitwise equal to the reference form on some rank) and the one chosen
                   "exchange_form": getattr(tr, "exchange_form", None),
                   "exchange_form_us": _finite(getattr(tr, "exchange_form_us", None))},
        "mean_loss": round(loss, 5),
        "deterministic_ms_per_step": round(det_ms, 4) if det_ms is not None else None,
    }

    # the training state travels in a dict that run_extras empties before the
    # 40 GB (N = 1) similarity workspace of the contrastive leg
    held = {"tr": tr, "model": model, "data": data, "rows": rows}
    del tr, model, data, rows, step_fn
    graph = graph_rem = None
    try:
        if not args.no_extras:
            run_extras(args, result, dev, pg, world, rank, held, B, n_batches, elapsed, nf, nc, D)
    except Exception as e:  # the headline is measured: report it whatever an extra leg does
        print(f"bench: extra legs failed: {e!r}", file=sys.stderr)
        result["extras_error"] = repr(e)[:300]

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(nf, nc, D, B)
    else:
        result["cpu_baseline"] = None
    if rank == 0:
        emit(json.dumps(result))
    if pg is not None:
        dist.destroy_process_group()


def run_extras(args, result, dev, pg, world, rank, held, B, n_batches, elapsed, nf, nc, D):
    """Per-kernel events and rooflines, the cosine kernel, the side config and
    the contrastive leg (after the headline measurement)."""
    from ceo_firm_matching import _native as N
    tr, rows = held["tr"], held["rows"]
    # ---- per-kernel HIP events on the launch stream (separate pass, K steps)
    st = N.stream_ptr(dev)
    # 2 events per kernel, stamped by the kernel's own dispatch
    # (tt_train_step_ev -> hipExtLaunchKernelGGL): kernel-only durations
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(12)] for _ in range(args.steps)]
    for row in evs:
        for e in row:
            e.record()  # materialise the hipEvent
    torch.cuda.synchronize()
    a = tr.arena
    # the steps as the timed region ran them: with the deferred late half
    # (TT_FLAG_DEFER_LATE) every step after the first carries the previous
    # one's late half in its k_l0_fwd, and k_reduce_adam holds the early half
    tr.flush()
    defer = tr.defer_late and pg is None
    batch = None
    for k in range(args.steps):
        arr = (ctypes.c_void_p * 12)(*[e.cuda_event for e in evs[k]])
        batch = tr._batch(rows, 0, B, cycle=n_batches)
        extra = (N.TT_FLAG_DEFER_LATE | (N.TT_FLAG_LATE_PENDING if k else 0)) if defer else 0
        tr.desc.flags |= extra
        rc = tr.lib.tt_train_step_ev(tr.desc, a.params.data_ptr(), a.buffers.data_ptr(), a.nbt.data_ptr(),
                                     batch, tr.hp, tr.seed, tr.state.data_ptr(), tr.ws.data_ptr(),
                                     tr.ws_bytes, tr.grad.data_ptr(), tr.exp_avg.data_ptr(),
                                     tr.exp_avg_sq.data_ptr(), int(pg is None), st, arr)
        tr.desc.flags &= ~extra
        N.check(rc, "tt_train_step_ev")
        if pg is not None:
            tr.allreduce_and_adam()
    if defer and batch is not None:
        tr.after_replay((B, batch))
        tr.flush()
    torch.cuda.synchronize()
    plan = N.step_plan(tr.desc, B)
    per = {}
    for i, name in enumerate(KERNELS):
        if name == "k_bwd_first" and plan["folded_bn0_backward"]:
            continue  # not launched: its work runs inside k_bwd_mid (folded BN0 backward)
        per[name] = sum(evs[k][2 * i].elapsed_time(evs[k][2 * i + 1]) for k in range(args.steps)) / args.steps * 1e3
    fl, by = kernel_work(nf, nc, D, B, a.params.numel(), plan)
    for on, (old, new) in ((plan["folded_bn0_backward"], ("k_bwd_mid", "k_bwd_mid_fold")),
                           (plan["top_pair"], ("k_top", "k_top_pair"))):
        if on:  # report the kernel that ran under its own name
            for d_ in (per, fl, by):
                d_[new] = d_.pop(old)
    dom = max(per, key=per.get)
    t_s = per[dom] * 1e-6
    tf = fl[dom] / t_s / 1e12
    gbs = by[dom] / t_s / 1e9
    # a kernel with GEMM work is priced on the MFMA roofline (its reference
    # FLOPs), the gradient reduce on HBM; the other figure rides along
    if fl[dom] > 0:
        roof = {"bound": "mfma", "achieved": round(tf, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tf / PEAK_FP32_TFLOPS, 4), "algorithmic_per_launch": fl[dom],
                "hbm_gbs_secondary": round(gbs, 1), "hbm_frac_secondary": round(gbs / PEAK_HBM_GBS, 4)}
    else:
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_per_launch": by[dom]}
    roof["kernel"] = dom
    roof["avg_us"] = round(per[dom], 3)
    roof["traffic"] = load_pmc_traffic(dom)
    roof["traffic_stale"] = pmc_traffic_stale()
    result["roofline"] = roof
    # the whole step against the same peaks: reference FLOPs per pair x B
    # over the timed ms_per_step, and the PMC bytes of all the step's
    # kernels against SURVEY 8d's compulsory bytes per pair
    fpp = flops_per_pair(nf, nc, D)
    cbp = compulsory_bytes_per_pair(nf, nc, a.params.numel(), B)
    step_s = elapsed / args.steps
    pmc_step = pmc_bytes_per_step(list(per))
    result["step_roofline"] = {
        "flops_per_pair": fpp, "flops_per_step": fpp * B,
        "achieved_tflops": round(fpp * B / step_s / 1e12, 2), "peak_tflops": PEAK_FP32_TFLOPS,
        "frac_mfma": round(fpp * B / step_s / 1e12 / PEAK_FP32_TFLOPS, 4),
        "compulsory_bytes_per_pair": round(cbp, 1), "compulsory_bytes_per_step": round(cbp * B),
        "compulsory_gbs": round(cbp * B / step_s / 1e9, 1),
        "pmc_bytes_per_step": pmc_step,
        "pmc_over_compulsory": round(pmc_step / (cbp * B), 2) if pmc_step else None}
    result["kernel_us"] = {k: round(v, 3) for k, v in per.items()}
    result["step_plan"] = plan
    result["step_us_sum_of_kernels"] = round(sum(per.values()), 2)
    if rank == 0:
        result["cosine_roofline"] = cosine_roofline(dev, D=D)
    if world == 1 and not args.no_side_config:  # the other single-GPU BASELINE config (cfg 2)
        others = [c for c in CONFIGS if c != args.config]
        result["other_configs"] = {c: side_config_leg(dev, c) for c in others}
    # drop the training state before the 40 GB (N=1) similarity workspace
    del tr, rows
    held.clear()
    gc.collect()
    torch.cuda.empty_cache()
    if world == 1 and not args.no_train_entry:  # training.train() itself, on the headline config
        result["train_entry"] = train_entry_leg(dev, args.config)
        result["train_entry_pairs_per_s"] = result["train_entry"]["train_entry_pairs_per_s"]
        gc.collect()
        torch.cuda.empty_cache()
    if not args.no_contrastive:
        result["contrastive"] = contrastive_leg(dev, pg, world, rank,
                                                cpu=(rank == 0 and world == 1 and not args.no_cpu_baseline))


if __name__ == "__main__":
    main()
