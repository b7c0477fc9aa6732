"""Second k_cosine shape probe (cos_probe2.hip): lanes per row, rows per lane
group, prefetch, load kind, grid; B = 4M, D = 128, loss sums in one line."""
import ctypes, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))
from ceo_firm_matching import _native as N
P = ctypes.CDLL(os.path.join(ROOT, "tools", "cosprobe", "cos_probe2.so"))
P.cos_probe2.argtypes = [ctypes.c_int, ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_float] + [ctypes.c_void_p] * 6
dev = torch.device("cuda:0")
B, D = 1 << 22, 128
g = torch.Generator(device=dev).manual_seed(0)
u = torch.randn(B, D, device=dev, generator=g); v = torch.randn(B, D, device=dev, generator=g)
tg = torch.randn(B, device=dev, generator=g); wt = torch.rand(B, device=dev, generator=g) + 1
ls = torch.tensor([0.3], device=dev)
sc, du, dv = torch.empty(B, device=dev), torch.empty_like(u), torch.empty_like(v)
acc = torch.zeros(2, device=dev)
st = torch.cuda.current_stream().cuda_stream
nbytes = 4 * (4 * D + 3) * B
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def timeit(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
ref = lambda: N.lib().tt_cosine_mse_fwd_bwd(u.data_ptr(), v.data_ptr(), tg.data_ptr(), wt.data_ptr(), B, D, ls.data_ptr(), ctypes.c_float(1.0 / B), sc.data_ptr(), du.data_ptr(), dv.data_ptr(), acc.data_ptr(), acc.data_ptr() + 4, st)
ref(); torch.cuda.synchronize(); r_sc, r_du = sc.clone(), du.clone()
names = {0: "lpr16 nv2 rpg2 pf nt (shipped shape)", 1: "lpr16 rpg1 pf", 2: "lpr16 rpg4 pf", 3: "lpr16 rpg2 pf plain-loads",
         4: "lpr8 nv4 rpg1 pf", 5: "lpr8 nv4 rpg2 pf", 6: "lpr32 nv1 rpg2 pf", 7: "lpr32 nv1 rpg4 pf",
         8: "lpr16 rpg2 no-pf", 9: "lpr8 rpg1 no-pf", 10: "lpr4 nv8 rpg1 pf"}
for rnd in range(2):
    t = timeit(ref); print(rnd, "shipped", round(t, 1), "us", round(nbytes / t / 1e3, 1), "GB/s", flush=True)
    for vid, nm in names.items():
        for grid in (8192, 16384, 32768):
            f = lambda: P.cos_probe2(vid, grid, u.data_ptr(), v.data_ptr(), tg.data_ptr(), wt.data_ptr(), B, D, ls.data_ptr(), 1.0 / B, sc.data_ptr(), du.data_ptr(), dv.data_ptr(), acc.data_ptr(), acc.data_ptr() + 4, st)
            t = timeit(f)
            ok = torch.allclose(sc, r_sc, rtol=1e-5, atol=1e-6) and torch.allclose(du, r_du, rtol=1e-4, atol=1e-10)
            print(rnd, f"{nm:38s} grid {grid:6d}", round(t, 1), "us", round(nbytes / t / 1e3, 1), "GB/s", "ok" if ok else "BAD", flush=True)
