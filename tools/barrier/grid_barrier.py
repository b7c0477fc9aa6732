"""Device time per grid barrier (tools/barrier/grid_barrier.hip) at 64 /
128 / 256 / 512 workgroups: launches of K = 0 and K = 200 barriers timed with
HIP events, (T(K) - T(0)) / K, median of 5.  Review r05 item 7."""
import ctypes
import os
import statistics

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
P = ctypes.CDLL(os.path.join(HERE, "grid_barrier.so"))
P.grid_barrier_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
dev = torch.device("cuda:0")
bar = torch.zeros(P.grid_barrier_bytes() // 4, dtype=torch.int32, device=dev)
pub = torch.zeros(512 * 256 * 16, device=dev)
st = torch.cuda.current_stream().cuda_stream
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
BOUND = 5_000_000  # 50 ms per wait


def launch(nb, iters, xcd, ppt):
    bar.zero_()
    e0.record()
    rc = P.grid_barrier_probe(bar.data_ptr(), pub.data_ptr(), ppt, nb, iters, xcd, BOUND, st)
    e1.record()
    torch.cuda.synchronize()
    assert rc == 0 and int(bar[8 * 32 + 64]) == 0, "a barrier wait timed out"  # err word
    return e0.elapsed_time(e1) * 1e3


K = 200
print("form  WGs  publish_B/WG  us_per_barrier")
for ppt, label in ((0, 0), (16, 16384)):
    for xcd in (1, 0):
        for nb in (64, 128, 256, 512):
            launch(nb, K, xcd, ppt)
            ts = [(launch(nb, K, xcd, ppt) - launch(nb, 0, xcd, ppt)) / K for _ in range(5)]
            print(f"{'xcd' if xcd else 'flat':4s} {nb:4d} {label:8d} {statistics.median(ts):8.2f}  "
                  f"(min {min(ts):.2f} max {max(ts):.2f})", flush=True)
