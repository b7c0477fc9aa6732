"""Time the copy variants of copy_probe.hip and tt_stream_copy (2 GiB, read+write bytes / time)."""
import ctypes, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "ceo-recommender_amd"))
from ceo_firm_matching import _native as N
P = ctypes.CDLL(os.path.join(ROOT, "tools", "copyprobe", "copy_probe.so"))
P.copy_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
dev = torch.device("cuda:0")
src = torch.ones(1 << 29, device=dev); dst = torch.empty_like(src); nb = src.numel() * 4
st = torch.cuda.current_stream().cuda_stream
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
def timeit(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return 2 * nb / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
for rnd in range(2):
    for v in range(8):
        print(rnd, "variant", v, round(timeit(lambda: P.copy_probe(src.data_ptr(), dst.data_ptr(), nb, v, st)), 1))
    for v in (8, 9):  # read-only: bytes read / time
        print(rnd, "read variant", v, round(timeit(lambda: P.copy_probe(src.data_ptr(), dst.data_ptr(), nb, v, st)) / 2, 1))
    print(rnd, "tt_stream_copy", round(timeit(lambda: N.lib().tt_stream_copy(src.data_ptr(), dst.data_ptr(), nb, st)), 1))
    print(rnd, "torch copy_", round(timeit(lambda: dst.copy_(src)), 1))
