"""ctypes binding of libceo_tt.so (include/ceo_tt.h).

The HIP extension is REQUIRED for every CUDA/HIP-device computation of this
package: there is no silent fallback.  If the library cannot be loaded,
:func:`lib` raises ``NativeLibraryError`` with the build command.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch

TT_ABI_VERSION = 6
TT_MAX_CAT = 16
TT_SLOTS_PER_TOWER = 10
TT_NUM_OFFSETS = 2 * TT_MAX_CAT + 2 * TT_SLOTS_PER_TOWER + 1
SLOT_NAMES = ("0.weight", "0.bias", "1.weight", "1.bias", "4.weight", "4.bias",
              "5.weight", "5.bias", "8.weight", "8.bias")

TT_OK = 0
TT_ERR_ARG = -1
TT_ERR_BATCH_TOO_SMALL = -2
TT_ERR_UNSUPPORTED = -3
TT_ERR_WORKSPACE = -4
TT_FLAG_DETERMINISTIC = 1
TT_FLAG_DEFER_LATE = 2
TT_FLAG_LATE_PENDING = 4
TT_STRUCT_MODEL_DESC, TT_STRUCT_BATCH, TT_STRUCT_ADAM_HP, TT_STRUCT_STATE, TT_STRUCT_AR_PEERS = range(5)
TT_STATE_BYTES = 32  # tt_state: step_done, step_cur (int64), loss_sum, pad0 (f32), pad1 (int64)

_PKG_PARENT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# CEO_TT_LIB: diagnostic override (e.g. the -DTT_STAMPS build); the in-tree library otherwise
LIB_PATH = os.environ.get("CEO_TT_LIB") or os.path.join(_PKG_PARENT, "lib", "libceo_tt.so")
EXPORTED = ("tt_abi_version", "tt_struct_size", "tt_stream_copy", "tt_param_count", "tt_param_offsets", "tt_buffer_count",
            "tt_workspace_bytes", "tt_forward", "tt_backward", "tt_backward_ex", "tt_embed_forward",
            "tt_embed_backward", "tt_embed_backward_ex", "tt_train_step", "tt_train_steps", "tt_train_flush", "tt_train_step_ev", "tt_train_step_dp",
            "tt_adam_apply", "tt_cosine_forward", "tt_cosine_mse_fwd_bwd",
            "tt_nce_workspace_bytes", "tt_nce_norms", "tt_nce_forward", "tt_nce_loss", "tt_nce_backward",
            "tt_rank_workspace_bytes", "tt_retrieval_ranks", "tt_step_plan",
            "tt_nce_maxes", "tt_nce_forward_lse", "tt_nce_loss_lse", "tt_nce_backward_lse",
            "tt_range_push", "tt_range_pop", "tt_randperm")


class NativeLibraryError(RuntimeError):
    pass


class TTModelDesc(ctypes.Structure):
    _fields_ = [("n_num", ctypes.c_int32 * 2), ("n_cat", ctypes.c_int32 * 2),
                ("emb_dim", ctypes.c_int32 * 2), ("latent", ctypes.c_int32),
                ("cat_counts", (ctypes.c_int32 * TT_MAX_CAT) * 2),
                ("dropout_p", ctypes.c_float), ("bn_eps", ctypes.c_float),
                ("bn_momentum", ctypes.c_float), ("flags", ctypes.c_int32)]


class TTBatch(ctypes.Structure):
    _fields_ = [("num", ctypes.c_void_p * 2), ("num_ld", ctypes.c_int64 * 2),
                ("cat", ctypes.c_void_p * 2), ("cat_ld", ctypes.c_int64 * 2),
                ("target", ctypes.c_void_p), ("weight", ctypes.c_void_p),
                ("rows", ctypes.c_void_p), ("row0", ctypes.c_int64),
                ("n_rows", ctypes.c_int64), ("cycle", ctypes.c_int64),
                ("t_base", ctypes.c_int64)]


class TTAdamHP(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("eps", ctypes.c_double)]


TT_AR_MAX_RANKS = 16
TT_AR_HANDLE_BYTES = 64


TT_AR_PULL, TT_AR_PUSH = 0, 1  # tt_ar_peers.protocol


class TTArPeers(ctypes.Structure):  # tt_ar_peers
    _fields_ = [("region", ctypes.c_void_p * TT_AR_MAX_RANKS), ("protocol", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


_LIB: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP extension.  Raises if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"HIP extension not built: {LIB_PATH} is missing. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C "
            "ceo-recommender_amd/csrc`).")
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    P, I32, I64, U64, F = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
    D = ctypes.POINTER(TTModelDesc)
    Bt = ctypes.POINTER(TTBatch)
    H = ctypes.POINTER(TTAdamHP)
    sig = {
        "tt_abi_version": (I32, []),
        "tt_range_push": (None, [ctypes.c_char_p]),
        "tt_range_pop": (None, []),
        "tt_randperm": (I32, [I64, U64, P]),
        "tt_struct_size": (I64, [I32]),
        "tt_stream_copy": (I32, [P, P, I64, P]),
        "tt_param_count": (I64, [D]),
        "tt_param_offsets": (I32, [D, ctypes.POINTER(ctypes.c_int64)]),
        "tt_buffer_count": (I64, [D]),
        "tt_workspace_bytes": (I64, [D, I64]),
        "tt_forward": (I32, [D, P, P, P, Bt, I32, U64, I64, P, I64, P, P]),
        "tt_backward": (I32, [D, P, Bt, P, U64, I64, P, I64, P, P]),
        "tt_embed_forward": (I32, [D, P, P, P, Bt, I32, U64, I64, P, I64, P, P]),
        "tt_embed_backward": (I32, [D, P, Bt, P, U64, I64, P, I64, P, P]),
        "tt_backward_ex": (I32, [D, P, P, Bt, P, I32, U64, I64, P, I64, P, P, P, P]),
        "tt_embed_backward_ex": (I32, [D, P, P, Bt, P, I32, U64, I64, P, I64, P, P, P, P]),
        "tt_train_step": (I32, [D, P, P, P, Bt, H, U64, P, P, I64, P, P, P, I32, P]),
        "tt_train_steps": (I32, [D, P, P, P, Bt, H, U64, P, P, I64, P, P, P, I32, P]),
        "tt_train_flush": (I32, [D, P, P, P, Bt, H, P, P, I64, P, P, P, P]),
        "tt_train_step_ev": (I32, [D, P, P, P, Bt, H, U64, P, P, I64, P, P, P, I32, P, ctypes.POINTER(P)]),
        "tt_adam_apply": (I32, [P, P, P, P, I64, H, P, I64, P]),
        "tt_cosine_forward": (I32, [P, P, I64, I32, P, P, P]),
        "tt_cosine_mse_fwd_bwd": (I32, [P, P, P, P, I64, I32, P, F, P, P, P, P, P, P]),
        "tt_nce_workspace_bytes": (I64, [I64, I64, I32]),
        "tt_nce_norms": (I32, [P, P, I64, I64, I32, P, P]),
        "tt_nce_forward": (I32, [P, P, I64, I64, I32, I64, F, P, P, I64, P, P]),
        "tt_nce_loss": (I32, [I64, I64, I32, I64, I64, F, P, I64, P, P, P, P]),
        "tt_nce_backward": (I32, [P, P, I64, I64, I32, I64, I64, F, P, I64, P, P, P]),
        "tt_nce_maxes": (I32, [P, P, I64, I64, I32, I64, F, P, I64, P, P]),
        "tt_nce_forward_lse": (I32, [P, P, I64, I64, I32, I64, F, P, P, I64, P, P]),
        "tt_nce_loss_lse": (I32, [I64, I64, I32, I64, I64, P, I64, P, P, P, P, P]),
        "tt_nce_backward_lse": (I32, [P, P, I64, I64, I32, I64, I64, F, P, I64, P, P, P]),
        "tt_rank_workspace_bytes": (I64, [I64]),
        "tt_retrieval_ranks": (I32, [P, P, I64, I64, I32, I64, P, I64, P, P]),
        "tt_ar_region_bytes": (I64, [I64]),
        "tt_step_plan": (I32, [ctypes.POINTER(TTModelDesc), I64, P, I32]),
        "tt_ar_alloc": (I32, [I64, ctypes.POINTER(P), P]),
        "tt_ar_open": (I32, [P, ctypes.POINTER(P)]),
        "tt_ar_close": (I32, [P]),
        "tt_ar_free": (I32, [P]),
        "tt_ar_reset": (I32, [P, I64, P]),
        "tt_ar_allreduce_adam": (I32, [ctypes.POINTER(TTArPeers), I32, I32, I64, P, P, P, P, P, H, P, I64, P, I64, P]),
        "tt_train_step_dp": (I32, [D, P, P, P, Bt, H, U64, P, P, I64, P, P, P, ctypes.POINTER(TTArPeers), I32, I32,
                                   I32, P, I64, P]),
        "tt_triplet_workspace_bytes": (I64, [I64, I64, I32]),
        "tt_triplet_forward": (I32, [P, P, I64, I64, I32, I64, F, I64, P, I64, P, P, P, P]),
        "tt_triplet_backward": (I32, [P, P, I64, I64, I32, I64, I64, P, P, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name, None)
        if fn is None:
            if os.environ.get("CEO_TT_LIB"):  # a diagnostic build of an older ABI: bind what it has
                continue
            raise NativeLibraryError(f"{LIB_PATH} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    v = L.tt_abi_version()
    if v != TT_ABI_VERSION:
        raise NativeLibraryError(f"{LIB_PATH}: ABI version {v}, expected {TT_ABI_VERSION}")
    for which, st in ((TT_STRUCT_MODEL_DESC, TTModelDesc), (TT_STRUCT_BATCH, TTBatch), (TT_STRUCT_ADAM_HP, TTAdamHP),
                      (TT_STRUCT_AR_PEERS, TTArPeers)):
        if L.tt_struct_size(which) != ctypes.sizeof(st):
            raise NativeLibraryError(f"{LIB_PATH}: sizeof({st.__name__}) = {ctypes.sizeof(st)} here, "
                                     f"{L.tt_struct_size(which)} in the library")
    _LIB = L
    return L


def check(rc: int, what: str, batch: int = 0, width: int = 64):
    if rc == TT_OK:
        return
    if rc == TT_ERR_BATCH_TOO_SMALL:
        # torch.nn.functional.batch_norm's message (reference behaviour)
        raise ValueError(f"Expected more than 1 value per channel when training, "
                         f"got input size torch.Size([{batch}, {width}])")
    if rc == TT_ERR_ARG:
        raise ValueError(f"{what}: invalid argument")
    if rc == TT_ERR_UNSUPPORTED:
        raise NotImplementedError(f"{what}: shape not supported by the fused HIP kernels")
    if rc == TT_ERR_WORKSPACE:
        raise RuntimeError(f"{what}: workspace too small")
    raise RuntimeError(f"{what}: HIP error {rc}")


def make_desc(n_num: Sequence[int], cat_counts: Sequence[Sequence[int]],
              emb_dim: Sequence[int], latent: int, dropout_p: float = 0.1,
              bn_eps: float = 1e-5, bn_momentum: float = 0.1, flags: int = 0) -> TTModelDesc:
    d = TTModelDesc()
    for t in range(2):
        if len(cat_counts[t]) > TT_MAX_CAT:
            raise NotImplementedError(f"at most {TT_MAX_CAT} categorical columns per tower")
        d.n_num[t] = int(n_num[t])
        d.n_cat[t] = len(cat_counts[t])
        d.emb_dim[t] = int(emb_dim[t])
        for j, c in enumerate(cat_counts[t]):
            d.cat_counts[t][j] = int(c)
    d.latent = int(latent)
    d.dropout_p = float(dropout_p)
    d.bn_eps = float(bn_eps)
    d.bn_momentum = float(bn_momentum)
    d.flags = int(flags)
    return d


def deterministic_default() -> bool:
    """Deterministic reductions when torch's deterministic-algorithms mode is
    on (torch.use_deterministic_algorithms(True)) or CEO_TT_DETERMINISTIC=1."""
    env = os.environ.get("CEO_TT_DETERMINISTIC")
    if env is not None:
        return env not in ("", "0")
    return bool(torch.are_deterministic_algorithms_enabled())


def set_deterministic(desc: TTModelDesc, on: bool) -> TTModelDesc:
    if on:
        desc.flags |= TT_FLAG_DETERMINISTIC
    else:
        desc.flags &= ~TT_FLAG_DETERMINISTIC
    return desc


def step_plan(desc: TTModelDesc, batch: int) -> dict:
    """How one fused training step runs at this batch size (tt_step_plan)."""
    info = (ctypes.c_int32 * 8)()
    check(lib().tt_step_plan(ctypes.byref(desc), int(batch), info, 8), "tt_step_plan")
    return {"folded_bn0_backward": bool(info[0]), "top_rows": info[1], "mid_rows": info[2], "kernels": info[3],
            "top_pair": bool(info[4]), "ndt": info[5], "fwd_rows": info[6], "train_top_rows": info[7]}


def param_count(desc: TTModelDesc) -> int:
    n = lib().tt_param_count(ctypes.byref(desc))
    if n < 0:
        check(int(n), "tt_param_count")
    return int(n)


def param_offsets(desc: TTModelDesc):
    out = (ctypes.c_int64 * TT_NUM_OFFSETS)()
    check(lib().tt_param_offsets(ctypes.byref(desc), out), "tt_param_offsets")
    return list(out)


def workspace_bytes(desc: TTModelDesc, max_batch: int) -> int:
    n = lib().tt_workspace_bytes(ctypes.byref(desc), int(max_batch))
    if n < 0:
        check(int(n), "tt_workspace_bytes")
    return int(n)


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def make_batch(f_num, f_cat, c_num, c_cat, target=None, weight=None, rows=None,
               row0=0, n_rows=None, cycle=0, t_base=0) -> TTBatch:
    """Describe a batch over (possibly dataset-resident) device tensors."""
    b = TTBatch()
    for t, (num, cat) in enumerate(((f_num, f_cat), (c_num, c_cat))):
        if num is not None and num.numel() > 0:
            b.num[t] = num.data_ptr()
            b.num_ld[t] = num.stride(0)
        if cat is not None and cat.dim() == 2 and cat.shape[1] > 0:
            b.cat[t] = cat.data_ptr()
            b.cat_ld[t] = cat.stride(0)
    b.target = ptr(target)
    b.weight = ptr(weight)
    b.rows = ptr(rows)
    b.row0 = int(row0)
    b.n_rows = int(n_rows if n_rows is not None else f_num.shape[0])
    b.cycle = int(cycle)
    b.t_base = int(t_base)
    return b


def adam_hp(lr: float, betas=(0.9, 0.999), eps: float = 1e-8) -> TTAdamHP:
    h = TTAdamHP()
    h.lr, h.beta1, h.beta2, h.eps = float(lr), float(betas[0]), float(betas[1]), float(eps)
    return h


class trace_range:
    """``with trace_range("name"):`` -- a roctx range (tt_range_push / pop)
    around host code, e.g. bench.py's timed region and graph replays."""

    def __init__(self, name: str):
        self.name = name.encode()

    def __enter__(self):
        lib().tt_range_push(self.name)
        return self

    def __exit__(self, *exc):
        lib().tt_range_pop()
        return False


def randperm(n: int, seed: int, pin: bool = False):
    """torch.randperm(n, generator=torch.Generator().manual_seed(seed)) on the
    host, bit for bit (tt_randperm: the same mt19937 Fisher-Yates with the
    swap targets prefetched).  None when the library does not cover n."""
    import torch
    out = torch.empty(n, dtype=torch.int64, pin_memory=pin)
    rc = lib().tt_randperm(int(n), int(seed) & ((1 << 64) - 1), out.data_ptr() if n else None)
    if rc == TT_ERR_UNSUPPORTED:
        return None
    check(rc, "tt_randperm")
    return out
