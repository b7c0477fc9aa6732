"""Training entry point (drop-in for the reference ``training.py:15-64``).

``train_model(train_loader, val_loader, metadata, config)`` keeps the
reference signature, stdout lines and semantics: the model is built with the
same RNG draws, batches come in exactly the order the DataLoader would yield
them (its RandomSampler is driven from the same global generator), the last
partial batch is kept, Adam(lr=config.LEARNING_RATE), and every 5th epoch
prints the mean of the batch losses.

On a HIP device the loop runs on the fused engine (``engine.FusedTrainer``):
the dataset behind a ``CEOFirmDataset`` loader is uploaded to HBM once and
every step is one C-ABI call (six kernels) with no per-step host sync.  Any
other loader is consumed batch by batch (``.to(DEVICE)``) through the same
fused step.  On CPU the reference loop runs with ATen ops.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.optim as optim
from torch.utils.data import DataLoader

from .config import Config
from .engine import DATA_KEYS, FusedTrainer
from .model import CEOFirmMatcher


def sampler_batches(loader: DataLoader) -> List[List[int]]:
    """Index lists of one epoch of ``loader``, consuming the global RNG exactly
    as ``iter(loader)`` does (torch 2.10 ``_BaseDataLoaderIter.__init__`` draws
    the worker base seed first; the RandomSampler draws its seed lazily)."""
    torch.empty((), dtype=torch.int64).random_(generator=loader.generator)
    return [list(b) for b in loader.batch_sampler]


def epoch_order_plan(loader: DataLoader, pin: bool = False) -> Optional[Callable[[], Tuple[torch.Tensor, List[int]]]]:
    """One epoch's batch order of ``loader`` as ONE int64 index tensor (the
    batches concatenated) and the batch sizes -- the order and global-RNG
    consumption of ``sampler_batches`` without Python index lists (at 1M
    pairs those took 80 ms per epoch, 25x the epoch's fused steps).

    Consumes the global RNG now, exactly as ``iter(loader)`` does, and
    returns a thunk that builds the order: for the default ``RandomSampler``
    (its own generator seeded from that draw) the thunk depends on nothing
    else, so epochs' permutations can be built on worker threads.  Covers the
    samplers ``DataLoader(shuffle=...)`` builds (torch 2.10 ``RandomSampler``
    without replacement over the whole dataset, or ``SequentialSampler``)
    under the default ``BatchSampler``; None for any other sampler (the
    caller then uses ``sampler_batches``).  ``pin``: the thunk returns the
    order in pinned host memory (for an asynchronous upload)."""
    from torch.utils.data import BatchSampler, RandomSampler, SequentialSampler
    bsamp = loader.batch_sampler
    if type(bsamp) is not BatchSampler:
        return None
    samp = bsamp.sampler
    n = len(loader.dataset)
    if type(samp) is RandomSampler:
        if samp.replacement or samp.num_samples != n or len(samp.data_source) != n:
            return None
    elif type(samp) is not SequentialSampler:
        return None
    bs = bsamp.batch_size
    sizes = [bs] * (n // bs)
    if n % bs and not bsamp.drop_last:
        sizes.append(n % bs)
    total = sum(sizes)
    torch.empty((), dtype=torch.int64).random_(generator=loader.generator)  # the iterator's base seed
    if type(samp) is SequentialSampler:
        return lambda: (torch.arange(total, dtype=torch.int64), sizes)
    if samp.generator is not None:
        # a caller-owned generator: its draws are sequential, made now (the
        # exhausted iterator's trailing randperm(n)[:0] advances it too)
        order = torch.randperm(n, generator=samp.generator)
        torch.randperm(n, generator=samp.generator)
        return lambda: (order[:total], sizes)
    seed = int(torch.empty((), dtype=torch.int64).random_().item())  # RandomSampler.__iter__

    def build():
        order = host_randperm(n, seed, pin)
        return order[:total], sizes
    return build


_RANDPERM_AGREES = None


def native_randperm_agrees() -> bool:
    """Whether tt_randperm (a restatement of torch 2.10's CPU randperm:
    mt19937 Fisher-Yates) still equals this process's ``torch.randperm``:
    compared once per process on a few sizes and seeds that cover the small-n
    and the Fisher-Yates paths.  A torch whose randperm draws otherwise makes
    host_randperm fall back to torch (with a warning) instead of silently
    training in another order than the reference's DataLoader."""
    global _RANDPERM_AGREES
    if _RANDPERM_AGREES is None:
        from . import _native as N
        agree = True
        try:
            for n, seed in ((0, 1), (1, 3), (7, 0), (1000, 12345), (70_001, 2 ** 40 + 7)):
                got = N.randperm(n, seed, False)
                if got is None:
                    continue
                gen = torch.Generator()
                gen.manual_seed(seed)
                if not torch.equal(got, torch.randperm(n, generator=gen)):
                    agree = False
                    break
        except N.NativeLibraryError:
            agree = True  # (host_randperm then uses torch anyway)
        if not agree:
            import warnings
            warnings.warn(f"tt_randperm differs from torch {torch.__version__}'s randperm: "
                          "epoch orders are drawn with torch.randperm")
        _RANDPERM_AGREES = agree
    return _RANDPERM_AGREES


def host_randperm(n: int, seed: int, pin: bool = False) -> torch.Tensor:
    """``torch.randperm(n, generator=Generator().manual_seed(seed))``, the
    RandomSampler's draw, built by the library's tt_randperm (the same
    mt19937 Fisher-Yates, bit for bit, with the swap targets prefetched: the
    sequential torch loop is 23 ns per pair, a cache miss per swap); torch's
    own randperm where the library does not cover n or is not built (host
    work, identical result), or where this torch's randperm no longer draws
    what tt_randperm restates (checked once per process:
    ``native_randperm_agrees``)."""
    from . import _native as N
    order = None
    if native_randperm_agrees():
        try:
            order = N.randperm(n, seed, pin)
        except N.NativeLibraryError:
            order = None
    if order is None:
        gen = torch.Generator()
        gen.manual_seed(seed)
        order = torch.randperm(n, generator=gen)
        if pin:
            order = order.pin_memory()
    return order


def dp_epoch_order_plan(loader: DataLoader, epoch: int, rank: int, world: int,
                        pin: bool = False) -> Callable[[], Tuple[torch.Tensor, List[int]]]:
    """Data-parallel counterpart of ``epoch_order_plan``: this rank's batch
    order for ``epoch`` under DistributedSampler semantics
    (``distributed.rank_epoch_order``: permutation from seed + epoch, padded
    to ceil(N / world) per rank).  A loader that already holds a
    ``DistributedSampler`` keeps its shuffle / seed / drop_last (its
    num_replicas and rank must be this process group's); any other loader is
    sharded as ``DistributedSampler(dataset)`` would (shuffle as the loader's
    sampler, seed 0).  Batches of the loader's batch size, the last partial
    one kept unless the loader drops it.  Consumes the global RNG as
    ``iter(loader)`` does (the iterator's base seed) so the draws after
    training match the single-process run's."""
    from torch.utils.data import RandomSampler
    from torch.utils.data.distributed import DistributedSampler
    from .distributed import rank_epoch_order
    samp = loader.sampler
    n = len(loader.dataset)
    if isinstance(samp, DistributedSampler):
        if (samp.num_replicas, samp.rank) != (world, rank):
            raise ValueError(f"DistributedSampler(num_replicas={samp.num_replicas}, rank={samp.rank}) in a "
                             f"process group of {world} (this rank {rank})")
        shuffle, seed, drop = samp.shuffle, samp.seed, samp.drop_last
    else:
        shuffle, seed, drop = isinstance(samp, RandomSampler), 0, False
    bs = loader.batch_size or 1
    drop_batch = bool(getattr(loader.batch_sampler, "drop_last", False))
    torch.empty((), dtype=torch.int64).random_(generator=loader.generator)  # the iterator's base seed

    def build():
        order = rank_epoch_order(n, epoch, rank, world, shuffle=shuffle, seed=seed, drop_last=drop)
        m = order.numel()
        sizes = [bs] * (m // bs) + ([m % bs] if m % bs and not drop_batch else [])
        order = order[:sum(sizes)]
        return (order.pin_memory() if pin else order), sizes
    return build


def epoch_order(loader: DataLoader) -> Optional[Tuple[torch.Tensor, List[int]]]:
    """``epoch_order_plan`` built at once: (order, batch sizes) or None."""
    plan = epoch_order_plan(loader)
    return None if plan is None else plan()


def _resident_data(loader: DataLoader) -> Optional[Dict[str, torch.Tensor]]:
    ds = loader.dataset
    data = getattr(ds, "data", None)
    if not isinstance(data, dict) or any(k not in data for k in DATA_KEYS):
        return None
    if loader.batch_sampler is None or getattr(loader, "_dataset_kind", 0) != 0:
        return None
    if loader.collate_fn is not torch.utils.data.default_collate:
        return None
    return {k: data[k] for k in DATA_KEYS}


def _process_group():
    """(group, rank, world) of an initialised torch.distributed job with more
    than one rank, else (None, 0, 1)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.group.WORLD, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def _select_local_device(config: Config):
    """One process per GPU: a device without an index resolves to the
    current one, so make that LOCAL_RANK's (when such a device exists; ranks
    sharing one GPU in a rehearsal keep theirs)."""
    import os
    dev = torch.device(config.DEVICE)
    local = os.environ.get("LOCAL_RANK")
    if dev.type == "cuda" and dev.index is None and local is not None:
        if int(local) < torch.cuda.device_count():
            torch.cuda.set_device(int(local))


def _mean_over_ranks(x: float, pg, device) -> float:
    import torch.distributed as dist
    dev = device if dist.get_backend(pg) == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, group=pg)
    return float(t.item()) / dist.get_world_size(pg)


def train_model(train_loader: DataLoader, val_loader: DataLoader,
                metadata: Dict[str, int], config: Config) -> Optional[CEOFirmMatcher]:
    """Train the CEOFirmMatcher model (reference training.py:15-64).

    Under an initialised ``torch.distributed`` job with world size > 1 (one
    process per GPU, ``torchrun``) this is the reference loop under
    DistributedDataParallel (BASELINE cfg 4): each rank runs on
    its LOCAL_RANK device, trains on its DistributedSampler shard of every
    epoch (``dp_epoch_order_plan``) with local BatchNorm statistics, starts
    from rank 0's parameters, and averages the gradient over the ranks every
    step (inside the fused step's reduction, the peer-memory exchange, or an
    RCCL / gloo all-reduce); rank 0 prints the lines, with the epoch loss
    averaged over the ranks."""
    pg, rank, world = _process_group()
    if pg is not None:
        _select_local_device(config)
    model = CEOFirmMatcher(metadata, config).to(config.DEVICE)
    if rank == 0:
        print(f"Starting training on {config.DEVICE} for {config.EPOCHS} epochs...")
    if torch.device(config.DEVICE).type == "cuda":
        return _train_fused(model, train_loader, config, pg)
    return _train_cpu(model, train_loader, config, pg)


train = train_model  # the north-star name


# epochs whose batch order is built ahead on worker threads (one thread and
# one pinned order each: 80 MB at 10M pairs).  torch.randperm of the
# reference's sampler is sequential (0.23 s per 10M-pair epoch per thread)
# against 33 ms of fused steps, so as many threads as the process's CPU share
# allows (the GPU box gives each GPU 16), keeping two for the launching thread
_ORDER_AHEAD_MAX = 12


def _usable_cpus() -> int:
    import os
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return n


def _order_ahead() -> int:
    return max(2, min(_ORDER_AHEAD_MAX, _usable_cpus() - 2))


class _EpochSteps:
    """An epoch's full batches as hipGraph replays.  The epoch's order lives
    in one persistent device buffer (refilled before each epoch, stream
    ordered), batch j of every epoch is rows[j*bs : (j+1)*bs], and the steps
    run in cycle mode: cycle = the epoch's step count (the partial batch, a
    host-mode step, takes the last slot), t_base = the device step counter at
    the start of training, so the batch index ((t-1-t_base) % cycle) is j in
    every epoch and the captured launches replay unchanged.  Epoch 0 runs
    eagerly (first launches load the kernels); the graphs, chunks of 16 steps
    (the bench's measured best), are captured after it.  Any capture failure
    keeps eager cycle-mode steps."""

    CHUNK = 16

    def __init__(self, trainer: FusedTrainer, rows: torch.Tensor, bs: int, n_full: int, cycle: int, t_base: int):
        self.tr, self.rows, self.bs, self.n_full, self.cycle, self.t_base = trainer, rows, bs, n_full, cycle, t_base
        self.graphs = None
        self.eager = False

    def _step(self):
        self.tr.step_cycle(self.rows, self.bs, self.cycle, t_base=self.t_base)

    def _capture(self):
        try:
            graphs = []
            sizes = [self.CHUNK] * (self.n_full // self.CHUNK) + ([self.n_full % self.CHUNK] if self.n_full % self.CHUNK else [])
            made = {}
            for k in sizes:  # one graph per distinct chunk length
                if k not in made:
                    g = torch.cuda.CUDAGraph()
                    # thread_local: the order workers pin host memory meanwhile
                    with torch.cuda.graph(g, capture_error_mode="thread_local"):  # recorded only
                        for _ in range(k):
                            self._step()
                    made[k] = g
                graphs.append(made[k])
            self.tr.steps_host -= sum(made)  # captured launches are not steps taken
            self.graphs = graphs
        except Exception:  # noqa: BLE001 -- capture unsupported here: eager steps
            self.eager = True
            import ctypes
            try:  # the failed capture's error stays pending for the next launch check
                ctypes.CDLL("libamdhip64.so").hipGetLastError()
            except OSError:
                pass
        pg = self.tr.pg
        if pg is not None:  # data parallel: every rank replays, or none does
            import torch.distributed as dist
            dev = self.tr.device if dist.get_backend(pg) == "nccl" else "cpu"
            ok = torch.tensor([0 if self.eager else 1], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=pg)
            if int(ok.item()) == 0:
                self.eager, self.graphs = True, None

    def run(self, epoch: int):
        if epoch == 0 or self.eager:
            for _ in range(self.n_full):
                self._step()
            return
        if self.graphs is None:
            self._capture()
            if self.eager:
                return self.run(epoch)
        for g in self.graphs:
            g.replay()
        self.tr.steps_host += self.n_full


def _dp_loader(loader: DataLoader, rank: int, world: int) -> DataLoader:
    """Any map-style loader as its data-parallel shard: the same dataset,
    batch size and collate behind a DistributedSampler (shuffle as the
    loader's sampler), unless it already holds one."""
    from torch.utils.data import RandomSampler
    from torch.utils.data.distributed import DistributedSampler
    if isinstance(loader.sampler, DistributedSampler):
        return loader
    samp = DistributedSampler(loader.dataset, num_replicas=world, rank=rank,
                              shuffle=isinstance(loader.sampler, RandomSampler))
    return DataLoader(loader.dataset, batch_size=loader.batch_size, sampler=samp, collate_fn=loader.collate_fn,
                      drop_last=loader.drop_last, num_workers=loader.num_workers)


def _train_fused(model: CEOFirmMatcher, loader: DataLoader, config: Config, pg=None) -> CEOFirmMatcher:
    dev = model.logit_scale.device
    bs = loader.batch_size or 1
    rank, world = (0, 1) if pg is None else (pg.rank(), pg.size())
    trainer = FusedTrainer(model, lr=config.LEARNING_RATE, max_batch=max(bs, 2), process_group=pg)
    data = _resident_data(loader)
    if data is not None:
        trainer.set_data(data)
    elif pg is not None:
        loader = _dp_loader(loader, rank, world)
    # the epochs' batch orders: global-RNG draws in epoch order, the
    # permutations built on worker threads a few epochs ahead (torch.randperm
    # of the reference's sampler is sequential: 23 ns per pair, 10x an
    # epoch's fused steps), so the device rarely waits for the host
    pool, ahead, depth = None, [], min(_order_ahead(), config.EPOCHS)
    pin = torch.cuda.is_available()

    def plan_of(epoch):
        if pg is not None:
            return dp_epoch_order_plan(loader, epoch, rank, world, pin)
        return epoch_order_plan(loader, pin)
    plan = plan_of(0) if data is not None and config.EPOCHS > 0 else None
    nxt = None
    if plan is not None:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=depth)
        ahead.append(pool.submit(plan))
        for e in range(1, depth):
            ahead.append(pool.submit(plan_of(e)))
        nxt = ahead.pop(0).result()
    runner = None
    if nxt is not None:
        # DataLoader(shuffle=...) epochs all have the same batch sizes: full
        # batches replayed from graphs (_EpochSteps), the partial one eager
        sizes0 = nxt[1]
        n_full = sum(1 for b in sizes0 if b == bs)
        if n_full and sizes0[:n_full] == [bs] * n_full:
            rows_dev = torch.empty(len(nxt[0]), dtype=torch.int64, device=dev)
            runner = _EpochSteps(trainer, rows_dev, bs, n_full, len(sizes0), trainer.steps_done())
            if pg is not None and not _dp_graphs_ok(trainer):
                runner.eager = True  # a host collective per step (gloo) cannot be captured
    for epoch in range(config.EPOCHS):
        model.train()
        n_batches = 0
        if data is not None:
            if nxt is not None:
                order, sizes = nxt
            else:
                batches = sampler_batches(loader)
                order = torch.tensor([i for b in batches for i in b], dtype=torch.int64)
                sizes = [len(b) for b in batches]
            if runner is not None:
                runner.rows.copy_(order, non_blocking=True)
                runner.run(epoch)
                for bsz in sizes[runner.n_full:]:  # the partial batch: host mode, the cycle's last slot
                    trainer.step(runner.rows, runner.n_full * bs, bsz)
                n_batches = len(sizes)
            else:
                rows = order.to(dev, non_blocking=True)
                off = 0
                for bsz in sizes:
                    trainer.step(rows, off, bsz)
                    off += bsz
                    n_batches += 1
            # keep `depth` epochs' orders in flight (host RNG only: the fused steps
            # draw nothing from it); the next one is usually built already
            if pool is not None:
                if epoch + depth < config.EPOCHS:
                    ahead.append(pool.submit(plan_of(epoch + depth)))
                nxt = ahead.pop(0).result() if ahead else None
        else:
            if pg is not None and hasattr(loader.sampler, "set_epoch"):
                loader.sampler.set_epoch(epoch)
            for batch in loader:
                batch = {k: v.to(dev) for k, v in batch.items()}
                trainer.set_data(batch)
                trainer.step(None, 0, batch["target"].shape[0])
                n_batches += 1
        if epoch % 5 == 0:
            avg_loss = trainer.pop_loss_sum() / max(n_batches, 1)
            if pg is not None:
                avg_loss = _mean_over_ranks(avg_loss, pg, dev)
            if rank == 0:
                print(f"Epoch {epoch}: Avg Train Loss = {avg_loss:.4f}")
        else:
            trainer.pop_loss_sum(read=False)
    if pool is not None:
        pool.shutdown()
    trainer.check_exchange()
    model._trainer = trainer  # keeps optimizer state reachable for callers/tests
    return model


def _dp_graphs_ok(trainer: FusedTrainer) -> bool:
    """Data-parallel steps can be captured when their exchange is a kernel
    (peer memory) or an RCCL collective; a gloo all-reduce is host work."""
    import torch.distributed as dist
    return trainer.peer is not None or dist.get_backend(trainer.pg) == "nccl"


def _train_cpu(model: CEOFirmMatcher, loader: DataLoader, config: Config, pg=None) -> CEOFirmMatcher:
    """The reference loop with ATen ops; under a process group the DDP form:
    rank 0's initial parameters everywhere, the rank's DistributedSampler
    shard, local BatchNorm statistics, gradients averaged over the ranks
    (one flat all-reduce) before every Adam step."""
    from .distributed import average_gradients_, broadcast_state_
    params = list(model.parameters())
    if pg is not None:
        loader = _dp_loader(loader, pg.rank(), pg.size())
        flat = torch.cat([p.detach().reshape(-1) for p in params])
        broadcast_state_(flat, None, pg)
        with torch.no_grad():
            off = 0
            for p in params:
                p.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()
    optimizer = optim.Adam(model.parameters(), lr=config.LEARNING_RATE)
    for epoch in range(config.EPOCHS):
        model.train()
        total_loss = 0.0
        if pg is not None:
            loader.sampler.set_epoch(epoch)
        for batch in loader:
            optimizer.zero_grad()
            preds = model(batch['firm_numeric'], batch['firm_cat'], batch['ceo_numeric'], batch['ceo_cat'])
            loss = (batch['weights'] * (preds - batch['target']) ** 2).mean()
            loss.backward()
            if pg is not None:  # DDP: one flat all-reduce (average) of every gradient
                g = torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.zeros(p.numel())
                               for p in params])
                average_gradients_(g, pg)
                off = 0
                for p in params:
                    p.grad = g[off:off + p.numel()].view_as(p).clone()
                    off += p.numel()
            optimizer.step()
            total_loss += loss.item()
        avg_loss = total_loss / len(loader)
        if pg is not None:
            avg_loss = _mean_over_ranks(avg_loss, pg, "cpu")
        if epoch % 5 == 0 and (pg is None or pg.rank() == 0):
            print(f"Epoch {epoch}: Avg Train Loss = {avg_loss:.4f}")
    return model
