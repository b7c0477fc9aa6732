"""Fused, device-resident training engine for CEOFirmMatcher.

One ``step`` = the reference's training.py:44-57 (zero_grad, forward,
weighted MSE, backward, Adam.step) as six HIP kernels enqueued by one C-ABI
call (``tt_train_step``): no per-step host sync, no ``.item()``, no per-sample
collate.  The dataset lives in HBM; a batch is a slice of a row-index
permutation that the first kernel gathers from.

Data parallel (one process per GPU, ``torch.distributed`` over RCCL) --
DistributedDataParallel semantics with per-rank (local) BatchNorm
statistics: with the peer-memory exchange (``distributed.PeerExchange``) the
mean over ranks happens inside the step's last kernel (``tt_train_step_dp``:
the gradient reduction publishes, waits for the peers and applies Adam);
otherwise the step stops after the gradient reduction (``apply_adam=0``), the
flat fp32 gradient is all-reduced (AVG, one call per step), and
``tt_adam_apply`` finishes the step.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _native as N
from .distributed import PeerExchange, average_gradients_, broadcast_state_, choose_exchange_form, world_of
from .model import CEOFirmMatcher, check_category_codes

DATA_KEYS = ("firm_numeric", "firm_cat", "ceo_numeric", "ceo_cat", "target", "weights")


class FusedTrainer:
    def __init__(self, model: CEOFirmMatcher, lr: float = 4e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_batch: int = 256, seed: Optional[int] = None, process_group=None,
                 deterministic: Optional[bool] = None, defer_late: bool = False):
        dev = model.logit_scale.device
        if dev.type != "cuda":
            raise RuntimeError("FusedTrainer needs the model on a HIP device")
        self.model = model
        self.device = dev
        # bitwise-repeatable steps (TT_FLAG_DETERMINISTIC; None: the model's
        # setting, which follows torch.use_deterministic_algorithms)
        self.deterministic = deterministic
        self.arena = model.bind_arena()
        self.desc = self.arena.desc
        self.lib = N.lib()
        n = self.arena.params.numel()
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        # tt_state: step_done, step_cur (int64), loss_sum (f32), pad
        self.state = torch.zeros(4, dtype=torch.int64, device=dev)
        self.hp = N.adam_hp(lr, betas, eps)
        self.seed = (int(torch.cuda.initial_seed()) if seed is None else int(seed)) & ((1 << 63) - 1)
        self.pg = process_group
        # data-parallel step (grad -> all-reduce -> Adam) whenever a process
        # group is given, also at world size 1 (exercises the N > 1 path)
        self.dp = process_group is not None
        self.world = world_of(process_group) if self.dp else 1
        if self.world > 1:  # DDP construction semantics: rank 0's state everywhere
            broadcast_state_(self.arena.params, self.arena.buffers, process_group)
        # one-launch gradient exchange + Adam over peer memory when every rank
        # can map it and it beats the collective (else the RCCL all-reduce)
        self.peer = PeerExchange.create(n, process_group, dev) if self.dp else None
        # exchange inside the step's reduction (None: not decided yet; the
        # first data-parallel step validates it against the two-launch form on
        # this topology, _validate_fused_exchange).  Only with one rank per
        # GPU: a rank spinning in its reduction holds LDS and wave slots that a
        # co-located rank's forward kernels need, so ranks sharing a device
        # (rehearsals) keep the two-launch form unless CEO_TT_FUSED_EX=1
        # (tests with small kernels: the bitwise check alone then decides,
        # not the timing); CEO_TT_FUSED_EX=0 turns it off
        import os
        fx = os.environ.get("CEO_TT_FUSED_EX")
        self.fused_exchange = None if self.peer is not None and fx != "0" and (
            self.peer.co_ranks == 1 or fx == "1") else False
        # (fused, two-launch) device us per step, MAX over ranks, measured by
        # _validate_fused_exchange on the first data-parallel step
        self.fused_vs_two_launch_us = None
        self.exchange_form_us = None  # {form: us}, all forms timed by the validation
        self.exchange_form = None     # the form it chose (engine._validate_fused_exchange)
        # TT_FLAG_DEFER_LATE: each single-GPU step leaves the late half of its
        # reduction (W4, BN1 affine, W8, logit_scale, the loss) to the next
        # step's first kernel; flush() finishes it (run automatically before
        # the loss, the parameters or a step of another batch size are used)
        self.defer_late = bool(defer_late)
        self._late_rows = 0       # batch rows of the step whose late half is pending (0: none)
        self._late_batch = None   # that step's tt_batch (for tt_train_flush)
        self._no_defer = set()    # batch sizes whose geometry has no deferred form (TT_ERR_UNSUPPORTED)
        self.max_batch = 0
        self.ws = None
        self.ensure_batch(max_batch)
        self.data: Dict[str, torch.Tensor] = {}
        self.steps_host = 0

    # ------------------------------------------------------------------ setup
    def ensure_batch(self, max_batch: int):
        if max_batch <= self.max_batch:
            return
        # a pending late half lives in the workspace (slabs, replicas, the
        # deferral record): finish it before the workspace is replaced
        self.flush()
        self.ws_bytes = N.workspace_bytes(self.desc, max_batch)
        self.ws = torch.zeros(self.ws_bytes // 4, dtype=torch.float32, device=self.device)
        self.max_batch = max_batch

    def set_data(self, data: Dict[str, torch.Tensor]):
        """Upload (once) the six dataset arrays of a CEOFirmDataset dict."""
        out = {}
        for k in DATA_KEYS:
            t = data[k]
            if k in ("firm_cat", "ceo_cat"):
                t = t.to(device=self.device, dtype=torch.int64)
                if t.dim() == 1:
                    t = t.view(-1, 1)
            elif k in ("target", "weights"):
                t = t.to(device=self.device, dtype=torch.float32).reshape(-1)
            else:
                t = t.to(device=self.device, dtype=torch.float32)
            out[k] = t.contiguous()
        g = self.model._geom
        for t, key in enumerate(("firm_cat", "ceo_cat")):
            check_category_codes(out[key], g["cat_counts"][t], key)
        self.data = out

    def _batch(self, rows, row0, n_rows, cycle=0, t_base=0):
        d = self.data
        return N.make_batch(d["firm_numeric"], d["firm_cat"], d["ceo_numeric"], d["ceo_cat"],
                            target=d["target"], weight=d["weights"], rows=rows, row0=row0,
                            n_rows=n_rows, cycle=cycle, t_base=t_base)

    # ------------------------------------------------------------------ steps
    def is_deterministic(self) -> bool:
        return self.model.is_deterministic() if self.deterministic is None else bool(self.deterministic)

    def _launch(self, batch, n_rows, apply_adam: bool):
        self.ensure_batch(n_rows)
        N.set_deterministic(self.desc, self.is_deterministic())
        defer_ok = apply_adam and not self.dp and n_rows >= 2 and n_rows not in self._no_defer
        pending = False
        if self._late_rows:
            if defer_ok and n_rows == self._late_rows:
                pending = True
            else:
                self.flush()
        defer = self.defer_late and defer_ok
        a = self.arena

        def call(extra):
            self.desc.flags |= extra
            try:
                return self.lib.tt_train_step(self.desc, a.params.data_ptr(), a.buffers.data_ptr(),
                                              a.nbt.data_ptr(), batch, self.hp, self.seed, self.state.data_ptr(),
                                              self.ws.data_ptr(), self.ws_bytes, self.grad.data_ptr(),
                                              self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), int(apply_adam),
                                              N.stream_ptr(self.device))
            finally:
                self.desc.flags &= ~(N.TT_FLAG_DEFER_LATE | N.TT_FLAG_LATE_PENDING)
        extra = (N.TT_FLAG_DEFER_LATE if defer else 0) | (N.TT_FLAG_LATE_PENDING if pending else 0)
        rc = call(extra)
        if rc == N.TT_ERR_UNSUPPORTED and extra:  # geometry without the deferred form: plain steps
            self._no_defer.add(n_rows)
            if pending:
                self.flush()
            defer = False
            rc = call(0)
        N.check(rc, "tt_train_step", n_rows, 64)
        if defer:
            self._late_rows, self._late_batch = n_rows, batch
            # a strong reference while (only while) a late half is pending: a
            # trainer dropped now is kept alive by the model until that late
            # half has run (sync_trainer), so the update is never lost
            self.model._pending_flush = self.flush
        elif self._late_rows:  # (consumed by this step's first kernel)
            self._late_rows, self._late_batch = 0, None
            self.model._pending_flush = None

    def flush(self):
        """Run the pending late half of the last deferred step (tt_train_flush):
        parameters, Adam moments and the loss sum are then complete."""
        if not self._late_rows:
            return
        N.set_deterministic(self.desc, self.is_deterministic())
        a = self.arena
        rc = self.lib.tt_train_flush(self.desc, a.params.data_ptr(), a.buffers.data_ptr(), a.nbt.data_ptr(),
                                     self._late_batch, self.hp, self.state.data_ptr(), self.ws.data_ptr(),
                                     self.ws_bytes, self.grad.data_ptr(), self.exp_avg.data_ptr(),
                                     self.exp_avg_sq.data_ptr(), N.stream_ptr(self.device))
        N.check(rc, "tt_train_flush")
        self._late_rows, self._late_batch = 0, None
        self.model._pending_flush = None

    def deferral_state(self):
        """The host's record of a pending late half, e.g. right after
        capturing steps into a graph (what a replay of that graph leaves)."""
        return (self._late_rows, self._late_batch)

    def after_replay(self, state):
        """Replaying a captured graph does not pass through step(): restore
        the record the capture ended with, so the next flush (or step) runs the
        last replayed step's late half.  The device guard makes a flush of
        nothing a no-op, never a second late half."""
        self._late_rows, self._late_batch = state
        self.model._pending_flush = self.flush if state[0] else None

    def _launch_dp(self, batch, n_rows):
        """The data-parallel step: the exchange inside the step's reduction
        when the peer exchange is mapped and the reduction's blocks can all be
        resident (tt_train_step_dp; decided once), else reduce -> exchange
        (peer launch or RCCL all-reduce) -> Adam."""
        if self.peer is not None and self.fused_exchange is None and not torch.cuda.is_current_stream_capturing():
            self.ensure_batch(n_rows)
            self.fused_exchange = self._validate_fused_exchange(batch, n_rows)
        if self.peer is not None and self.fused_exchange is True:
            self.ensure_batch(n_rows)
            N.set_deterministic(self.desc, self.is_deterministic())
            rc = self.peer.train_step(self, batch)
            if rc != N.TT_ERR_UNSUPPORTED:
                N.check(rc, "tt_train_step_dp", n_rows, 64)
                self.fused_exchange = True
                return
            self.fused_exchange = False
            self.peer.protocol = N.TT_AR_PULL  # (the validated two-launch form)
        self._launch(batch, n_rows, False)
        self.allreduce_and_adam()

    def _validate_fused_exchange(self, batch, n_rows) -> bool:
        """Decide once, on this job's real topology, whether the exchange
        inside the reduction (tt_train_step_dp) may be used: run the first
        batch both ways in deterministic mode -- the in-reduction exchange,
        then reduce -> standalone exchange + Adam (itself checked against the
        collective by PeerExchange.create) -- from the same saved state, and
        keep the fused form only if every rank finished both without a
        timeout and got bitwise the same parameters, Adam moments, BN buffers
        and gradient.  The state is restored (and the exchange regions reset)
        afterwards, so the real step runs from where it started.  The
        protocol (distributed.choose_exchange_form) runs the same collectives
        on every rank whatever each rank's outcome, so a rank whose check or
        timing fails cannot leave its peers waiting."""
        a = self.arena
        live = (a.params, a.buffers, a.nbt, self.grad, self.exp_avg, self.exp_avg_sq, self.state)
        saved = [t.clone() for t in live]

        def restore():
            torch.cuda.synchronize(self.device)
            for dst, src in zip(live, saved):
                dst.copy_(src)
            self.ws.zero_()  # a timed-out launch may leave accumulators behind
            if self.pg is not None:
                self.peer.reset(self.pg)
            else:
                self.peer.err.zero_()

        def result():
            torch.cuda.synchronize(self.device)
            if self.peer.failed():
                return None
            return torch.cat([a.params, self.exp_avg, self.exp_avg_sq, a.buffers, self.grad]).clone()

        def fused_step():
            N.check(self.peer.train_step(self, batch), "tt_train_step_dp")

        def two_launch():
            self._launch(batch, n_rows, False)
            self.allreduce_and_adam()

        def run(fn, proto):
            def go():
                self.peer.protocol = proto
                fn()
                return result()
            return go

        def timed(fn, proto):
            def go():
                self.peer.protocol = proto
                t = self._time_steps(fn)
                if self.peer.failed():
                    raise RuntimeError("an exchange timed out while timing")
                return t
            return go
        # (name, step, protocol): the reference -- reduce, then the standalone
        # pull exchange + Adam, itself checked against the collective -- and
        # the candidates: the exchange inside the reduction (pull / push) and
        # the standalone push exchange
        pull, push = N.TT_AR_PULL, N.TT_AR_PUSH
        forms = {"two_launch": (two_launch, pull), "fused": (fused_step, pull),
                 "fused_push": (fused_step, push), "two_launch_push": (two_launch, push)}

        prev_det = self.deterministic

        def steps_mode():  # time in the mode the steps will run in
            self.deterministic = prev_det
            N.set_deterministic(self.desc, self.is_deterministic())
        self.deterministic = True  # the bitwise check in deterministic mode
        N.set_deterministic(self.desc, True)
        import os
        entry = lambda k: (k, run(*forms[k]), timed(*forms[k]))  # noqa: E731
        try:
            use, times = choose_exchange_form(
                entry("two_launch"), [entry(k) for k in forms if k != "two_launch"], restore, self.pg, self.device,
                prefer=os.environ.get("CEO_TT_EXCHANGE_FORM") or
                ("fused" if os.environ.get("CEO_TT_FUSED_EX") == "1" else None), before_timing=steps_mode)
        finally:
            steps_mode()
        self.exchange_form_us = times
        self.exchange_form = use
        self.fused_vs_two_launch_us = (times["fused"], times["two_launch"])
        self.peer.protocol = forms[use][1]
        return use in ("fused", "fused_push")

    def _time_steps(self, fn, k: int = 8) -> float:
        """Device time per step (us) of k back-to-back calls of ``fn``: the
        launches queue behind a short GPU spin so the events bracket the
        kernels, not the host's enqueue rate.  Collective: every rank calls it
        (a barrier first)."""
        import torch.distributed as dist
        torch.cuda.synchronize(self.device)
        if self.pg is not None:
            dist.barrier(group=self.pg)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        try:
            torch.cuda._sleep(2_000_000)  # ~1 ms: the host enqueues the k steps meanwhile
        except Exception:  # noqa: BLE001 -- timing then includes the host's enqueue rate
            pass
        e0.record()
        for _ in range(k):
            fn()
        e1.record()
        torch.cuda.synchronize(self.device)
        return 1e3 * e0.elapsed_time(e1) / k

    def step(self, rows: Optional[torch.Tensor], row0: int, n_rows: int):
        """One optimizer step on dataset rows rows[row0:row0+n_rows]."""
        batch = self._batch(rows, row0, n_rows)
        if not self.dp:
            self._launch(batch, n_rows, True)
        else:
            self._launch_dp(batch, n_rows)
            self._check_eager()
        self.steps_host += 1

    def step_cycle(self, rows: torch.Tensor, batch_size: int, n_batches: int, t_base: int = 0):
        """Graph-replayable step: batch k = ((t-1-t_base) % n_batches) of
        ``rows`` taken from the device step counter (no host arguments change
        between steps)."""
        batch = self._batch(rows, 0, batch_size, cycle=n_batches, t_base=t_base)
        if not self.dp:
            self._launch(batch, batch_size, True)
        else:
            self._launch_dp(batch, batch_size)
            self._check_eager()
        self.steps_host += 1

    def step_cycle_n(self, rows: torch.Tensor, batch_size: int, n_batches: int, n_steps: int, t_base: int = 0):
        # (one C call for all n steps: no deferred late halves between them)
        """n_steps graph-free cycle-mode steps in ONE library call
        (tt_train_steps: the launches are issued from C++, no host work per
        step); the same steps as n_steps calls of step_cycle.  Data-parallel
        trainers loop over step_cycle."""
        if self.dp:
            for _ in range(n_steps):
                self.step_cycle(rows, batch_size, n_batches, t_base)
            return
        batch = self._batch(rows, 0, batch_size, cycle=n_batches, t_base=t_base)
        self.ensure_batch(batch_size)
        self.flush()
        N.set_deterministic(self.desc, self.is_deterministic())
        a = self.arena
        rc = self.lib.tt_train_steps(self.desc, a.params.data_ptr(), a.buffers.data_ptr(), a.nbt.data_ptr(),
                                     batch, self.hp, self.seed, self.state.data_ptr(), self.ws.data_ptr(),
                                     self.ws_bytes, self.grad.data_ptr(), self.exp_avg.data_ptr(),
                                     self.exp_avg_sq.data_ptr(), int(n_steps), N.stream_ptr(self.device))
        N.check(rc, "tt_train_steps", batch_size, 64)
        self.steps_host += n_steps

    def allreduce_and_adam(self):
        a = self.arena
        if self.peer is not None:  # mean over ranks + Adam, one launch
            self.peer.run(self.grad, grad_out=self.grad, params=a.params, exp_avg=self.exp_avg,
                          exp_avg_sq=self.exp_avg_sq, hp=self.hp, state=self.state)
            return
        average_gradients_(self.grad, self.pg)
        rc = self.lib.tt_adam_apply(a.params.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(),
                                    self.exp_avg_sq.data_ptr(), a.params.numel(), self.hp,
                                    self.state.data_ptr(), 0, N.stream_ptr(self.device))
        N.check(rc, "tt_adam_apply")

    def _check_eager(self):
        """Eager data-parallel steps on the peer exchange check it every step
        (a host sync); inside a hipGraph capture the check is the caller's
        (after each replayed chunk or on the next loss read)."""
        if self.peer is not None and not torch.cuda.is_current_stream_capturing():
            self.peer.check()

    # ------------------------------------------------------------------ metrics
    def loss_sum_tensor(self) -> torch.Tensor:
        return self.state.view(torch.float32)[4:5]

    def pop_loss_sum(self, read: bool = True) -> Optional[float]:
        """Sum of batch-mean losses since the last call (reads => host sync)."""
        self.flush()  # a deferred late half still has its step's loss to add
        t = self.loss_sum_tensor()
        v = float(t.item()) if read else None
        t.zero_()
        if read:
            self.check_exchange()
        return v

    def check_exchange(self):
        """Raise if the peer gradient exchange failed (host sync).  Called on
        every loss read, at the end of train_model and after bench's timed
        region; between checks a failed rank's launches are device-side no-ops,
        so its parameters stay at the last exchanged step."""
        if self.peer is not None:
            self.peer.check()

    def steps_done(self) -> int:
        return int(self.state[0].item())
