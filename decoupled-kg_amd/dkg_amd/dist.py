"""Multi-GPU Discrete KG: the (candidate x scalarisation) pair space split over ranks.

SURVEY.md §8(e): every (xnew, w) pair is independent (``discretekg.py:200-235``
loops over scalarisations and averages; ``:145`` loops over candidates), so the
only exchange is combining per-candidate results:

* ``axis="scalarisations"`` — rank r evaluates all B candidates on its
  contiguous slice of the S weight rows; the per-candidate partial sums
  ``S_r * mean_r`` meet in ONE all-reduce (sum, fp64, count B) and are divided
  by S.  This is the north-star layout (one RCCL all-reduce of per-candidate
  KG values over xGMI).
* ``axis="candidates"`` — rank r evaluates its contiguous slice of the B
  candidates on all S rows; the slices meet in one all-gather.

One process per GPU (``torch.distributed``; backend "nccl" is RCCL on ROCm,
"gloo" for the CPU tests).  GP state is replicated: each rank builds its
device caches from the same host tensors.  The local evaluation is
``DiscreteKnowledgeGradient`` on the rank's device unless ``local_forward``
is injected (the multi-process CPU tests inject the oracle).

The result is differentiable w.r.t. X on every rank (``optimize_acqf``'s
L-BFGS-B needs dKG/dX): the exchange is wrapped in autograd functions whose
backward routes each rank's share of the gradient back to its own
evaluation, and the gradient w.r.t. X is summed over ranks, so every rank
receives the full dKG/dX.  Like the forward, ``backward`` is collective:
every rank must call it with the same incoming gradient.
"""

from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist
from torch import Tensor

from .errors import BotorchTensorDimensionError

LocalForward = Callable[[Tensor, Tensor], Tensor]  # (X [B, d], W [S_r, m]) -> KG averaged over W, [B]


def _to_comm(t: Tensor, cdev: torch.device) -> Tensor:
    return t.to(cdev, torch.double).contiguous()


class _SumGradOverRanks(torch.autograd.Function):
    """Identity forward; backward all-reduces (sums) the gradient over the ranks, so each rank's
    input receives every rank's contribution."""

    @staticmethod
    def forward(ctx, x, cdev, group):
        ctx.cdev, ctx.group = cdev, group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        gc = _to_comm(g, ctx.cdev)
        dist.all_reduce(gc, op=dist.ReduceOp.SUM, group=ctx.group)
        return gc.to(g.device, g.dtype), None, None


class _AllReduceSum(torch.autograd.Function):
    """Forward: the sum over ranks of every rank's partial (one all-reduce).  Backward: the
    incoming gradient (the same on every rank) is the gradient of this rank's partial."""

    @staticmethod
    def forward(ctx, part, group):
        out = part.detach().clone()
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return g, None


class _AllGather(torch.autograd.Function):
    """Forward: the ranks' equal-length slices concatenated in rank order (one all-gather).
    Backward: this rank's slice of the incoming gradient."""

    @staticmethod
    def forward(ctx, mine, world, rank, group):
        ctx.rank, ctx.n = rank, mine.shape[0]
        allv = torch.empty(mine.shape[0] * world, dtype=mine.dtype, device=mine.device)
        if mine.device.type == "cuda":
            dist.all_gather_into_tensor(allv, mine.detach().contiguous(), group=group)
        else:
            dist.all_gather(list(allv.view(world, -1)), mine.detach().contiguous(), group=group)
        return allv

    @staticmethod
    def backward(ctx, g):
        return g[ctx.rank * ctx.n:(ctx.rank + 1) * ctx.n], None, None, None


class _ZerosConnected(torch.autograd.Function):
    """Zeros [n] on ``cdev`` that stay in the autograd graph of ``x`` (a rank with no local work must
    still join the collective backward); the backward hands ``x`` an exact zero gradient, so a
    non-finite coordinate in ``x`` cannot leak into the zeros (``0 * inf`` would be NaN)."""

    @staticmethod
    def forward(ctx, x, n, cdev):
        ctx.shape, ctx.dtype, ctx.device = x.shape, x.dtype, x.device
        return torch.zeros(n, dtype=torch.double, device=cdev)

    @staticmethod
    def backward(ctx, g):
        return torch.zeros(ctx.shape, dtype=ctx.dtype, device=ctx.device), None, None


def _zeros_like_graph(x: Tensor, n: int, cdev: torch.device) -> Tensor:
    if x.requires_grad:
        return _ZerosConnected.apply(x, n, cdev)
    return torch.zeros(n, dtype=torch.double, device=cdev)


def shard_range(total: int, rank: int, world: int) -> tuple:
    """Contiguous slice [lo, hi) of ``total`` items owned by ``rank`` (chunks of ceil(total/world))."""
    chunk = -(-total // world) if total > 0 else 0
    lo = min(total, rank * chunk)
    return lo, min(total, lo + chunk)


class ShardedDiscreteKG:
    """``DiscreteKnowledgeGradient.forward`` with the pair space split across ranks.

    Every rank calls ``forward`` with the same X and receives the full [*batch]
    result (the unsharded KG up to fp64 summation order of the S average).
    """

    AXES = ("scalarisations", "candidates")

    def __init__(self, model, x_discretisation: Tensor, scalarisation_weights: Tensor,
                 target_output_ix: Optional[int] = None, axis: str = "scalarisations", group=None,
                 local_forward: Optional[LocalForward] = None, device=None):
        if axis not in self.AXES:
            raise ValueError(f"axis must be one of {self.AXES}; got {axis!r}")
        if scalarisation_weights.dim() != 2:
            raise BotorchTensorDimensionError("Expected 'scalarisation_weights' to have two dimensions.")
        self.axis = axis
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # the exchange runs whenever a process group exists (world size 1 included: one RCCL / gloo
        # collective over a single rank), and is skipped without one
        self.collective = dist.is_initialized()
        self.W = scalarisation_weights
        self.S = scalarisation_weights.shape[0]
        self.d = x_discretisation.shape[-1]
        self.w_lo, self.w_hi = shard_range(self.S, self.rank, self.world) if axis == "scalarisations" \
            else (0, self.S)
        self.device = torch.device(device) if device is not None else None
        if local_forward is None:
            from .discretekg import DiscreteKnowledgeGradient
            W_local = scalarisation_weights[self.w_lo:self.w_hi]
            self._acq = None
            if self.w_hi > self.w_lo:
                self._acq = DiscreteKnowledgeGradient(model, x_discretisation, W_local, target_output_ix,
                                                      device=device)

            def local_forward(X, W):  # noqa: ARG001 - W is baked into the plan
                return self._acq(X.unsqueeze(-2))

        self._local = local_forward

    def _comm_device(self, like: Tensor) -> torch.device:
        backend = dist.get_backend(self.group) if dist.is_initialized() else "gloo"
        if backend == "nccl":
            return self.device or torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def forward(self, X: Tensor) -> Tensor:
        if X.dim() < 2 or X.shape[-2] != 1:
            raise AssertionError(f"Expected X to be `batch_shape x q=1 x d`, but got X with shape {X.shape}.")
        batch_shape = X.shape[:-2]
        flat = X.reshape(-1, self.d)
        B = flat.shape[0]
        cdev = self._comm_device(flat)
        if self.collective and flat.requires_grad:
            flat = _SumGradOverRanks.apply(flat, cdev, self.group)
        if self.axis == "scalarisations":
            n_local = self.w_hi - self.w_lo
            if n_local > 0 and B > 0:
                part = self._local(flat, self.W[self.w_lo:self.w_hi]).to(cdev, torch.double) * n_local
            else:
                part = _zeros_like_graph(flat, B, cdev)
            if self.collective:
                part = _AllReduceSum.apply(part, self.group)
            out = part / self.S
        else:
            chunk = -(-B // self.world) if B > 0 else 0
            lo, hi = shard_range(B, self.rank, self.world)
            pieces = []
            if hi > lo:
                pieces.append(self._local(flat[lo:hi], self.W).to(cdev, torch.double))
            pad = chunk - (hi - lo)
            if pad > 0 or not pieces:
                pieces.append(_zeros_like_graph(flat, pad, cdev))
            mine = torch.cat(pieces) if len(pieces) > 1 else pieces[0]
            allv = _AllGather.apply(mine, self.world, self.rank, self.group) if self.collective else mine
            out = allv[:B]
        return out.to(X.device).reshape(batch_shape)

    __call__ = forward

    def forward_async(self, X: Tensor) -> "PendingKG":
        """The no-grad forward with its exchange left in flight: the local evaluation is enqueued and the
        collective started asynchronously (``async_op=True``), so a caller evaluating many batches (the
        raw-sample scoring of ``optimize_acqf``, bench.py) can issue the next batch before this one's
        collective completes.  ``.wait()`` returns what ``forward`` returns.  The gradient path stays
        synchronous (its backward is a collective too)."""
        if X.dim() < 2 or X.shape[-2] != 1:
            raise AssertionError(f"Expected X to be `batch_shape x q=1 x d`, but got X with shape {X.shape}.")
        batch_shape = X.shape[:-2]
        flat = X.detach().reshape(-1, self.d)
        B = flat.shape[0]
        cdev = self._comm_device(flat)
        if self.axis == "scalarisations":
            n_local = self.w_hi - self.w_lo
            if n_local > 0 and B > 0:
                buf = (self._local(flat, self.W[self.w_lo:self.w_hi]).detach().to(cdev, torch.double) * n_local)
            else:
                buf = torch.zeros(B, dtype=torch.double, device=cdev)
            buf = buf.contiguous()
            work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True) \
                if self.collective else _Done()
            return PendingKG(work, lambda: (buf / self.S).to(X.device).reshape(batch_shape))
        chunk = -(-B // self.world) if B > 0 else 0
        lo, hi = shard_range(B, self.rank, self.world)
        mine = torch.zeros(chunk, dtype=torch.double, device=cdev)
        if hi > lo:
            mine[:hi - lo] = self._local(flat[lo:hi], self.W).detach().to(cdev, torch.double)
        if not self.collective:
            return PendingKG(_Done(), lambda: mine[:B].to(X.device).reshape(batch_shape))
        allv = torch.empty(chunk * self.world, dtype=torch.double, device=cdev)
        if cdev.type == "cuda":
            work = dist.all_gather_into_tensor(allv, mine, group=self.group, async_op=True)
        else:
            work = dist.all_gather(list(allv.view(self.world, -1)), mine, group=self.group, async_op=True)
        return PendingKG(work, lambda: allv[:B].to(X.device).reshape(batch_shape))


class PendingKG:
    """An exchange in flight (ShardedDiscreteKG.forward_async); ``wait()`` completes it and returns the KG."""

    def __init__(self, work, result: Callable[[], Tensor]):
        self._work, self._result, self._out = work, result, None

    def wait(self) -> Tensor:
        if self._out is None:
            self._work.wait()
            self._out = self._result()
        return self._out


class BatchExchange:
    """K forward batches per collective ("loop K forward batches per all-reduce,
    count = K*B"): the throughput driver's exchange of per-candidate KG values.

    Step k writes its ``B`` values into ``row(k)`` (row k % K of one of two [K, B] buffers);
    after the K-th row of a buffer ``done(k)`` starts one async collective over the whole
    buffer, and the next K steps fill the other buffer while it runs.  A buffer is only reused
    after its collective has completed.  ``mode="gather"`` (candidates sharded): an all-gather,
    every rank ends with [world, rows, B].  ``mode="reduce"`` (scalarisations sharded): the rows
    hold per-rank means over ``S_local`` rows; they are scaled to partial sums and all-reduced
    (the caller divides by the total S).  ``sink`` (tests): completed results are appended to it.
    """

    def __init__(self, B: int, every: int, mode: str = "gather", S_local: int = 1, device=None,
                 dtype=torch.double, sink: Optional[list] = None):
        if mode not in ("gather", "reduce"):
            raise ValueError(f"mode must be 'gather' or 'reduce', got {mode!r}")
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.collective = dist.is_initialized()  # as ShardedDiscreteKG: world size 1 included
        self.B, self.E, self.mode, self.S_local = int(B), max(1, int(every)), mode, S_local
        self.bufs = [torch.zeros(self.E, self.B, dtype=dtype, device=device) for _ in range(2)]
        self.gathered = [torch.zeros(self.world * self.E * self.B, dtype=dtype, device=device) for _ in range(2)]
        self.works = [None, None]
        self.rows = [0, 0]
        self.sink = sink

    def _slot(self, k: int):
        return (k // self.E) % 2, k % self.E

    def _finish(self, slot: int) -> None:
        if self.works[slot] is not None:
            self.works[slot].wait()
            self.works[slot] = None
            if self.sink is not None:
                r = self.rows[slot]
                if self.mode == "gather":
                    self.sink.append(self.gathered[slot][:self.world * r * self.B].view(self.world, r, self.B).clone())
                else:
                    self.sink.append(self.bufs[slot][:r].clone())

    def row(self, k: int) -> Tensor:
        """The [B] buffer step k writes (waits for the collective that last used its buffer)."""
        slot, r = self._slot(k)
        if r == 0:
            self._finish(slot)
        return self.bufs[slot][r]

    def block(self, k: int, g: int) -> Tensor:
        """The [g * B] buffer steps k .. k + g - 1 write (one launch of g forward batches,
        ``ForwardPlan.forward_batches_into``): rows of one buffer, so they may not cross an exchange."""
        slot, r = self._slot(k)
        if g < 1 or r + g > self.E:
            raise ValueError(f"steps {k}..{k + g - 1} cross an exchange of {self.E} steps")
        if r == 0:
            self._finish(slot)
        return self.bufs[slot][r:r + g].view(-1)

    def _exchange(self, slot: int, rows: int) -> None:
        self.rows[slot] = rows
        if not self.collective:
            if self.mode == "gather":
                self.gathered[slot][:rows * self.B].copy_(self.bufs[slot][:rows].reshape(-1))
            self.works[slot] = _Done()
            return
        blk = self.bufs[slot][:rows].view(-1)
        if self.mode == "gather":
            self.works[slot] = dist.all_gather_into_tensor(self.gathered[slot][:self.world * rows * self.B], blk,
                                                           async_op=True)
        else:
            blk.mul_(self.S_local)
            self.works[slot] = dist.all_reduce(blk, op=dist.ReduceOp.SUM, async_op=True)

    def done(self, k: int) -> None:
        """Step k has written its row: exchange the buffer if it is full."""
        slot, r = self._slot(k)
        if r == self.E - 1:
            self._exchange(slot, self.E)

    def flush(self, nsteps: int) -> None:
        """After ``nsteps`` steps: exchange a partially filled last buffer, then wait for everything."""
        rem = nsteps % self.E
        if rem:
            self._exchange((nsteps // self.E) % 2, rem)
        last = ((nsteps - 1) // self.E) % 2 if nsteps > 0 else 1
        for slot in (1 - last, last):  # the older buffer's collective first
            self._finish(slot)


class _Done:
    def wait(self):
        return None
