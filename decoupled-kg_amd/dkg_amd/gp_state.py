"""Device-resident GP state for the Discrete-KG kernels.

Builds, per output, the caches GPyTorch's exact prediction keeps behind
``model.posterior`` (``discretekg.py:182-185, 275-284``) — the ones BoTorch's
``fast_pred_var`` posterior uses:

* ``K = s k(X, X) + noise I``, ``L = psd_safe_cholesky(K)`` (linear_operator's
  jitter policy: absolute 1e-8 * 10**i, 3 retries), ``R = L^{-T}``
  (root_inv_decomposition) and ``alpha = K^{-1}(y - c)``:
                                              HIP ``dkg_prepare_output`` (blocked
                                              Cholesky / triangular inverse kernels)
* ``root_frag`` = R in MFMA fragment order    HIP ``dkg_pack_root``
* ``Q_D = K(D, X) R``, ``mu_D = c + K(D,X) alpha`` over the discretisation
                                              HIP ``dkg_cross_root``

All of it runs once per (model, discretisation) — the reference rebuilds the
same caches once per BO iteration — and stays in HBM for every forward call.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List

import torch

from . import _lib
from .errors import UnsupportedError
from .model import ModelListGPState, SingleTaskGPState, kernel_id


def _pad16(x: int) -> int:
    return (x + 15) // 16 * 16


def current_stream_ptr(device) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)


def _raw_stream(device) -> int:
    """current_stream_ptr without building a Stream object (the B = 1 host path: ~0.3 instead of ~3 us)."""
    idx = device.index if isinstance(device, torch.device) and device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


@dataclass
class OutputCache:
    """Device tensors of one output; ``struct`` points into them."""

    state: SingleTaskGPState
    inv_ls: torch.Tensor
    train_x: torch.Tensor
    alpha: torch.Tensor
    root_frag: torch.Tensor
    disc_frag: torch.Tensor
    disc_mean: torch.Tensor
    L: torch.Tensor
    jitter: float = 0.0  # absolute jitter psd_safe_cholesky needed (0: none)
    struct: _lib.DkgOutput = field(repr=False, default=None)


def _base_struct(st: SingleTaskGPState, inv_ls, train_x) -> _lib.DkgOutput:
    o = _lib.DkgOutput()
    o.n = st.num_train
    o.kernel = kernel_id(st.kernel, st.nu)
    o.outputscale = float(st.outputscale)
    o.noise = float(st.noise)
    o.mean_constant = float(st.mean_constant)
    o.y_mean = float(st.y_mean)
    o.y_std = float(st.y_std)
    o.inv_lengthscale = _lib.ptr(inv_ls)
    o.train_x = _lib.ptr(train_x)
    return o


def prepare_outputs(models, D: torch.Tensor) -> List[OutputCache]:
    """Every output's device caches over the discretisation ``D`` (device, N x d): the factorisations of
    all outputs side by side (dkg_prepare_outputs: one chain of launches, one status check), then each
    output's Q_D and mu_D (dkg_cross_root)."""
    lib = _lib.load()
    dev = D.device
    stream = current_stream_ptr(dev)
    N = D.shape[0]
    parts = []
    # every output's training inputs, inverse lengthscales and targets in one host-to-device copy (a copy
    # from pageable memory costs ~3 us each; a model of m outputs had 3 m of them)
    host = []
    for st in models:
        n, d = st.train_x.shape
        if _pad16(n) > 1024:
            raise UnsupportedError(f"n={n} training points > 1024 per output is not supported")
        host += [st.train_x.detach().to(torch.double).reshape(-1), (1.0 / st.lengthscale).detach().to(torch.double)
                 .reshape(-1), st.train_y.detach().to(torch.double).reshape(-1)]
    flat = torch.cat([t.cpu() for t in host]).to(dev) if host else None
    views, off = [], 0
    for t in host:
        views.append(flat[off:off + t.numel()])
        off += t.numel()
    for k, st in enumerate(models):
        n, d = st.train_x.shape
        X = views[3 * k].view(n, d)
        inv_ls = views[3 * k + 1]
        o = _base_struct(st, inv_ls, X)
        y = views[3 * k + 2]
        L = torch.empty(n, n, dtype=torch.double, device=dev)
        work = torch.empty(lib.dkg_prepare_workspace(n), dtype=torch.uint8, device=dev)
        alpha = torch.empty(_pad16(n), dtype=torch.double, device=dev)
        root_frag = torch.empty(lib.dkg_frag_elems(n, n), dtype=torch.double, device=dev)
        parts.append((st, o, X, inv_ls, y, L, work, alpha, root_frag))
    m = len(parts)
    d = D.shape[1]
    outs = (_lib.DkgOutput * m)(*[p[1] for p in parts])
    ptrs = lambda k: (ctypes.c_void_p * m)(*[_lib.ptr(p[k]) for p in parts])  # noqa: E731
    jit = (ctypes.c_double * m)()
    wbytes = (ctypes.c_size_t * m)(*[p[6].numel() for p in parts])
    _lib.check(lib.dkg_prepare_outputs(outs, m, d, ptrs(4), 3, ptrs(5), ptrs(6), wbytes, ptrs(7), ptrs(8), jit, stream),
               "dkg_prepare_outputs")
    caches = []
    for i, (st, o, X, inv_ls, y, L, work, alpha, root_frag) in enumerate(parts):
        o.alpha = _lib.ptr(alpha)
        o.root_frag = _lib.ptr(root_frag)
        disc_frag = torch.empty(max(1, lib.dkg_frag_elems(N, o.n)), dtype=torch.double, device=dev)
        disc_mean = torch.empty(max(16, _pad16(N)), dtype=torch.double, device=dev)
        if N > 0:
            _lib.check(lib.dkg_cross_root(o, d, _lib.ptr(D), N, _lib.ptr(disc_frag), _lib.ptr(disc_mean), stream),
                       "dkg_cross_root")
        o.disc_frag = _lib.ptr(disc_frag)
        o.disc_mean = _lib.ptr(disc_mean)
        caches.append(OutputCache(st, inv_ls, X, alpha, root_frag, disc_frag, disc_mean, L, jit[i], o))
    return caches


def prepare_output(st: SingleTaskGPState, D: torch.Tensor) -> OutputCache:
    """One output's device caches (prepare_outputs of one)."""
    return prepare_outputs([st], D)[0]


class DeviceGPState:
    """All outputs' caches over one discretisation, plus a reusable workspace."""

    def __init__(self, model: ModelListGPState, x_discretisation: torch.Tensor, device=None):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise UnsupportedError("the Discrete-KG kernels run on a ROCm (HIP) device; got " + str(self.device))
        if model.num_outputs > _lib.MAX_OUTPUTS:
            raise UnsupportedError(f"{model.num_outputs} outputs > {_lib.MAX_OUTPUTS}")
        if model.input_dim > _lib.MAX_DIM:
            raise UnsupportedError(f"input dimension {model.input_dim} > {_lib.MAX_DIM}")
        self.model = model
        self.D = x_discretisation.detach().to(self.device, torch.double).contiguous()
        self.N, self.d = self.D.shape
        self.outputs: List[OutputCache] = prepare_outputs(model.models, self.D)
        self.m = len(self.outputs)
        self.structs = (_lib.DkgOutput * self.m)(*[c.struct for c in self.outputs])
        self._ws = None
        self._ws_key = None

    def plan(self, W: torch.Tensor, target, max_B: int, grad: bool = False, force_walk: bool = False,
             f32: bool = False, fused: bool = False, no_chain: bool = False) -> "ForwardPlan":
        return ForwardPlan(self, W, target, max_B, grad, force_walk, f32, fused, no_chain)

    def forward(self, X: torch.Tensor, W: torch.Tensor, target, kg_pairs=None, timed: bool = False):
        """One-shot forward (builds a plan on the fly); see ForwardPlan for the fast path."""
        p = ForwardPlan(self, W, target, max(1, X.shape[0]))
        return p.forward(X, kg_pairs=kg_pairs, timed=timed)


class ForwardPlan:
    """A DKG plan (include/dkg.h "Plan API"): weights, target and workspace for
    up to ``max_B`` candidates, device copy written once; ``forward`` is one
    C call that launches the forward on the current stream: the three stage
    kernels, or with ``fused=True`` one launch whose stages hand off inside it
    (dkg_fused.h; same bits, not faster on MI355X: DESIGN.md 4.8).  With ``grad=True`` the
    workspace also holds the gradient buffers and ``forward_grad`` returns
    dKG/dx alongside KG."""

    def __init__(self, state: DeviceGPState, W: torch.Tensor, target, max_B: int, grad: bool = False,
                 force_walk: bool = False, f32: bool = False, fused: bool = False, no_chain: bool = False):
        lib = _lib.load()
        self.state = state
        self.device = state.device
        # a snapshot: the plan's intercept cache and top hints (Plan::icpt / itop, built at init) are derived from
        # these weights, so a caller editing its own weights tensor in place must not reach the plan's copy
        self.W = W.detach().to(self.device, torch.double, copy=True).contiguous()
        if self.W.dim() != 2 or self.W.shape[1] != state.m:
            raise ValueError(f"weights must be S x {state.m}")
        self.S = self.W.shape[0]
        if target is not None and not (0 <= int(target) < state.m):
            # the C ABI's -1 means "all outputs observed": a negative index never reaches it
            raise ValueError(f"target must be None (all outputs) or in [0, {state.m}), got {target}")
        self.target = -1 if target is None else int(target)
        self.max_B = int(max_B)
        self.grad = bool(grad)
        self.f32 = bool(f32)
        flags = ((_lib.DKG_PLAN_GRAD if self.grad else 0) | (_lib.DKG_PLAN_FORCE_WALK if force_walk else 0)
                 | (_lib.DKG_PLAN_F32 if self.f32 else 0) | (_lib.DKG_PLAN_FUSED if fused else 0)
                 | (_lib.DKG_PLAN_NO_CHAIN if no_chain else 0))
        need = lib.dkg_plan_workspace(state.structs, state.m, state.d, state.N, self.max_B, self.S, flags)
        self.ws = torch.zeros(max(need, 256), dtype=torch.uint8, device=self.device)
        nbytes = lib.dkg_plan_bytes()
        self.host = ctypes.create_string_buffer(nbytes)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        _lib.check(lib.dkg_plan_init(state.structs, state.m, state.d, _lib.ptr(state.D), state.N, _lib.ptr(self.W),
                                     self.S, self.target, self.max_B, flags, _lib.ptr(self.ws), self.ws.numel(),
                                     self.host, _lib.ptr(self.dev), current_stream_ptr(self.device)),
                   "dkg_plan_init")
        self.fused = bool(lib.dkg_plan_fused(self.host))  # forward_into is one fused launch
        self._fwd = lib.dkg_plan_forward
        self._fwd_batches = lib.dkg_plan_forward_batches
        self._fwd_timed = lib.dkg_plan_forward_timed
        self._fwd_grad_hostx = lib.dkg_plan_forward_grad_hostx
        self._dev_ptr = _lib.ptr(self.dev)

    def status(self, reset: bool = False) -> int:
        """The bits of the fused launches' in-launch waits that gave up since the last reset (0: every hand-off
        matched; dkg_plan_status); synchronises the plan's stream."""
        err = ctypes.c_int(0)
        _lib.check(_lib.load().dkg_plan_status(self.host, ctypes.byref(err), int(reset),
                                               current_stream_ptr(self.device)), "dkg_plan_status")
        return err.value

    def _check_handoffs(self) -> None:
        """A fused launch whose bounded in-launch waits gave up computed on unready data: raise on the call
        that produced it (and reset the bits, so the next call starts clean)."""
        bits = self.status(reset=True)
        if bits:
            raise RuntimeError(f"fused Discrete-KG forward: in-launch hand-off wait gave up (bits 0x{bits:x}); "
                               "the result is invalid")

    def forward_into(self, X: torch.Tensor, kg: torch.Tensor, kg_pairs=None) -> None:
        """Hot path: X (device, B x d, contiguous fp64) -> kg (device, B)."""
        st = self._fwd(self.host, self._dev_ptr, X.data_ptr(), X.shape[0], kg.data_ptr(),
                       0 if kg_pairs is None else kg_pairs.data_ptr(),
                       torch.cuda.current_stream(self.device).cuda_stream)
        if st:
            _lib.check(st, "dkg_plan_forward")

    def forward_batches_into(self, X: torch.Tensor, kg: torch.Tensor, B: int) -> None:
        """K = X.shape[0] // B forward batches of B candidates in one launch per stage
        (``dkg_plan_forward_batches``): X (device, K*B x d, contiguous fp64, batch k = rows kB .. kB+B-1)
        -> kg (device, K*B).  Bit-for-bit the results of K ``forward_into`` calls, one per batch."""
        n = X.shape[0]
        if B < 1 or n % B:
            raise ValueError(f"{n} candidates are not whole batches of {B}")
        st = self._fwd_batches(self.host, self._dev_ptr, X.data_ptr(), B, n // B, kg.data_ptr(),
                               torch.cuda.current_stream(self.device).cuda_stream)
        if st:
            _lib.check(st, "dkg_plan_forward_batches")

    def forward_stats(self, X: torch.Tensor):
        """One forward with diagnostics: KG [B], KG per (candidate, scalarisation) [B, S] and the number
        of upper-envelope lines per pair [B, S] (int32; 1 = short-circuit), all on the device."""
        X = X.detach().to(self.device, torch.double).contiguous()
        B = X.shape[0]
        if B > self.max_B:
            raise ValueError(f"{B} candidates > plan capacity {self.max_B}")
        kg = torch.empty(B, dtype=torch.double, device=self.device)
        pairs = torch.empty(B, self.S, dtype=torch.double, device=self.device)
        hull = torch.empty(B, self.S, dtype=torch.int32, device=self.device)
        self.forward_into(X, kg, pairs)
        _lib.check(_lib.load().dkg_plan_hull_sizes(self.host, _lib.ptr(hull), B, current_stream_ptr(self.device)),
                   "dkg_plan_hull_sizes")
        if self.fused:
            self._check_handoffs()
        return kg, pairs, hull

    def lines(self, X: torch.Tensor):
        """The lines the envelope stage builds for candidates X (B x d), bit for bit:
        (intercepts, slopes), each [B, S, N + 1] on the device (line 0 = the candidate; dkg_plan_lines)."""
        X = X.detach().to(self.device, torch.double).contiguous()
        B = X.shape[0]
        if B > self.max_B:
            raise ValueError(f"{B} candidates > plan capacity {self.max_B}")
        a = torch.empty(B, self.S, self.state.N + 1, dtype=torch.double, device=self.device)
        b = torch.empty_like(a)
        _lib.check(_lib.load().dkg_plan_lines(self.host, self._dev_ptr, _lib.ptr(X), B, _lib.ptr(a), _lib.ptr(b),
                                              current_stream_ptr(self.device)), "dkg_plan_lines")
        return a, b

    def forward_grad(self, X: torch.Tensor):
        """KG[B] and dKG/dx [B, d] for candidates X (B x d): one C call."""
        if not self.grad:
            raise ValueError("plan was built without grad=True")
        X = X.detach().to(self.device, torch.double).contiguous()
        B = X.shape[0]
        if B > self.max_B:
            raise ValueError(f"{B} candidates > plan capacity {self.max_B}")
        kg = torch.empty(B, dtype=torch.double, device=self.device)
        dkg = torch.empty(B, self.state.d, dtype=torch.double, device=self.device)
        _lib.check(_lib.load().dkg_plan_forward_grad(self.host, self._dev_ptr, _lib.ptr(X), B, _lib.ptr(kg),
                                                     _lib.ptr(dkg), current_stream_ptr(self.device)),
                   "dkg_plan_forward_grad")
        return kg, dkg

    def forward_grad_host(self, X_host: torch.Tensor, graph: bool = False):
        """KG[B] and dKG/dx [B, d] for host candidates X (B x d), returned as host tensors: the L-BFGS-B
        evaluation of ``optimize_acqf`` (``bo_loop.py:127-129``), whose host needs both back every call.

        B x d <= DKG_XARG_MAX (the default path): one C call (``dkg_plan_forward_grad_hostx``) -- the
        candidates travel in the first kernel's arguments, the envelope kernel writes [KG | dKG/dx] into a
        plan-owned pinned buffer, the call returns after the stream has finished -- then one host copy
        out.  Larger batches, or ``graph``: one pinned H2D copy of X, the launches of
        ``dkg_plan_forward_grad`` (eager, or a HIP graph captured once per batch size; measured slower than
        eager launches at B = 1), one pinned D2H copy and one event wait.  Everything is
        ordered on the current stream of the plan's device; the results are the same bits as
        ``forward_grad``."""
        if not self.grad:
            raise ValueError("plan was built without grad=True")
        B, d = X_host.shape[0], self.state.d
        if X_host.dim() != 2 or X_host.shape[1] != d:
            raise ValueError(f"X must be B x {d}")
        if B > self.max_B:
            raise ValueError(f"{B} candidates > plan capacity {self.max_B}")
        if B == 0:
            return torch.empty(0, dtype=torch.double), torch.empty(0, d, dtype=torch.double)
        if not graph and B * d <= _lib.DKG_XARG_MAX and torch.cuda.current_device() == self.device.index:
            return self._forward_grad_hostx(X_host, B, d)
        with torch.cuda.device(self.device):
            if not graph and B * d <= _lib.DKG_XARG_MAX:
                return self._forward_grad_hostx(X_host, B, d)
            return self._forward_grad_host(X_host, B, d, graph)

    def forward_grad_host_shaped(self, X_host: torch.Tensor, B: int, kshape, xshape):
        """``forward_grad_host`` for a contiguous fp64 host tensor holding B candidates in any shape (e.g. the
        ``[*batch, 1, d]`` X of ``optimize_acqf``), the results viewed as ``kshape`` / ``xshape``: the
        B = 1 L-BFGS-B path, with no reshape of X and the results copied out once through numpy (a torch
        slice or view costs about a microsecond of host time each, on a call whose device chain is ~30 us)."""
        d = self.state.d
        if (self.grad and 0 < B <= self.max_B and B * d <= _lib.DKG_XARG_MAX
                and torch.cuda.current_device() == self.device.index):
            r = self._forward_grad_hostx_raw(X_host, B, d)
            return torch.from_numpy(r[:B].reshape(kshape)), torch.from_numpy(r[B:].reshape(xshape))
        kg, dkg = self.forward_grad_host(X_host.reshape(B, d))
        return kg.reshape(kshape), dkg.reshape(xshape)

    def _forward_grad_hostx(self, X_host: torch.Tensor, B: int, d: int):
        r = self._forward_grad_hostx_raw(X_host, B, d)
        return torch.from_numpy(r[:B]), torch.from_numpy(r[B:].reshape(B, d))

    def _forward_grad_hostx_raw(self, X_host: torch.Tensor, B: int, d: int):
        # the plan's device is current; one C call launches, lets the envelope kernel write the pinned
        # buffer and synchronises the stream; returns a numpy copy of [KG | dKG/dx]
        io = self._io.get(B) if getattr(self, "_io", None) is not None else None
        if io is None:
            self._host_buffers(d)
            dx = self._dx[:B * d]
            out = self._hout[:B * (d + 1)]
            io = self._io[B] = (dx.data_ptr(), self._dout[:B].data_ptr(), self._dout[B:B * (d + 1)].data_ptr(),
                                out.data_ptr(), out.numpy())
        xc = X_host
        if xc.dtype != torch.double or not xc.is_contiguous():
            xc = xc.to(torch.double).contiguous()
        st = self._fwd_grad_hostx(self.host, self._dev_ptr, xc.data_ptr(), io[0], B, io[1], io[2], io[3],
                                  _raw_stream(self.device))
        if st:
            _lib.check(st, "dkg_plan_forward_grad_hostx")
        return io[4].copy()

    def _host_buffers(self, d: int):
        """The pinned host and device staging buffers of the host entries (made once, sized for max_B)."""
        if getattr(self, "_hx", None) is None:
            self._hx = torch.empty(self.max_B * d, dtype=torch.double).pin_memory()
            self._hout = torch.empty(self.max_B * (d + 1), dtype=torch.double).pin_memory()
            self._dx = torch.empty(self.max_B * d, dtype=torch.double, device=self.device)
            self._dout = torch.empty(self.max_B * (d + 1), dtype=torch.double, device=self.device)
            self._done = torch.cuda.Event()
            self._graphs = {}
            self._io = {}

    def _forward_grad_host(self, X_host: torch.Tensor, B: int, d: int, graph: bool):
        # runs with the plan's device current: the copies, the launches and the event share its stream
        stream = torch.cuda.current_stream(self.device)
        self._host_buffers(d)
        dx = self._dx[:B * d].view(B, d)
        kg, dkg = self._dout[:B], self._dout[B:B * (d + 1)].view(B, d)
        lib = _lib.load()

        def launch(stream):
            _lib.check(lib.dkg_plan_forward_grad(self.host, self._dev_ptr, _lib.ptr(dx), B, _lib.ptr(kg),
                                                 _lib.ptr(dkg), stream), "dkg_plan_forward_grad")

        hx = self._hx[:B * d].view(B, d)
        hx.copy_(X_host.detach().reshape(B, d))
        dx.copy_(hx, non_blocking=True)
        if graph:
            g = self._graphs.get(B)
            if g is None:
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    launch(torch.cuda.current_stream(self.device).cuda_stream)
                self._graphs[B] = g
                torch.cuda.synchronize(self.device)
            g.replay()
        else:
            launch(stream.cuda_stream)
        out = self._hout[:B * (d + 1)]
        out.copy_(self._dout[:B * (d + 1)], non_blocking=True)
        self._done.record(stream)
        self._done.synchronize()
        return out[:B].clone(), out[B:].view(B, d).clone()

    def forward_host(self, X_host: torch.Tensor) -> torch.Tensor:
        """KG[B] for host candidates X (B x d) as a host tensor: one pinned H2D copy, the forward's launches
        and one pinned D2H copy on the plan device's current stream (``forward`` of a host X without grad)."""
        B, d = X_host.shape[0], self.state.d
        if X_host.dim() != 2 or X_host.shape[1] != d:
            raise ValueError(f"X must be B x {d}")
        if B > self.max_B:
            raise ValueError(f"{B} candidates > plan capacity {self.max_B}")
        if B == 0:
            return torch.empty(0, dtype=torch.double)
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device)
            self._host_buffers(d)
            hx = self._hx[:B * d].view(B, d)
            hx.copy_(X_host.detach().reshape(B, d))
            dx = self._dx[:B * d].view(B, d)
            dx.copy_(hx, non_blocking=True)
            kg = self._dout[:B]
            st = self._fwd(self.host, self._dev_ptr, dx.data_ptr(), B, kg.data_ptr(), 0, stream.cuda_stream)
            if st:
                _lib.check(st, "dkg_plan_forward")
            out = self._hout[:B]
            out.copy_(kg, non_blocking=True)
            self._done.record(stream)
            self._done.synchronize()
            if self.fused:
                self._check_handoffs()
            return out.clone()

    def time_stage(self, X: torch.Tensor, stage: int, reps: int) -> float:
        """Average duration (ms) of ``reps`` back-to-back launches of one kernel
        (0 cross_root, 1 posterior_cov, 2 envelope; 3 the whole forward as ``forward_into`` launches it),
        HIP events on the launch stream."""
        X = X.detach().to(self.device, torch.double).contiguous()
        kg = torch.empty(X.shape[0], dtype=torch.double, device=self.device)
        ms = _lib.c_float()
        _lib.check(_lib.load().dkg_plan_time_stage(self.host, self._dev_ptr, _lib.ptr(X), X.shape[0], _lib.ptr(kg),
                                                   None, current_stream_ptr(self.device), stage, reps,
                                                   ctypes.byref(ms)), "dkg_plan_time_stage")
        return ms.value

    def time_stage_batches(self, X: torch.Tensor, B: int, stage: int, reps: int) -> float:
        """time_stage for the launches of ``forward_batches_into`` (X: K*B candidates, K batches of B)."""
        X = X.detach().to(self.device, torch.double).contiguous()
        if B < 1 or X.shape[0] % B:
            raise ValueError(f"{X.shape[0]} candidates are not whole batches of {B}")
        kg = torch.empty(X.shape[0], dtype=torch.double, device=self.device)
        ms = _lib.c_float()
        _lib.check(_lib.load().dkg_plan_time_stage_batches(self.host, self._dev_ptr, _lib.ptr(X), B, X.shape[0] // B,
                                                           _lib.ptr(kg), current_stream_ptr(self.device), stage,
                                                           reps, ctypes.byref(ms)), "dkg_plan_time_stage_batches")
        return ms.value

    def forward(self, X: torch.Tensor, kg_pairs=None, timed: bool = False):
        X = X.detach().to(self.device, torch.double).contiguous()
        B = X.shape[0]
        if B > self.max_B:
            raise ValueError(f"{B} candidates > plan capacity {self.max_B}")
        kg = torch.empty(B, dtype=torch.double, device=self.device)
        if timed:
            ms = (_lib.c_float * 3)()
            _lib.check(self._fwd_timed(self.host, self._dev_ptr, _lib.ptr(X), B, _lib.ptr(kg), _lib.ptr(kg_pairs),
                                       current_stream_ptr(self.device), ms), "dkg_plan_forward_timed")
            return kg, list(ms)
        self.forward_into(X, kg, kg_pairs)
        return kg
