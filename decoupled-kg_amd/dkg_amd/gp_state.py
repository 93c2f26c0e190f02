"""Device-resident GP state for the Discrete-KG kernels.

Builds, per output, the caches GPyTorch's exact prediction keeps behind
``model.posterior`` (``discretekg.py:182-185, 275-284``) — the ones BoTorch's
``fast_pred_var`` posterior uses:

* ``K = s k(X, X) + noise I``                 HIP ``dkg_kernel_matrix``
* ``L = psd_safe_cholesky(K)``                torch.linalg on the GPU, with
  linear_operator's jitter policy (absolute 1e-8 * 10**i, 3 retries)
* ``R = L^{-T}`` (root_inv_decomposition)     torch.linalg.solve_triangular
* ``alpha = cholesky_solve(y - c, L)``        torch.cholesky_solve
* ``root_frag`` = R in MFMA fragment order    HIP ``dkg_pack_root``
* ``Q_D = K(D, X) R``, ``mu_D = c + K(D,X) alpha`` over the discretisation
                                              HIP ``dkg_cross_root``

All of it runs once per (model, discretisation) — the reference rebuilds the
same caches once per BO iteration — and stays in HBM for every forward call.
"""

from __future__ import annotations

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


def psd_safe_cholesky(A: torch.Tensor, jitter: float = 1e-8, max_tries: int = 3) -> torch.Tensor:
    L, info = torch.linalg.cholesky_ex(A)
    if int(info) == 0:
        return L
    prev = 0.0
    Ap = A.clone()
    eye = torch.eye(A.shape[-1], dtype=A.dtype, device=A.device)
    for i in range(max_tries):
        new = jitter * 10**i
        Ap = Ap + (new - prev) * eye
        prev = new
        L, info = torch.linalg.cholesky_ex(Ap)
        if int(info) == 0:
            return L
    raise torch.linalg.LinAlgError("covariance not positive definite after jitter retries (NotPSDError)")


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


def prepare_output(st: SingleTaskGPState, D: torch.Tensor) -> OutputCache:
    """Build one output's device caches over the discretisation ``D`` (device, N x d)."""
    lib = _lib.load()
    dev = D.device
    stream = current_stream_ptr(dev)
    n, d = st.train_x.shape
    N = D.shape[0]
    if _pad16(n) > 1024:
        raise UnsupportedError(f"n={n} training points > 1024 per output is not supported")
    X = st.train_x.to(dev).contiguous()
    inv_ls = (1.0 / st.lengthscale).to(dev).contiguous()
    o = _base_struct(st, inv_ls, X)

    K = torch.empty(n, n, dtype=torch.double, device=dev)
    _lib.check(lib.dkg_kernel_matrix(o, d, _lib.ptr(X), n, _lib.ptr(X), n, float(st.noise), _lib.ptr(K), stream),
               "dkg_kernel_matrix")
    L = psd_safe_cholesky(K)
    eye = torch.eye(n, dtype=torch.double, device=dev)
    R = torch.linalg.solve_triangular(L, eye, upper=False).mT.contiguous()
    y = st.train_y.to(dev)
    alpha = torch.zeros(_pad16(n), dtype=torch.double, device=dev)
    alpha[:n] = torch.cholesky_solve((y - st.mean_constant).unsqueeze(-1), L).squeeze(-1)

    root_frag = torch.empty(lib.dkg_frag_elems(n, n), dtype=torch.double, device=dev)
    _lib.check(lib.dkg_pack_root(_lib.ptr(R), n, _lib.ptr(root_frag), stream), "dkg_pack_root")
    o.alpha = _lib.ptr(alpha)
    o.root_frag = _lib.ptr(root_frag)

    disc_frag = torch.empty(max(1, lib.dkg_frag_elems(N, n)), dtype=torch.double, device=dev)
    disc_mean = torch.empty(max(16, _pad16(N)), dtype=torch.double, device=dev)
    if N > 0:
        _lib.check(lib.dkg_cross_root(o, d, _lib.ptr(D), N, _lib.ptr(disc_frag), _lib.ptr(disc_mean), stream),
                   "dkg_cross_root")
    o.disc_frag = _lib.ptr(disc_frag)
    o.disc_mean = _lib.ptr(disc_mean)
    return OutputCache(st, inv_ls, X, alpha, root_frag, disc_frag, disc_mean, L, o)


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
        self.outputs: List[OutputCache] = [prepare_output(m, self.D) for m in model.models]
        self.m = len(self.outputs)
        self.structs = (_lib.DkgOutput * self.m)(*[c.struct for c in self.outputs])
        self._ws = None
        self._ws_key = None

    def workspace(self, B: int, S: int) -> torch.Tensor:
        lib = _lib.load()
        need = lib.dkg_forward_workspace(self.structs, self.m, self.N, B, S)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.zeros(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def forward(self, X: torch.Tensor, W: torch.Tensor, target, kg_pairs=None, timed: bool = False):
        """kg[B] for candidates X (device, B x d) and weights W (device, S x m)."""
        lib = _lib.load()
        X = X.detach().to(self.device, torch.double).contiguous()
        W = W.detach().to(self.device, torch.double).contiguous()
        B = X.shape[0]
        S = W.shape[0]
        kg = torch.empty(B, dtype=torch.double, device=self.device)
        ws = self.workspace(B, S)
        stream = current_stream_ptr(self.device)
        tgt = -1 if target is None else int(target)
        args = (self.structs, self.m, self.d, _lib.ptr(self.D), self.N, _lib.ptr(X), B, _lib.ptr(W), S, tgt,
                _lib.ptr(kg), _lib.ptr(kg_pairs), _lib.ptr(ws), ws.numel(), stream)
        if timed:
            ms = (_lib.c_float * 3)()
            _lib.check(lib.dkg_forward_timed(*args, ms), "dkg_forward_timed")
            return kg, list(ms)
        _lib.check(lib.dkg_forward(*args), "dkg_forward")
        return kg
