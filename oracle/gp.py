"""ORACLE (test infrastructure only) — GP posterior semantics the hot path consumes.

The reference's KG functions call ``model.posterior(...)`` at
``src/decoupledbo/modules/acquisition/discretekg.py:182-185`` (ModelListGP,
full evaluation) and ``:275-284`` (per sub-model, decoupled).  The models are
built by ``src/decoupledbo/modules/model/factory.py:63-135``: a ModelListGP of
SingleTaskGPs with ``ScaleKernel(Matern(nu)|RBF, ARD)``, ``ConstantMean``,
``GaussianLikelihood`` and an optional ``Standardize(m=1)`` outcome transform.

The posterior arithmetic lives in external libraries pinned by the reference
(gpytorch==1.11, linear-operator==0.5.1, botorch@c14808f).  They are NOT
vendored in /root/reference and not installed here, so this module restates
their published algorithm at those call sites:

* kernels: gpytorch ``MaternKernel.forward`` (inputs centred on the mean of
  x1, divided by the lengthscale), ``RBFKernel`` (``exp(-sq_dist/2)``),
  ``ScaleKernel`` (outputscale *), with gpytorch's ``sq_dist`` quadratic
  expansion for ``x1 == x2`` blocks and ``torch.cdist`` (clamped at 1e-15)
  otherwise;
* ``psd_safe_cholesky``: plain Cholesky, then up to 3 retries adding absolute
  diagonal jitter 1e-8 * 10**i (double) on failure;
* exact prediction with ``fast_pred_var`` (BoTorch's ``gpt_posterior_settings``):
  ``mean = c + K*X @ alpha`` with ``alpha = cholesky_solve(y - c, L)``, and
  ``cov = K** - (K*X R)(K*X R)^T`` with the root ``R = L^{-T}`` obtained by an
  explicit triangular inverse (linear_operator ``root_inv_decomposition``);
  the test rows of the joint [train; test] kernel are evaluated eagerly as
  one block ``K(test, [train; test])`` (gpytorch ``exact_prediction``);
* ``observation_noise=True`` adds the likelihood noise to the diagonal;
* ``Standardize.untransform_posterior``: ``mean*sd + mu``, ``cov*sd^2``.

Rounding-level choices of those libraries that cannot be checked offline are
noted where they occur; they perturb results at the 1e-16 relative level and
are covered by the parity tolerance (DESIGN.md "Parity tolerance").
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
from torch import Tensor

DTYPE = torch.double


def _as_row(v, d: int) -> Tensor:
    t = torch.as_tensor(v, dtype=DTYPE)
    if t.dim() == 0:
        t = t.repeat(d)
    return t.reshape(1, d)


@dataclass
class OutputGP:
    """State of one fitted SingleTaskGP (one output of the ModelListGP).

    ``train_y`` is in *model space*, i.e. already standardised when a
    Standardize outcome transform is present (``y_mean``/``y_std`` then hold
    the transform's means/stdvs); factory.py:75-78.
    """

    train_x: Tensor
    train_y: Tensor
    lengthscale: Tensor
    outputscale: float
    noise: float
    mean_constant: float = 0.0
    kernel: str = "matern"
    nu: float = 2.5
    y_mean: float = 0.0
    y_std: float = 1.0
    _cache: Optional[dict] = field(default=None, repr=False)

    def __post_init__(self):
        self.train_x = torch.as_tensor(self.train_x, dtype=DTYPE)
        self.train_y = torch.as_tensor(self.train_y, dtype=DTYPE).reshape(-1)
        self.lengthscale = _as_row(self.lengthscale, self.train_x.shape[-1])

    # -- kernel -------------------------------------------------------------
    def covar(self, x1: Tensor, x2: Tensor) -> Tensor:
        return self.outputscale * base_kernel(x1, x2, self.lengthscale, self.kernel, self.nu)

    # -- caches (GPyTorch DefaultPredictionStrategy) ------------------------
    def cache(self) -> dict:
        if self._cache is None:
            X = self.train_x
            K = self.covar(X, X)
            K = K + self.noise * torch.eye(K.shape[-1], dtype=DTYPE)
            L = psd_safe_cholesky(K)
            eye = torch.eye(L.shape[-1], dtype=DTYPE)
            R = torch.linalg.solve_triangular(L, eye, upper=False).mT
            alpha = torch.cholesky_solve((self.train_y - self.mean_constant).unsqueeze(-1), L).squeeze(-1)
            self._cache = {"L": L, "R": R, "alpha": alpha}
        return self._cache

    # -- posterior (BoTorch GPyTorchModel.posterior for one SingleTaskGP) ----
    def posterior(self, Xt: Tensor, observation_noise: bool = False):
        """Return (mean[q], cov[q, q]) of the untransformed posterior at ``Xt``."""
        c = self.cache()
        n = self.train_x.shape[0]
        joint = torch.cat([self.train_x, Xt], dim=0)
        test_rows = self.covar(Xt, joint)  # eager K(test, [train; test]) block
        test_train = test_rows[:, :n]
        test_test = test_rows[:, n:]
        mean = test_train @ c["alpha"] + self.mean_constant
        Q = test_train @ c["R"]
        cov = test_test - Q @ Q.mT
        if observation_noise:
            cov = cov + self.noise * torch.eye(cov.shape[-1], dtype=DTYPE)
        return mean * self.y_std + self.y_mean, cov * (self.y_std**2)


def base_kernel(x1: Tensor, x2: Tensor, lengthscale: Tensor, kind: str, nu: float) -> Tensor:
    """gpytorch 1.11 Matern/RBF ``forward`` (non-diag, ARD) restated."""
    if kind == "matern":
        centre = x1.reshape(-1, x1.shape[-1]).mean(0)
        z1 = (x1 - centre) / lengthscale
        z2 = (x2 - centre) / lengthscale
        r = _dist(z1, z2)
        e = torch.exp(-math.sqrt(2.0 * nu) * r)
        if nu == 0.5:
            return e
        if nu == 1.5:
            return (math.sqrt(3.0) * r + 1.0) * e
        if nu == 2.5:
            return (math.sqrt(5.0) * r + 1.0 + (5.0 / 3.0) * r**2) * e
        raise ValueError(f"unsupported Matern nu={nu}")
    if kind == "rbf":
        z1 = x1 / lengthscale
        z2 = x2 / lengthscale
        return torch.exp(-0.5 * _sq_dist(z1, z2, torch.equal(z1, z2)))
    raise ValueError(f"unsupported kernel {kind!r}")


def _sq_dist(x1: Tensor, x2: Tensor, x1_eq_x2: bool) -> Tensor:
    """gpytorch ``sq_dist``: centred quadratic expansion, clamped at 0."""
    shift = x1.mean(-2, keepdim=True)
    a = x1 - shift
    na = a.pow(2).sum(-1, keepdim=True)
    grad = x1.requires_grad or x2.requires_grad
    if x1_eq_x2 and not grad:
        b, nb = a, na
    else:
        b = x2 - shift
        nb = b.pow(2).sum(-1, keepdim=True)
    lhs = torch.cat([-2.0 * a, na, torch.ones_like(na)], dim=-1)
    rhs = torch.cat([b, torch.ones_like(nb), nb], dim=-1)
    res = lhs @ rhs.mT
    if x1_eq_x2 and not grad:
        res = res.clone()
        res.diagonal().fill_(0.0)
    return res.clamp_min(0.0)


def _dist(x1: Tensor, x2: Tensor) -> Tensor:
    """gpytorch ``dist``: cdist (clamped 1e-15) unless x1 == x2."""
    if not torch.equal(x1, x2):
        return torch.cdist(x1, x2).clamp_min(1e-15)
    return _sq_dist(x1, x2, True).clamp_min(1e-30).sqrt()


def psd_safe_cholesky(A: Tensor, jitter: float = 1e-8, max_tries: int = 3) -> Tensor:
    """linear_operator 0.5.1 ``psd_safe_cholesky`` (absolute jitter, 3 tries)."""
    L, info = torch.linalg.cholesky_ex(A)
    if int(info) == 0:
        return L
    Ap = A.clone()
    prev = 0.0
    for i in range(max_tries):
        new = jitter * (10**i)
        Ap = Ap + (new - prev) * torch.eye(A.shape[-1], dtype=A.dtype)
        prev = new
        L, info = torch.linalg.cholesky_ex(Ap)
        if int(info) == 0:
            return L
    raise RuntimeError("NotPSDError: matrix not positive definite after jitter retries")


@dataclass
class ModelList:
    """ModelListGP stand-in: independent outputs (factory.py:45-56)."""

    models: List[OutputGP]

    @property
    def num_outputs(self) -> int:
        return len(self.models)

    def posterior_list(self, Xt: Tensor, observation_noise: bool = False):
        return [m.posterior(Xt, observation_noise) for m in self.models]


def model_list_from_state_dict(state: dict, train_x: Tensor, train_y: Tensor,
                               kernel: str = "matern", nu: float = 2.5) -> ModelList:
    """Build a ModelList from the reference's ``.pt`` GP-problem format.

    Format written by ``src/decoupledbo/pipeline/data_catalog.py:99-111``
    (``model_state_dict`` of a ModelListGP, raw GPyTorch parameters).  Raw
    values go through GPyTorch's constraint transforms: Positive/Interval =
    ``softplus`` + lower bound for lengthscale/outputscale; the noise
    constraint ``GreaterThan(lb)`` likewise (``raw_noise=-inf`` -> lb).
    """
    sd = {k: torch.as_tensor(v, dtype=DTYPE) for k, v in state.items()}
    models = []
    i = 0
    while f"models.{i}.covar_module.raw_outputscale" in sd:
        p = f"models.{i}."

        def cons(raw_key):
            lb = sd.get(p + raw_key + "_constraint.lower_bound", torch.tensor(0.0, dtype=DTYPE))
            return torch.nn.functional.softplus(sd[p + raw_key]) + lb

        ls = cons("covar_module.base_kernel.raw_lengthscale").reshape(-1)
        os_ = float(cons("covar_module.raw_outputscale"))
        noise = float(cons("likelihood.noise_covar.raw_noise").reshape(-1)[0])
        c = float(sd.get(p + "mean_module.raw_constant", torch.tensor(0.0, dtype=DTYPE)))
        models.append(OutputGP(train_x, train_y[:, i], ls, os_, noise, c, kernel, nu))
        i += 1
    return ModelList(models)
