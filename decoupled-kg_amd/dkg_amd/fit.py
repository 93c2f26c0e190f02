"""MAP hyperparameter fitting of the BO surrogate: the ``once`` / ``always`` paths of the reference's model
step (SURVEY.md §8(f) rank 4 remainder), without GPyTorch or BoTorch.

What it restates (reference files, read for behaviour only):

* ``modules/model/factory.py:24-60, 63-151`` ``build_mll_and_model``: per output a ``SingleTaskGP`` with a
  ``ConstantMean`` (no prior), ``ScaleKernel(MaternKernel(nu, ard_num_dims=d, lengthscale_prior=Gamma))`` with an
  ``outputscale_prior`` Gamma, and a ``GaussianLikelihood`` whose noise has a Gamma prior and the constraint
  ``GreaterThan(min_noise_se**2, transform=None, initial_value=prior.mode)`` -- no transform, so the noise is its
  raw value; a ``SumMarginalLogLikelihood`` over the outputs;
* GPyTorch's parametrisation and objective, as those modules use it: lengthscales and outputscale through
  ``Positive()`` (softplus of a raw value initialised at 0), the constant initialised at 0, and
  ``ExactMarginalLogLikelihood`` = (log N(y | c, s K + noise I) + the log priors) / n per output;
* ``pipeline/nodes/bo_loop.py:63-79`` ``fit_hyperparameters`` (``once``: n = 1000 Sobol points of the problem,
  ``fix_zero_noise`` outputs pinned at ``MIN_NOISE_SE**2`` and not fitted, ``fit_gpytorch_mll``) and
  ``:589-619`` (``always``: refit at every iteration; after the first, the constants stay at the first fit's);
* ``fit_gpytorch_mll``'s default optimiser: scipy L-BFGS-B over the raw parameters of every output at once.

Parity unpinned: BoTorch / GPyTorch are absent here and the reference ships no fitted hyperparameters for
these problems.  GPyTorch also switches from Cholesky to CG / Lanczos estimates of the solve and log-determinant
above ``max_cholesky_size`` = 800 training points (the ``once`` path's 1000), where this module keeps the
exact Cholesky objective.  tests/test_fit.py checks the objective against a numpy restatement, the gradient
against central differences, and recovery of known hyperparameters.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch import Tensor

MIN_NOISE_SE = 1e-2  # factory.py:15 (fitted paths)
JITTERS = (1e-8, 1e-7, 1e-6)  # psd_safe_cholesky's retries for float64


def gamma_log_prob(x: Tensor, concentration: float, rate: float) -> Tensor:
    """GammaPrior(concentration, rate).log_prob(x), summed over x's entries."""
    a, b = float(concentration), float(rate)
    return (a * math.log(b) - math.lgamma(a) + (a - 1.0) * torch.log(x) - b * x).sum()


def matern(X: Tensor, lengthscale: Tensor, nu: float) -> Tensor:
    """kappa(||(x - x') / l||) of MaternKernel (nu 0.5, 1.5, 2.5) or, nu = inf, RBFKernel."""
    Z = X / lengthscale
    sq = (Z * Z).sum(-1)
    r2 = (sq[:, None] + sq[None, :] - 2.0 * Z @ Z.T).clamp_min(1e-30)
    if math.isinf(nu):
        return torch.exp(-0.5 * r2)
    r = r2.sqrt()
    if nu == 0.5:
        return torch.exp(-r)
    if nu == 1.5:
        t = math.sqrt(3.0) * r
        return (1.0 + t) * torch.exp(-t)
    t = math.sqrt(5.0) * r
    return (1.0 + t + t * t / 3.0) * torch.exp(-t)


def _chol(K: Tensor) -> Tensor:
    L, info = torch.linalg.cholesky_ex(K)
    if int(info) == 0:
        return L
    eye = torch.eye(K.shape[0], dtype=K.dtype)
    for j in JITTERS:
        L, info = torch.linalg.cholesky_ex(K + j * eye)
        if int(info) == 0:
            return L
    raise torch.linalg.LinAlgError("kernel matrix not positive definite after jitter")


def _prior(cfg: Optional[dict]):
    if not cfg:
        return None
    if cfg.get("type") != "gamma":
        raise ValueError(f"Unsupported prior 'type'. Got {cfg.get('type')!r}.")
    return float(cfg["args"]["concentration"]), float(cfg["args"]["rate"])


class _Output:
    """One output's data, priors and the slice of the raw parameter vector it owns."""

    def __init__(self, X: Tensor, y: Tensor, cfg: dict, min_noise_se: float, fixed_mean: Optional[float]):
        self.X, self.y = X, y
        self.n, self.d = X.shape
        kern = cfg.get("kernel") or {}
        self.nu = float((kern.get("args") or {}).get("nu", 2.5)) if kern.get("type", "matern") == "matern" else math.inf
        self.ard = bool(kern.get("ard", True))
        self.ls_prior = _prior(kern.get("lengthscale_prior"))
        self.os_prior = _prior(kern.get("outputscale_prior"))
        lik = cfg.get("likelihood") or {}
        self.noise_prior = _prior(lik.get("noise_prior"))
        self.fix_noise = bool(cfg.get("fix_zero_noise", False))
        # fix_zero_noise pins the noise at MIN_NOISE_SE**2 (bo_loop.py:74-77, 594-597); otherwise it starts at
        # the prior's mode (initial_value=prior.mode, factory.py:102-104) and is fitted untransformed
        self.noise0 = (min_noise_se ** 2 if self.fix_noise else
                       ((self.noise_prior[0] - 1.0) / self.noise_prior[1] if self.noise_prior else 1e-4))
        self.fixed_mean = fixed_mean
        nls = self.d if self.ard else 1
        # raw layout: [constant (unless fixed)] [raw lengthscales] [raw outputscale] [noise (unless fixed)]
        self.n_raw = (0 if fixed_mean is not None else 1) + nls + 1 + (0 if self.fix_noise else 1)
        self.nls = nls

    def initial(self) -> List[float]:
        v = [] if self.fixed_mean is not None else [0.0]
        return v + [0.0] * self.nls + [0.0] + ([] if self.fix_noise else [self.noise0])

    def unpack(self, raw: Tensor):
        k = 0
        if self.fixed_mean is None:
            c = raw[0]
            k = 1
        else:
            c = torch.tensor(self.fixed_mean, dtype=raw.dtype)
        ls = torch.nn.functional.softplus(raw[k:k + self.nls])
        os = torch.nn.functional.softplus(raw[k + self.nls])
        noise = torch.tensor(self.noise0, dtype=raw.dtype) if self.fix_noise else raw[k + self.nls + 1]
        return c, ls, os, noise

    def mll(self, raw: Tensor) -> Tensor:
        """ExactMarginalLogLikelihood of this output (divided by n), priors included."""
        c, ls, os, noise = self.unpack(raw)
        lsv = ls if self.ard else ls.expand(self.d)
        K = os * matern(self.X, lsv, self.nu) + noise * torch.eye(self.n, dtype=self.X.dtype)
        L = _chol(K)
        r = (self.y - c).unsqueeze(-1)
        a = torch.linalg.solve_triangular(L, r, upper=False)
        logp = -0.5 * (a * a).sum() - torch.log(torch.diagonal(L)).sum() - 0.5 * self.n * math.log(2.0 * math.pi)
        lp = torch.zeros((), dtype=self.X.dtype)
        if self.ls_prior:
            lp = lp + gamma_log_prob(ls, *self.ls_prior)
        if self.os_prior:
            lp = lp + gamma_log_prob(os.reshape(1), *self.os_prior)
        if self.noise_prior:
            lp = lp + gamma_log_prob(noise.reshape(1), *self.noise_prior)
        return (logp + lp) / self.n


def fit_map(train_x: Sequence[Tensor], train_y: Sequence[Tensor], model_config: dict,
            fixed_means: Optional[Sequence[float]] = None, max_iter: int = 1000) -> Dict[str, object]:
    """Maximise the SumMarginalLogLikelihood of a ModelListGP built from ``model_config`` (the reference's
    ``model`` section: ``outputs[i]`` priors and ``fix_zero_noise``, ``fit_hyperparams``) on output i's data
    (train_x[i] in [0, 1]^d, train_y[i]); ``fixed_means``: the ``always`` path's constants after its first fit.
    Returns ``length_scales``, ``output_scales``, ``means``, ``noises`` (per output, bo_smoke's ``hyper``
    layout), the final objective ``mll`` and the optimiser's ``success`` / ``iterations``."""
    from scipy.optimize import minimize

    min_noise_se = 1e-4 if model_config.get("fit_hyperparams", "once") == "never" else MIN_NOISE_SE
    outs = [_Output(torch.as_tensor(train_x[i], dtype=torch.double), torch.as_tensor(train_y[i], dtype=torch.double),
                    model_config["outputs"][i], min_noise_se, None if fixed_means is None else float(fixed_means[i]))
            for i in range(len(train_x))]
    x0 = np.array([v for o in outs for v in o.initial()], dtype=np.float64)
    bounds = []
    for o in outs:
        bounds += [(None, None)] * (o.n_raw - (0 if o.fix_noise else 1))
        if not o.fix_noise:
            bounds.append((None, None))  # transform=None: the constraint is not enforced (factory.py:100-104)

    def split(raw: Tensor):
        k = 0
        for o in outs:
            yield o, raw[k:k + o.n_raw]
            k += o.n_raw

    def objective(v: np.ndarray):
        raw = torch.tensor(v, dtype=torch.double, requires_grad=True)
        loss = -sum(o.mll(r) for o, r in split(raw))
        (g,) = torch.autograd.grad(loss, raw)
        return float(loss.detach()), g.numpy().astype(np.float64)

    res = minimize(objective, x0, jac=True, method="L-BFGS-B", bounds=bounds, options={"maxiter": max_iter})
    raw = torch.tensor(res.x, dtype=torch.double)
    hyper: Dict[str, list] = {"length_scales": [], "output_scales": [], "means": [], "noises": []}
    for o, r in split(raw):
        c, ls, os, noise = o.unpack(r)
        hyper["length_scales"].append((ls if o.ard else ls.expand(o.d)).tolist())
        hyper["output_scales"].append(float(os))
        hyper["means"].append(float(c))
        hyper["noises"].append(float(noise))
    return {**hyper, "mll": -float(res.fun), "success": bool(res.success), "iterations": int(res.nit)}


def neg_mll(train_x: Sequence[Tensor], train_y: Sequence[Tensor], model_config: dict,
            hyper: Dict[str, Sequence]) -> float:
    """The SumMarginalLogLikelihood at given hyperparameters (means, length_scales, output_scales, noises)."""
    min_noise_se = 1e-4 if model_config.get("fit_hyperparams", "once") == "never" else MIN_NOISE_SE
    total = 0.0
    for i in range(len(train_x)):
        o = _Output(torch.as_tensor(train_x[i], dtype=torch.double), torch.as_tensor(train_y[i], dtype=torch.double),
                    model_config["outputs"][i], min_noise_se, float(hyper["means"][i]))
        ls = torch.as_tensor(hyper["length_scales"][i], dtype=torch.double).reshape(-1)
        raw = [ls + torch.log(-torch.expm1(-ls)),
               torch.tensor([float(hyper["output_scales"][i])], dtype=torch.double)]
        raw[1] = raw[1] + torch.log(-torch.expm1(-raw[1]))
        if not o.fix_noise:
            raw.append(torch.tensor([float(hyper["noises"][i])], dtype=torch.double))
        total += float(o.mll(torch.cat(raw)))
    return -total
