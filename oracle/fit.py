"""ORACLE (test infrastructure only) — MAP fit of the reference test models.

The end-to-end known answers of the reference
(``tests/modules/acquisition/test_discretekg.py:62,78,93,108``) are taken on a
ModelListGP of two *default* BoTorch SingleTaskGPs fitted with
``fit_gpytorch_mll(SumMarginalLogLikelihood)``
(``tests/modules/acquisition/conftest.py:30-47``).  BoTorch@c14808f and
GPyTorch 1.11 are not installable here, so this module restates:

* ``draw_sobol_samples(bounds, n, q=1, seed)``: scrambled ``SobolEngine(q*d,
  seed)`` draw scaled into the bounds (torch core);
* the default SingleTaskGP of that BoTorch release: Matern-5/2 with ARD,
  lengthscale prior Gamma(3, 6), ScaleKernel outputscale prior
  Gamma(2, 0.15), ConstantMean, GaussianLikelihood with noise prior
  Gamma(1.1, 0.05) and ``GreaterThan(1e-4, transform=None)`` noise
  constraint initialised at the prior mode (2.0); softplus-constrained
  lengthscale / outputscale with raw initial value 0;
* ``fit_gpytorch_mll`` on a SumMarginalLogLikelihood over a ModelListGP:
  each sub-model's ExactMarginalLogLikelihood is fitted independently by
  ``scipy.optimize.minimize(method="L-BFGS-B", jac=True)`` with default
  options, over the raw parameters that require grad, with bounds only for
  non-enforced constraints (the noise lower bound 1e-4);
* the loss ``-(log N(y; c, K + s2 I) + sum log-priors) / n`` with GPyTorch's
  Cholesky-based ``inv_quad_logdet`` (logdet = sum log diag(L)^2).

These defaults are external and cannot be verified offline; the KAT tests
record how closely they reproduce the reference numbers.
"""

from __future__ import annotations

import math

import numpy as np
import torch
from scipy.optimize import minimize

from .gp import DTYPE, ModelList, OutputGP, base_kernel, psd_safe_cholesky


def draw_sobol_samples(bounds: torch.Tensor, n: int, q: int, seed: int) -> torch.Tensor:
    lower, upper = bounds[0], bounds[1]
    d = bounds.shape[-1]
    eng = torch.quasirandom.SobolEngine(q * d, scramble=True, seed=seed)
    raw = eng.draw(n, dtype=lower.dtype).view(n, q, d)
    return lower + (upper - lower) * raw


def _gamma_logpdf(x, conc, rate):
    return conc * math.log(rate) + (conc - 1.0) * torch.log(x) - rate * x - math.lgamma(conc)


def _softplus(x):
    return torch.nn.functional.softplus(x)


def fit_default_single_task_gp(train_x: torch.Tensor, train_y: torch.Tensor,
                               fixed_noise: float | None = None) -> OutputGP:
    """MAP-fit one default SingleTaskGP; returns its constrained state."""
    n, d = train_x.shape
    y = train_y.reshape(-1).to(DTYPE)
    # raw parameters in SingleTaskGP.named_parameters() order
    names = []
    init = []
    if fixed_noise is None:
        names.append("raw_noise")
        init.append(np.array([2.0]))
    names += ["raw_constant", "raw_outputscale", "raw_lengthscale"]
    init += [np.array([0.0]), np.array([0.0]), np.zeros(d)]
    sizes = [len(v) for v in init]
    x0 = np.concatenate(init)
    lo = np.full(x0.shape, -np.inf)
    if fixed_noise is None:
        lo[0] = 1e-4

    def unpack(theta):
        parts = torch.split(theta, sizes)
        p = dict(zip(names, parts))
        noise = p["raw_noise"][0] if fixed_noise is None else torch.tensor(fixed_noise, dtype=DTYPE)
        return noise, p["raw_constant"][0], _softplus(p["raw_outputscale"][0]), _softplus(p["raw_lengthscale"]).reshape(1, d)

    def loss_fn(theta):
        noise, c, s, ls = unpack(theta)
        K = s * base_kernel(train_x, train_x, ls, "matern", 2.5)
        K = K + noise * torch.eye(n, dtype=DTYPE)
        L = psd_safe_cholesky(K)
        diff = (y - c).unsqueeze(-1)
        inv_quad = (diff * torch.cholesky_solve(diff, L)).sum()
        logdet = L.diagonal().pow(2).log().sum()
        ll = -0.5 * (inv_quad + logdet + n * math.log(2 * math.pi))
        ll = ll + _gamma_logpdf(noise, 1.1, 0.05)
        ll = ll + _gamma_logpdf(ls, 3.0, 6.0).sum()
        ll = ll + _gamma_logpdf(s, 2.0, 0.15)
        return -ll / n

    def fun(x):
        theta = torch.tensor(x, dtype=DTYPE, requires_grad=True)
        val = loss_fn(theta)
        (g,) = torch.autograd.grad(val, theta)
        return float(val.detach()), g.detach().numpy().astype(np.float64)

    bounds = None if fixed_noise is not None else list(zip(lo, np.full(x0.shape, np.inf)))
    res = minimize(fun, x0, jac=True, method="L-BFGS-B", bounds=bounds)
    with torch.no_grad():
        noise, c, s, ls = unpack(torch.tensor(res.x, dtype=DTYPE))
    return OutputGP(train_x.clone(), y.clone(), ls.reshape(-1), float(s), float(noise), float(c))


def make_reference_test_model(use_noise: bool = True, seed: int = 1234) -> ModelList:
    """``tests/modules/acquisition/conftest.py:30-47`` with the seed of ``tests/conftest.py:5-9``."""
    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=DTYPE)
    state = torch.random.get_rng_state()
    try:
        torch.manual_seed(seed)
        train_x = draw_sobol_samples(bounds, 10, q=1, seed=seed).squeeze(-2)
        train_y = torch.randn(10, 2, dtype=DTYPE)
    finally:
        torch.random.set_rng_state(state)
    fixed = None if use_noise else 1e-4
    return ModelList([fit_default_single_task_gp(train_x, train_y[:, i], fixed) for i in range(2)])


def reference_test_discretisation() -> torch.Tensor:
    """3x3 grid of ``test_discretekg.py:17-25``."""
    g = torch.linspace(0, 1, 3, dtype=DTYPE)
    return torch.stack([torch.repeat_interleave(g, 3), torch.tile(g, (3,))]).T
