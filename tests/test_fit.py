"""MAP hyperparameter fitting (dkg_amd.fit; the reference's once / always model paths, bo_loop.py:63-79,
589-619, factory.py:24-151).  Parity with fit_gpytorch_mll is unpinned (BoTorch / GPyTorch are absent):
these tests pin the objective against a numpy restatement, its gradient against central differences, and
the optimiser against the data's own optimum (the fit's objective beats the generating hyperparameters')."""

import math

import numpy as np
import pytest
import torch
from scipy.linalg import cho_factor, cho_solve
from scipy.special import gammaln

from dkg_amd.bo_smoke import reference_model_config
from dkg_amd.fit import _Output, fit_map, neg_mll


def _data(n=120, seed=0, ls=(0.15, 0.5), os=2.0, mean=0.3, noise=1e-4):
    g = torch.Generator().manual_seed(seed)
    X = torch.quasirandom.SobolEngine(2, scramble=True, seed=seed).draw(n, dtype=torch.double)
    Z = X / torch.tensor(ls, dtype=torch.double)
    r = torch.cdist(Z, Z)
    t = math.sqrt(5) * r
    K = os * (1 + t + t * t / 3) * torch.exp(-t) + noise * torch.eye(n, dtype=torch.double)
    y = mean + torch.linalg.cholesky(K) @ torch.randn(n, generator=g, dtype=torch.double)
    return X, y


def _numpy_mll(X, y, cfg, mean, ls, os, noise):
    """(log N(y | mean, os kappa + noise I) + log priors) / n, Matern 5/2 ARD, Gamma priors."""
    X, y = X.numpy(), y.numpy()
    n = len(y)
    Z = X / np.asarray(ls)
    d2 = ((Z[:, None, :] - Z[None, :, :]) ** 2).sum(-1)
    t = np.sqrt(5.0 * np.maximum(d2, 1e-30))
    K = os * (1 + t + t * t / 3) * np.exp(-t) + noise * np.eye(n)
    c, low = cho_factor(K, lower=True)
    r = y - mean
    logp = -0.5 * r @ cho_solve((c, low), r) - np.log(np.diag(c)).sum() - 0.5 * n * np.log(2 * np.pi)

    def gam(x, p):
        a, b = p["args"]["concentration"], p["args"]["rate"]
        x = np.atleast_1d(x)
        return float((a * np.log(b) - gammaln(a) + (a - 1) * np.log(x) - b * x).sum())

    k = cfg["kernel"]
    lp = gam(ls, k["lengthscale_prior"]) + gam(os, k["outputscale_prior"]) + gam(noise, cfg["likelihood"]["noise_prior"])
    return (logp + lp) / n


def test_objective_matches_numpy_restatement():
    cfg = reference_model_config(2, [[0, 0], [1, 1]], "once")
    X, y = _data()
    hyper = {"means": [0.25, -0.1], "length_scales": [[0.2, 0.4], [0.7, 0.3]], "output_scales": [1.5, 3.0],
             "noises": [1e-4, 1e-4]}
    got = -neg_mll([X, X], [y, -y], cfg, hyper)
    ref = sum(_numpy_mll(X, yy, cfg["outputs"][i], hyper["means"][i], hyper["length_scales"][i],
                         hyper["output_scales"][i], 1e-4) for i, yy in enumerate([y, -y]))
    assert got == pytest.approx(ref, rel=1e-10, abs=1e-10)


def test_gradient_matches_central_differences():
    cfg = reference_model_config(1, [[0, 0], [1, 1]], "once")["outputs"][0]
    X, y = _data(n=40)
    out = _Output(X, y, cfg, 1e-2, None)
    raw = torch.tensor([0.1, -1.0, 0.3, 0.5], dtype=torch.double, requires_grad=True)
    (g,) = torch.autograd.grad(out.mll(raw), raw)
    h = 1e-6
    for k in range(raw.numel()):
        e = torch.zeros(4, dtype=torch.double)
        e[k] = h
        fd = (float(out.mll(raw.detach() + e)) - float(out.mll(raw.detach() - e))) / (2 * h)
        assert float(g[k]) == pytest.approx(fd, rel=1e-5, abs=1e-7)


def test_fit_beats_the_generating_hyperparameters():
    """The MAP fit's objective is at least the objective at the hyperparameters the data were drawn from,
    and it recovers their ordering (the shorter lengthscale on the first input)."""
    cfg = reference_model_config(1, [[0, 0], [1, 1]], "once")
    X, y = _data(n=150, seed=3)
    res = fit_map([X], [y], cfg)
    assert res["success"]
    truth = {"means": [0.3], "length_scales": [[0.15, 0.5]], "output_scales": [2.0], "noises": [1e-4]}
    assert res["mll"] >= -neg_mll([X], [y], cfg, truth) - 1e-9
    ls = res["length_scales"][0]
    assert ls[0] < ls[1]
    assert res["noises"] == [1e-4]  # fix_zero_noise: pinned at MIN_NOISE_SE**2, not fitted
    # the optimum is stationary: no coordinate move improves the objective
    fitted = {k: res[k] for k in ("means", "length_scales", "output_scales", "noises")}
    base = -neg_mll([X], [y], cfg, fitted)
    assert base == pytest.approx(res["mll"], rel=1e-9)
    for scale in (0.97, 1.03):
        moved = dict(fitted, output_scales=[fitted["output_scales"][0] * scale])
        assert -neg_mll([X], [y], cfg, moved) <= base + 1e-9


def test_fixed_means_are_kept():
    """The `always` path after its first fit: the constants stay at the first fit's (bo_loop.py:600-614)."""
    cfg = reference_model_config(2, [[0, 0], [1, 1]], "always")
    X, y = _data(n=60, seed=1)
    res = fit_map([X, X], [y, 2 * y], cfg, fixed_means=[0.123, -4.0])
    assert res["means"] == [0.123, -4.0]
    free = fit_map([X, X], [y, 2 * y], cfg)
    assert free["mll"] >= res["mll"] - 1e-9


def test_unexpected_fit_mode_raises():
    from dkg_amd.bo_smoke import run_mobo

    with pytest.raises(ValueError, match="fit_hyperparams"):
        run_mobo(None, {}, separate=True, fit_hyperparams="sometimes")
