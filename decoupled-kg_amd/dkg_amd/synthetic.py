"""Seeded synthetic Discrete-KG workloads (BASELINE.json ``configs``).

Hyperparameters follow the reference's ``lengthscales`` GP test-problem
family (``pipeline/main.py:84-88``: lengthscales (0.2, 1.8), outputscales
(1, 50), means 0) with the fitted-noise floor ``MIN_NOISE_SE**2 = 1e-4``
(``model/factory.py:15``).  Training targets are a draw from the GP prior of
each output; the discretisation is the reference's std grid
(``modules/utils.py:79-107``); scalarisation weights are the qMC simplex
sample of ``pipeline/nodes/bo_loop.py:84-118``.  Data only — this module is
not on the hot path.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .model import ModelListGPState, SingleTaskGPState
from .utils import make_torch_std_grid, sample_simplex


@dataclass(frozen=True)
class Workload:
    name: str
    m: int
    n_train: int
    grid: int          # discretisation = grid**d std-grid points
    S: int
    B: int
    d: int = 2
    lengthscales: tuple = (0.2, 1.8)
    outputscales: tuple = (1.0, 50.0)
    noise: float = 1e-4
    noise_rel: float = 0.0  # > 0: noise of output i = noise_rel * outputscale_i (overrides `noise`)

    @property
    def n_disc(self) -> int:
        return self.grid ** self.d


WORKLOADS = {
    # BASELINE.json configs[1]
    "small": Workload("small", m=2, n_train=64, grid=16, S=8, B=32),
    # BASELINE.json configs[2] — the headline
    "headline": Workload("headline", m=2, n_train=256, grid=32, S=16, B=128),
    # well-conditioned, non-degenerate parity variant
    "parity6d": Workload("parity6d", m=2, n_train=128, grid=3, S=8, B=32, d=6,
                         lengthscales=(0.4, 0.7), outputscales=(1.0, 3.0), noise=1e-2),
    # headline size (n_train 256, N = 1024, S = 16, B = 128) on a GP where the KG of every pair is > 0
    # (d = 6, Sobol discretisation): the envelope does real work; bench.py's non-degenerate leg
    "headline_nd": Workload("headline_nd", m=2, n_train=256, grid=0, S=16, B=128, d=6,
                            lengthscales=(0.25, 0.4), outputscales=(1.0, 1.0), noise=1e-2),
    # BASELINE.json configs[4] (the stress config; computed in fp64 here)
    "stress": Workload("stress", m=3, n_train=1024, grid=64, S=32, B=256,
                       lengthscales=(0.2, 1.8, 0.6), outputscales=(1.0, 50.0, 5.0), noise=1e-3),
    # BASELINE.json configs[4] as specified for fp32 (noise >= 1e-3 of the outputscale), the
    # workload of the DKG_PLAN_F32 path
    "stress32": Workload("stress32", m=3, n_train=1024, grid=64, S=32, B=256,
                         lengthscales=(0.2, 1.8, 0.6), outputscales=(1.0, 50.0, 5.0), noise_rel=1e-3),
}


def _matern52(x1, x2, ls, s):
    r = torch.cdist(x1 / ls, x2 / ls)
    return s * (1 + math.sqrt(5) * r + 5.0 / 3.0 * r * r) * torch.exp(-math.sqrt(5) * r)


def make_problem(w: Workload, seed: int = 0):
    """Return (model_state, discretisation[N,d], candidates[B,d], weights[S,m])."""
    dt = torch.double
    X = torch.quasirandom.SobolEngine(w.d, scramble=True, seed=1 + seed).draw(w.n_train, dtype=dt)
    g = torch.Generator().manual_seed(1000 + seed)
    outs = []
    for i in range(w.m):
        ls = w.lengthscales[i % len(w.lengthscales)]
        s = w.outputscales[i % len(w.outputscales)]
        noise = w.noise_rel * s if w.noise_rel > 0 else w.noise
        K = _matern52(X, X, ls, s) + noise * torch.eye(w.n_train, dtype=dt)
        y = torch.linalg.cholesky(K) @ torch.randn(w.n_train, generator=g, dtype=dt)
        outs.append(SingleTaskGPState(X, y, ls, s, noise, 0.0))
    model = ModelListGPState(*outs)
    if w.d <= 3:
        D = make_torch_std_grid(w.grid, w.d, {"dtype": dt})
    else:
        D = torch.quasirandom.SobolEngine(w.d, scramble=True, seed=7 + seed).draw(1024, dtype=dt)
    Xc = torch.quasirandom.SobolEngine(w.d, scramble=True, seed=4 + seed).draw(w.B, dtype=dt)
    W = sample_simplex(w.m, w.S, qmc=True, seed=11 + seed, dtype=dt)
    return model, D, Xc, W
