"""Small host helpers restating reference utilities used around the hot path.

* ``make_torch_std_grid``: ``src/decoupledbo/modules/utils.py:79-107`` (the
  grid discretisation DiscreteKgOptimisationSpec builds,
  ``acquisition_optimisation_strategy.py:209-216``).
* ``is_power_of_2``: ``src/decoupledbo/modules/utils.py:110-114``.
* ``sample_simplex``: BoTorch ``botorch.utils.sampling.sample_simplex`` as
  called by ``pipeline/nodes/bo_loop.py:84-118`` (qMC scalarisation weights).
"""

from __future__ import annotations

import torch


def make_torch_std_grid(n_points_per_axis: int, n_dimensions: int, tkwargs=None) -> torch.Tensor:
    """``n^d x d`` grid on [0,1]^d, last coordinate varying fastest."""
    tkwargs = tkwargs or {}
    if n_dimensions <= 0:
        raise ValueError(f"Expected n_dimensions >= 1. Got {n_dimensions}.")
    axis = torch.linspace(0, 1, n_points_per_axis, **tkwargs)
    mesh = torch.meshgrid(*([axis] * n_dimensions), indexing="ij")
    return torch.stack([g.reshape(-1) for g in mesh], dim=-1)


def is_power_of_2(n) -> bool:
    if not isinstance(n, int):
        raise TypeError(f"Expected n to be an int. Got {type(n)}.")
    return n != 0 and (n & (n - 1)) == 0


def sobol_draw(dim: int, n: int, seed=None, dtype=torch.double) -> torch.Tensor:
    """``n`` scrambled Sobol points in [0, 1)^dim of ``dtype``.  torch's ``SobolEngine`` computes its first
    point in the *default* dtype when it is constructed, so under a float32 default the first point would be
    rounded to float32 whatever ``draw``'s dtype; the reference runs with a float64 default
    (``pipeline/main.py:223``), so the engine is built under ``dtype`` here."""
    prev = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        eng = torch.quasirandom.SobolEngine(dim, scramble=True, seed=seed)
        return eng.draw(n, dtype=dtype)
    finally:
        torch.set_default_dtype(prev)


def sample_simplex(d: int, n: int = 1, qmc: bool = False, seed=None, device=None,
                   dtype=torch.double) -> torch.Tensor:
    """Uniform samples on the (d-1)-simplex via sorted uniforms (BoTorch)."""
    if d == 1:
        return torch.ones(n, 1, device=device, dtype=dtype)
    if qmc:
        u = sobol_draw(d - 1, n, seed, dtype)
    else:
        g = torch.Generator()
        if seed is not None:
            g.manual_seed(seed)
        else:
            g.seed()
        u = torch.rand(n, d - 1, dtype=dtype, generator=g)
    u, _ = torch.sort(u, dim=-1)
    z = torch.zeros(n, 1, dtype=dtype)
    o = torch.ones(n, 1, dtype=dtype)
    u = torch.cat([z, u, o], dim=-1)
    return (u[..., 1:] - u[..., :-1]).to(device=device)
