"""Acquisition optimisation over the device KG.

``DiscreteKgOptimisationSpec`` (reference ``acquisition_optimisation_strategy.py:166-273``)
hands ``DiscreteKnowledgeGradient`` to BoTorch's ``optimize_acqf`` with q = 1.  BoTorch is
pinned to a git revision (botorch@c14808f, ``requirements.txt:16``) and is neither vendored
nor installed here, so this module restates the parts of its published algorithm that path
uses:

* ``gen_batch_initial_conditions``: ``raw_samples`` scrambled-Sobol points in the bounds,
  their acquisition values (no gradient, in chunks of ``init_batch_limit``), and
  ``initialize_q_batch``'s Boltzmann selection of ``num_restarts`` starts (eta = 1, the best
  raw point always kept);
* ``gen_candidates_scipy``: L-BFGS-B (scipy) on ``-sum(acq(X))`` over one chunk of restarts
  with the analytic gradient and box bounds, candidates clamped to the bounds;
* ``optimize_acqf``: restarts in chunks of ``batch_limit``, the best candidate returned.

On the device a chunk's value + gradient is one C call for all of its restarts
(``dkg_plan_forward_grad``), so ``batch_limit = num_restarts`` evaluates every restart in the
same launch; the reference uses ``batch_limit = 1`` because its forward is a Python loop over
candidates (``pipeline/nodes/bo_loop.py:127-129``).  ``batch_limit`` keeps BoTorch's meaning:
restarts in one chunk share one L-BFGS-B problem (the sum of their values).
"""

from __future__ import annotations

import logging
import warnings
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor

logger = logging.getLogger(__name__)

# option keys consumed by the initial-condition stage, not passed to L-BFGS-B
# (BoTorch optimize_acqf's INIT_OPTION_KEYS subset that applies here)
INIT_OPTION_KEYS = {"batch_limit", "init_batch_limit", "eta", "seed", "nonnegative", "alpha"}


def draw_sobol_samples(bounds: Tensor, n: int, q: int, seed: Optional[int] = None) -> Tensor:
    """``botorch.utils.sampling.draw_sobol_samples``: n x q x d scrambled Sobol points in ``bounds``."""
    lower, upper = bounds[0], bounds[1]
    d = lower.shape[-1]
    if seed is None:
        seed = int(torch.randint(0, 10**6, (1,)).item())
    from .utils import sobol_draw

    raw = sobol_draw(d * q, n, seed, lower.dtype).to(lower.device).view(n, q, d)
    return lower + (upper - lower) * raw


def initialize_q_batch(X: Tensor, Y: Tensor, n: int, eta: float = 1.0) -> Tensor:
    """``botorch.optim.initializers.initialize_q_batch``: Boltzmann sample of n rows of X by
    ``exp(eta * standardised Y)``, always keeping the best raw point."""
    n_samples = X.shape[0]
    if n > n_samples:
        raise RuntimeError(f"n ({n}) cannot be larger than the number of provided samples ({n_samples})")
    if n == n_samples:
        return X
    Ystd = Y.std(dim=0)
    if bool(torch.any(Ystd == 0)):
        warnings.warn("All acquisition values for raw samples points are the same for at least one batch. "
                      "Choosing initial conditions at random.", RuntimeWarning)
        return X[torch.randperm(n=n_samples, device=X.device)][:n]
    max_idx = int(torch.argmax(Y))
    Z = (Y - Y.mean(dim=0)) / Ystd
    etaZ = eta * Z
    weights = torch.exp(etaZ)
    while bool(torch.isinf(weights).any()):
        etaZ = etaZ * 0.5
        weights = torch.exp(etaZ)
    idcs = torch.multinomial(weights, n)
    if max_idx not in idcs:
        idcs[-1] = max_idx
    return X[idcs]


def _no_grad_values(acq: Callable[[Tensor], Tensor], X: Tensor, chunk: int) -> Tensor:
    with torch.no_grad():
        return torch.cat([acq(X[i:i + chunk]).reshape(-1) for i in range(0, X.shape[0], chunk)])


def gen_batch_initial_conditions(acq_function: Callable[[Tensor], Tensor], bounds: Tensor, q: int,
                                 num_restarts: int, raw_samples: int, options: Optional[Dict] = None) -> Tensor:
    """``botorch.optim.initializers.gen_batch_initial_conditions`` (q-batch Sobol raw samples,
    ``initialize_q_batch``): num_restarts x q x d starting points."""
    options = options or {}
    X_rnd = draw_sobol_samples(bounds, raw_samples, q, seed=options.get("seed"))
    chunk = options.get("init_batch_limit", options.get("batch_limit", raw_samples)) or raw_samples
    Y_rnd = _no_grad_values(acq_function, X_rnd, max(1, int(chunk)))
    return initialize_q_batch(X_rnd, Y_rnd.to(X_rnd), n=num_restarts, eta=options.get("eta", 1.0))


def gen_candidates_scipy(initial_conditions: Tensor, acquisition_function: Callable[[Tensor], Tensor],
                         lower_bounds: Tensor, upper_bounds: Tensor,
                         options: Optional[Dict] = None) -> Tuple[Tensor, Tensor]:
    """``botorch.generation.gen.gen_candidates_scipy`` with L-BFGS-B: minimise -sum acq over the
    flattened restarts (box bounds, analytic gradient); returns (candidates, acq values)."""
    from scipy.optimize import minimize

    options = dict(options or {})
    ic = initial_conditions.clamp(lower_bounds, upper_bounds)
    shapeX = ic.shape
    lb = lower_bounds.expand(shapeX).reshape(-1).cpu().numpy()
    ub = upper_bounds.expand(shapeX).reshape(-1).cpu().numpy()
    bounds = list(zip(lb.tolist(), ub.tolist()))

    fast = getattr(acquisition_function, "value_and_grad_host", None)

    def f_np(x: np.ndarray):
        if fast is not None:
            # the device KG: value and gradient in one round trip (DiscreteKnowledgeGradient.value_and_grad_host)
            kg, g = fast(torch.from_numpy(x).view(shapeX))
            loss = -float(kg.sum())
            if not np.isfinite(loss):
                raise RuntimeError("acquisition function returned a non-finite value inside L-BFGS-B")
            return loss, (-g).reshape(-1).numpy()
        X = torch.from_numpy(x).to(ic).view(shapeX).contiguous().requires_grad_(True)
        loss = -acquisition_function(X).sum()
        if not torch.isfinite(loss):
            raise RuntimeError("acquisition function returned a non-finite value inside L-BFGS-B")
        (grad,) = torch.autograd.grad(loss, X)
        return float(loss.item()), grad.reshape(-1).double().cpu().numpy()

    minimize_opts = {k: v for k, v in options.items() if k not in ("method", "callback", "with_grad")}
    res = minimize(f_np, ic.reshape(-1).double().cpu().numpy(), method="L-BFGS-B", jac=True, bounds=bounds,
                   options=minimize_opts)
    candidates = torch.from_numpy(res.x).to(ic).view(shapeX).clamp(lower_bounds, upper_bounds)
    with torch.no_grad():
        batch_acquisition = acquisition_function(candidates)
    return candidates, batch_acquisition


def optimize_acqf(acq_function: Callable[[Tensor], Tensor], bounds: Tensor, q: int, num_restarts: int,
                  raw_samples: Optional[int] = None, options: Optional[Dict] = None,
                  batch_initial_conditions: Optional[Tensor] = None,
                  return_best_only: bool = True) -> Tuple[Tensor, Tensor]:
    """``botorch.optim.optimize_acqf`` for the q = 1 / no-constraint case the reference uses
    (``acquisition_optimisation_strategy.py:217-224, 259-266``)."""
    if q != 1:
        raise NotImplementedError("only q = 1 is supported (DiscreteKnowledgeGradient is q = 1)")
    options = dict(options or {})
    if batch_initial_conditions is None:
        if raw_samples is None:
            raise ValueError("Must specify `raw_samples` when `batch_initial_conditions` is None`.")
        batch_initial_conditions = gen_batch_initial_conditions(acq_function, bounds, q, num_restarts, raw_samples,
                                                                options)
    batch_limit = int(options.get("batch_limit", num_restarts) or num_restarts)
    gen_opts = {k: v for k, v in options.items() if k not in INIT_OPTION_KEYS}
    cands: List[Tensor] = []
    vals: List[Tensor] = []
    for start in range(0, batch_initial_conditions.shape[0], batch_limit):
        c, v = gen_candidates_scipy(batch_initial_conditions[start:start + batch_limit], acq_function,
                                    bounds[0], bounds[1], gen_opts)
        cands.append(c)
        vals.append(v.reshape(-1))
    batch_candidates = torch.cat(cands)
    batch_acq_values = torch.cat(vals)
    if return_best_only:
        best = int(torch.argmax(batch_acq_values))
        return batch_candidates[best], batch_acq_values[best]
    return batch_candidates, batch_acq_values


def _get_standard_bounds(dim: int, dtype=torch.double) -> Tensor:
    """``acquisition_optimisation_strategy.py:555``: the unit cube."""
    return torch.stack([torch.zeros(dim, dtype=dtype), torch.ones(dim, dtype=dtype)])


class DiscreteKgOptimisationSpec:
    """``DiscreteKgOptimisationSpec`` (``acquisition_optimisation_strategy.py:166-273``) on the
    device KG: same constructor, same two entry points, same tie-breaking.

    ``n_discretisation_points_per_axis``: grid points per axis of the discretisation
    (``make_torch_std_grid``); ``num_restarts`` / ``raw_samples`` / ``batch_limit`` /
    ``max_iter``: passed to ``optimize_acqf`` exactly as the reference does (:217-224).
    """

    def __init__(self, n_discretisation_points_per_axis: int, num_restarts: int, raw_samples: int,
                 batch_limit: int, max_iter: int, device=None, seed: Optional[int] = None,
                 acq_factory: Optional[Callable] = None):
        self.n_discretisation_points_per_axis = n_discretisation_points_per_axis
        self.num_restarts = num_restarts
        self.raw_samples = raw_samples
        self.batch_limit = batch_limit
        self.max_iter = max_iter
        self.device = device
        self.seed = seed
        # acq_factory(model, x_discretisation, scalarisation_weights, target_output_ix) -> acquisition:
        # None builds the device DiscreteKnowledgeGradient (tests inject the oracle's KG to compare runs)
        self.acq_factory = acq_factory

    def _options(self) -> Dict:
        opts = {"batch_limit": self.batch_limit, "maxiter": self.max_iter}
        if self.seed is not None:
            opts["seed"] = self.seed
        return opts

    def _acq(self, model, input_dim: int, scalarisation_weights: Tensor, target: Optional[int]):
        from .discretekg import DiscreteKnowledgeGradient
        from .utils import make_torch_std_grid

        disc = make_torch_std_grid(self.n_discretisation_points_per_axis, input_dim, {"dtype": torch.double})
        if self.acq_factory is not None:
            return self.acq_factory(model, disc, scalarisation_weights, target)
        return DiscreteKnowledgeGradient(model, x_discretisation=disc, scalarisation_weights=scalarisation_weights,
                                         target_output_ix=target, device=self.device)

    def optimize_for_single_objective(self, model, costs: Union[Tensor, Sequence], input_dim: int, *,
                                      scalarisation_weights: Tensor, **_unused_kwargs) -> Tuple[Tensor, int, Tensor]:
        """Decoupled KG per objective, best KG per cost (:196-240)."""
        from .discretekg import _as_model_state

        standard_bounds = _get_standard_bounds(input_dim)
        candidates = []
        for i in range(_as_model_state(model).num_outputs):
            acq_func = self._acq(model, input_dim, scalarisation_weights, i)
            candidate_x, acq_value = optimize_acqf(acq_function=acq_func, bounds=standard_bounds, q=1,
                                                   num_restarts=self.num_restarts, raw_samples=self.raw_samples,
                                                   options=self._options())
            if acq_value < 0:
                logger.warning("Optimal acquisition function value is negative: obj_index=%i, acq_value=%f", i,
                               acq_value)
            candidates.append((i, candidate_x.detach(), acq_value.detach()))
        best_i, best_x, best_kg_per_cost = self._choose_best_objective(candidates, costs)
        return best_x, best_i, best_kg_per_cost

    def optimize_for_full_evaluation(self, model, input_dim: int, *, scalarisation_weights: Tensor,
                                     **_unused_kwargs) -> Tuple[Tensor, Tensor]:
        """Coupled (full-evaluation) KG (:242-273)."""
        acq_func = self._acq(model, input_dim, scalarisation_weights, None)
        candidate_x, acq_value = optimize_acqf(acq_function=acq_func, bounds=_get_standard_bounds(input_dim), q=1,
                                               num_restarts=self.num_restarts, raw_samples=self.raw_samples,
                                               options=self._options())
        if acq_value < 0:
            logger.warning("Optimal acquisition function value is negative: acq_value=%f", acq_value)
        return candidate_x.detach(), acq_value.detach()

    @staticmethod
    def _choose_best_objective(candidates, costs):
        """:143-163 — clip negative values to 0, maximise value / cost, ties to the cheaper objective."""
        best_i, best_x, best_acq_value = max(candidates, key=lambda x: (max(x[-1], 0) / costs[x[0]], -costs[x[0]]))
        return best_i, best_x, best_acq_value / costs[best_i]
