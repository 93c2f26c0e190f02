"""Multi-objective BO loop over the device KG: the reference's ``SMOKE_TEST`` pipeline path
without BoTorch (BASELINE.json configs[0]).

What it restates (reference files, read for behaviour only):

* ``pipeline/main.py:171-216`` ``run_pipeline``: 6 initial Sobol points, then ``run_mobo`` twice,
  once with separate (decoupled) objective evaluations and costs ``[1, 10]``, once with full
  evaluations; ``max_n_batch = 2`` under ``SMOKE_TEST``;
* ``pipeline/nodes/bo_loop.py:48-59`` ``generate_initial_data`` (Sobol in the bounds, every
  objective evaluated at every point);
* ``:122-131`` the ``discrete_kg`` spec under ``SMOKE_TEST``: 3 grid points per axis, 2 restarts,
  4 raw samples, ``batch_limit = 1``, ``max_iter = 200``;
* ``run_mobo``'s query step (``:380-450``): decoupled, the spec's ``optimize_for_single_objective``
  picks (x, objective) by KG per cost and only that objective is evaluated and appended to its own
  training set; full, ``optimize_for_full_evaluation`` picks x and every objective is evaluated;
* ``modules/gp_testproblem.py:76-98``: the objective of a ``gp-sample`` problem is the posterior
  mean of the problem GP, evaluated here on the device (``dkg_prepare_output`` + ``dkg_cross_root``);
* the model paths of ``bo_loop.py:574-619``: ``never`` (the problem's fixed hyperparameters, noise at the
  1e-8 floor), ``once`` (MAP hyperparameters fitted once on 1000 Sobol points of the problem,
  ``fit_hyperparameters``, ``:63-79``) and ``always`` (refitted on the observations at every iteration, the
  constant means kept at the first fit's); the fit is ``dkg_amd.fit.fit_map`` (parity unpinned: GPyTorch /
  BoTorch are absent here), the fitted paths' noise ``MIN_NOISE_SE**2`` (``fix_zero_noise``).

Scalarisation weights are drawn per step with the reference's qMC simplex sampler
(``bo_loop.py:84-118``, ``dkg_amd.utils.sample_simplex``).

With a ``DataCatalog`` (``dkg_amd.catalog``, the reference's ``pipeline/data_catalog.py`` formats) the
loop writes what the reference's writes: ``initial_data.pt`` (``bo_loop.py:48-59``), a checkpoint per
iteration with the surrogate's ``ModelListGP`` state dict (``:281-290, 467-476``), the query history as
``bo_runs/bo_run_<run_key>.pqt`` in the reference's columns (``:231-255, 388-420``) and the compressed
checkpoints (``:558-561``); run keys ``eval_separate`` / ``eval_full`` (``main.py:42-43``).
"""

from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch import Tensor

from .catalog import DataCatalog
from .gp_state import DeviceGPState
from .model import ModelListGPState, SingleTaskGPState, to_state_dict
from .optim import DiscreteKgOptimisationSpec, draw_sobol_samples
from .utils import sample_simplex

NEVER_FIT_NOISE = 1e-8  # bo_loop.py:583-588
EVAL_SEPARATE = "eval_separate"  # main.py:42-43
EVAL_FULL = "eval_full"


def _output_config(lengthscale_rate: float) -> dict:
    return {"likelihood": {"type": "gaussian", "noise_prior": {"type": "gamma", "args": {"concentration": 1.1,
                                                                                        "rate": 0.05}}},
            "fix_zero_noise": True,
            "kernel": {"type": "matern", "ard": True, "args": {"nu": 2.5},
                       "lengthscale_prior": {"type": "gamma", "args": {"concentration": 3, "rate": lengthscale_rate}},
                       "outputscale_prior": {"type": "gamma", "args": {"concentration": 2, "rate": 0.15}}},
            "standardize_output": False}


def reference_model_config(m: int, bounds, fit_hyperparams: str = "never") -> dict:
    """The ``model_config`` the reference's SMOKE run checkpoints (``bo_loop.py:281-290``): the ``model``
    section of ``config/experiment-lengthscales.yaml`` (the ``gp-sample:lengthscales`` problem), completed
    as ``pipeline/cli.py:22-37`` does for ``--fit-hyperparams never`` (``fit_hyperparams``, and
    ``standardize_output = False`` per output), with the problem's bounds.  ``build_mll_and_model``
    (``factory.py:24-60``) reads ``bounds``, ``fit_hyperparams`` and ``outputs[i]`` from it.  Outputs past
    the config's two repeat its second output's section.  Pinned by tests/golden/ref_schema.json."""
    bnd = torch.as_tensor(bounds, dtype=torch.double).reshape(2, -1)
    return {"bounds": bnd.tolist(), "outputs": [_output_config(10 if i == 0 else 1.1) for i in range(m)],
            "fit_hyperparams": fit_hyperparams}
QUERY_COLUMNS = ("iteration", "x", "obj_index", "obj", "obj_true", "cost", "acq_per_cost", "init", "scalarisation")


class GPProblem:
    """A ``gp-sample`` test problem: objective i at x is the posterior mean of output i of a fixed GP
    (``gp_testproblem.py:76-98``), computed by the library's kernels on ``device``."""

    def __init__(self, gp: ModelListGPState, bounds: Optional[Tensor] = None, device=None):
        self.gp = gp
        d = gp.input_dim
        self.bounds = (torch.stack([torch.zeros(d, dtype=torch.double), torch.ones(d, dtype=torch.double)]) if bounds is None
                       else torch.as_tensor(bounds, dtype=torch.double).reshape(2, d))
        self.device = device
        self.num_objectives = gp.num_outputs
        self.evaluations = 0

    def __call__(self, X: Tensor) -> Tensor:
        """[n, d] -> [n, m] objective values (model-space posterior means, then any Standardize)."""
        X = torch.as_tensor(X, dtype=torch.double).reshape(-1, self.gp.input_dim)
        st = DeviceGPState(self.gp, X, self.device)
        n = X.shape[0]
        out = torch.stack([c.disc_mean[:n] * c.state.y_std + c.state.y_mean for c in st.outputs], dim=-1)
        self.evaluations += n
        return out.cpu()


def surrogate(train_x: Sequence[Tensor], train_y: Sequence[Tensor], hyper: Dict[str, Sequence[float]],
              noise: float = NEVER_FIT_NOISE) -> ModelListGPState:
    """The BO model on the observations so far, one output per objective with its own data
    (decoupled evaluations give every objective its own training set), fixed hyperparameters; the noise is
    ``hyper["noises"][i]`` when the hyperparameters were fitted, else ``noise``."""
    noises = hyper.get("noises") or [noise] * len(train_x)
    outs = [SingleTaskGPState(train_x[i], train_y[i], torch.tensor(hyper["length_scales"][i], dtype=torch.double),
                              float(hyper["output_scales"][i]), float(noises[i]), float(hyper["means"][i]))
            for i in range(len(train_x))]
    return ModelListGPState(*outs)


def fit_hyperparameters(problem: "GPProblem", model_config: dict, n: int = 1000) -> Dict[str, list]:
    """``bo_loop.fit_hyperparameters`` (``:63-79``): n Sobol points of the problem (global RNG, as
    ``draw_sobol_samples`` without a seed), every objective evaluated there, the MAP fit of the surrogate
    (``dkg_amd.fit.fit_map``)."""
    from .fit import fit_map

    x = draw_sobol_samples(problem.bounds, n, 1).squeeze(-2)
    y = problem(x)
    return fit_map([x] * problem.num_objectives, [y[:, i] for i in range(problem.num_objectives)], model_config)


def run_mobo(problem: GPProblem, hyper: Dict[str, Sequence[float]], separate: bool, n_iter: int = 2,
             n_init: int = 6, costs: Sequence[float] = (1, 10), n_scalarisations: int = 16,
             spec: Optional[DiscreteKgOptimisationSpec] = None, seed: int = 0,
             catalog: Optional[DataCatalog] = None, run_key: Optional[str] = None,
             fit_hyperparams: str = "never") -> Dict[str, List]:
    """``bo_loop.run_mobo`` with the discrete-KG strategy for ``n_iter`` BO steps; returns the
    query history (x, objective index or None for full evaluation, observed values, acquisition).
    With ``catalog`` it also writes the reference's checkpoints and query-history table under
    ``run_key`` (default ``eval_separate`` / ``eval_full``).  ``fit_hyperparams`` (``bo_loop.py:574-619``):
    ``never`` and ``once`` use ``hyper`` as given (``once``: the fitted values with their ``noises``);
    ``always`` refits on the observations before every model use, the constant means fixed at the first
    fit's (``:600-614``)."""
    if fit_hyperparams not in ("never", "once", "always"):
        raise ValueError(f"Unexpected value for fit_hyperparams. Got {fit_hyperparams!r}")
    m, d = problem.num_objectives, problem.gp.input_dim
    # the pipeline's --seed (main.py:235, utils.set_random_seed): every later draw comes from the global RNG, as
    # in the reference -- the initial Sobol points (generate_initial_data, bo_loop.py:48-49: no seed), each
    # optimize_acqf's raw-sample Sobol seed (options without "seed", acquisition_optimisation_strategy.py:217-224)
    # and initialize_q_batch's Boltzmann draw.  (A fixed raw-sample seed equal to the initial data's would make
    # the raw samples the training points, where the KG is 0.)
    torch.manual_seed(seed)
    spec = spec or DiscreteKgOptimisationSpec(n_discretisation_points_per_axis=3, num_restarts=2, raw_samples=4,
                                              batch_limit=1, max_iter=200, device=problem.device)
    x0 = draw_sobol_samples(problem.bounds, n_init, 1).squeeze(-2)
    y0 = problem(x0)
    train_x = [x0.clone() for _ in range(m)]
    train_y = [y0[:, i].clone() for i in range(m)]
    hist: Dict[str, List] = {"x": [], "obj_index": [], "obj": [], "acq": [], "cost": []}
    run_key = run_key or (EVAL_SEPARATE if separate else EVAL_FULL)
    qh: Dict[str, List] = {k: [] for k in QUERY_COLUMNS}

    def record(iteration, x, i, y, cost, acq_per_cost, init, w):
        # one row per observed objective value (bo_loop.py:244-255, 388-420); the problem is noise-free
        for k, v in zip(QUERY_COLUMNS, (iteration, np.asarray(x, dtype=np.float64), i, float(y), float(y),
                                        float(cost), acq_per_cost, init, w)):
            qh[k].append(v)

    model_config = reference_model_config(m, problem.bounds, fit_hyperparams)
    fitted_means = None

    def model_now(first: bool = False):
        # the surrogate for the next step: refitted on the data so far on the `always` path
        nonlocal hyper, fitted_means
        if fit_hyperparams == "always":
            from .fit import fit_map

            hyper = fit_map(train_x, train_y, model_config, fixed_means=None if first else fitted_means)
            if first:
                fitted_means = list(hyper["means"])
        return surrogate(train_x, train_y, hyper)

    def checkpoint(iteration, model):
        if catalog is not None:
            catalog.save_checkpoint(run_key, iteration, to_state_dict(model, model_config), model_config,
                                    [t.clone() for t in train_x], [t.clone() for t in train_y],
                                    [t.clone() for t in train_y], problem.bounds.clone())

    for i in range(m):
        for j in range(n_init):
            record(0, x0[j].numpy(), i, y0[j, i], costs[i], float("nan"), True, None)
    model = model_now(first=True)
    checkpoint(0, model)
    for it in range(n_iter):
        W = sample_simplex(m, n_scalarisations, qmc=True, seed=seed + 1 + it, dtype=torch.double)
        w_row = W[0].numpy().copy() if W.shape[0] == 1 else None
        if separate:
            x, i, acq = spec.optimize_for_single_objective(model, costs, d, scalarisation_weights=W)
            x = x.reshape(1, d).cpu()
            y = problem(x)[0]
            train_x[i] = torch.cat([train_x[i], x])
            train_y[i] = torch.cat([train_y[i], y[i:i + 1]])
            hist["obj_index"].append(int(i))
            hist["obj"].append(float(y[i]))
            hist["cost"].append(float(costs[i]))
            record(it + 1, x[0].numpy(), int(i), y[i], costs[i], float(acq), False, w_row)
        else:
            x, acq = spec.optimize_for_full_evaluation(model, d, scalarisation_weights=W)
            x = x.reshape(1, d).cpu()
            y = problem(x)[0]
            for i in range(m):
                train_x[i] = torch.cat([train_x[i], x])
                train_y[i] = torch.cat([train_y[i], y[i:i + 1]])
            hist["obj_index"].append(None)
            hist["obj"].append(y.tolist())
            hist["cost"].append(float(sum(costs)))
            for i in range(m):
                record(it + 1, x[0].numpy(), i, y[i], costs[i], float(acq) / float(sum(costs)), False, w_row)
        hist["x"].append(x[0].tolist())
        hist["acq"].append(float(acq))
        model = model_now()
        checkpoint(it + 1, model)
    hist["n_observations"] = [int(t.shape[0]) for t in train_x]
    hist["query_history"] = qh
    if catalog is not None:
        import pandas as pd

        catalog.save_bo_run(run_key, pd.DataFrame(qh))
        catalog.compress_checkpoints(run_key)
    return hist


def run_smoke(problem: GPProblem, hyper: Dict[str, Sequence[float]], seed: int = 0,
              catalog: Optional[DataCatalog] = None, fit_hyperparams: str = "never") -> Dict[str, Dict]:
    """``run_pipeline`` under ``SMOKE_TEST`` (``main.py:171-216``): the separate-evaluation run and
    the full-evaluation run, two BO steps each; with ``catalog`` both write the reference's files.
    ``fit_hyperparams = "once"`` fits the hyperparameters first (``main.py:181-182``, saved to the catalog's
    ``hyperparameters.pt`` as the fitted surrogate's state dict) and both runs use them; ``"always"`` refits
    inside the runs."""
    if fit_hyperparams == "once":
        torch.manual_seed(seed)
        cfg = reference_model_config(problem.num_objectives, problem.bounds, "once")
        hyper = fit_hyperparameters(problem, cfg)
        if catalog is not None:
            x = torch.zeros(1, problem.gp.input_dim, dtype=torch.double)
            y = torch.zeros(1, dtype=torch.double)
            catalog.save_model_hyperparameters(
                to_state_dict(surrogate([x] * problem.num_objectives, [y] * problem.num_objectives, hyper), cfg))
    return {"separate": run_mobo(problem, hyper, separate=True, seed=seed, catalog=catalog,
                                 fit_hyperparams=fit_hyperparams),
            "full": run_mobo(problem, hyper, separate=False, seed=seed, catalog=catalog,
                             fit_hyperparams=fit_hyperparams)}
