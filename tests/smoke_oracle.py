"""Test infrastructure: the SMOKE_TEST BO loop (dkg_amd.bo_smoke.run_mobo) on the CPU oracle.

The same loop the device runs (reference ``pipeline/main.py:171-216`` -> ``bo_loop.py:353-421``, the
``discrete_kg`` SMOKE presets of ``:122-131``), with two substitutions, both from ``oracle/``:
the acquisition is the oracle's structure-faithful discrete KG (``oracle.discretekg.discrete_kg_forward``,
differentiable by autograd, so the restated L-BFGS-B gets its gradient from the oracle), and the problem's
objective is the oracle GP's posterior mean (``gp_testproblem.py:76-98``).  Everything else -- initial
data, scalarisation draws, raw samples, Boltzmann starts, L-BFGS-B, the objective choice -- is the
product's own code, so a device run and this run differ only by the KG and posterior arithmetic.
"""

from __future__ import annotations

import torch

from dkg_amd.bo_smoke import GPProblem, run_mobo
from dkg_amd.discretekg import _as_model_state
from dkg_amd.optim import DiscreteKgOptimisationSpec
from helpers import to_oracle
from oracle.discretekg import discrete_kg_forward

# the reference's fixed hyperparameters of gp-sample:lengthscales (main.py:84-88)
HYPER = dict(length_scales=[0.2, 1.8], output_scales=[1, 50], means=[0, 0])


class OracleProblem(GPProblem):
    """The gp-sample objective (posterior mean of the problem GP) by the oracle."""

    def __init__(self, gp, bounds=None):
        super().__init__(gp, bounds=bounds, device=None)
        self.om = to_oracle(gp)

    def __call__(self, X):
        X = torch.as_tensor(X, dtype=torch.double).reshape(-1, self.gp.input_dim)
        out = torch.stack([p[0] for p in self.om.posterior_list(X, observation_noise=False)], dim=-1)
        self.evaluations += X.shape[0]
        return out.detach()


def oracle_acq_factory(model, x_discretisation, scalarisation_weights, target_output_ix):
    om = to_oracle(_as_model_state(model))

    def acq(X):
        return discrete_kg_forward(om, X, x_discretisation, scalarisation_weights, target_output_ix)

    return acq


def smoke_spec(acq_factory=None, device=None) -> DiscreteKgOptimisationSpec:
    """The discrete_kg spec under SMOKE_TEST (bo_loop.py:122-131): 3 points per axis, 2 restarts, 4 raw
    samples, batch_limit 1, maxiter 200; raw-sample seeds from the global RNG (as run_mobo's default)."""
    return DiscreteKgOptimisationSpec(n_discretisation_points_per_axis=3, num_restarts=2, raw_samples=4,
                                      batch_limit=1, max_iter=200, device=device, acq_factory=acq_factory)


def run_oracle_smoke(state, seed: int = 0):
    """run_smoke's two runs (separate, then full evaluations) with the oracle KG and objective."""
    problem = OracleProblem(state)
    return {"separate": run_mobo(problem, HYPER, separate=True, seed=seed,
                                 spec=smoke_spec(oracle_acq_factory)),
            "full": run_mobo(OracleProblem(state), HYPER, separate=False, seed=seed,
                             spec=smoke_spec(oracle_acq_factory))}


def trajectory(res) -> dict:
    """The decisions of a run: per mode and step the chosen x, objective index (None: full) and value."""
    return {mode: {"x": h["x"], "obj_index": h["obj_index"], "acq": h["acq"], "obj": h["obj"]}
            for mode, h in res.items()}
