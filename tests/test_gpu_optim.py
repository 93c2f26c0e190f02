"""DiscreteKgOptimisationSpec / optimize_acqf on the device KG.

The reference optimises DiscreteKnowledgeGradient with BoTorch's optimize_acqf
(acquisition_optimisation_strategy.py:209-224, 252-266; production settings
bo_loop.py:123-131: 11 grid points per axis, 10 restarts, 32 raw samples,
maxiter 200).  Here the device KG and the oracle KG are optimised from the same
initial conditions; their values and gradients agree to ~1e-10, so L-BFGS-B
follows the same path and the optima agree.
"""

import pytest
import torch

from dkg_amd import DiscreteKnowledgeGradient, make_torch_std_grid
from dkg_amd.optim import DiscreteKgOptimisationSpec, draw_sobol_samples, optimize_acqf
from dkg_amd.synthetic import WORKLOADS, make_problem
from helpers import to_oracle
from oracle.discretekg import discrete_kg_forward

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def small_model():
    model, _, _, W = make_problem(WORKLOADS["small"])
    return model, W[:4]


@pytest.mark.parametrize("target", [None, 0])
def test_device_and_oracle_optimise_to_the_same_candidate(target):
    model, W = small_model()
    D = make_torch_std_grid(7, 2, {"dtype": torch.double})
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    om = to_oracle(model)

    def oracle_acq(X):
        return discrete_kg_forward(om, X, D, W, target)

    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double)
    ic = draw_sobol_samples(bounds, 3, 1, seed=21)
    opts = {"batch_limit": 1, "maxiter": 40}
    Xd, Vd = optimize_acqf(acq, bounds, 1, 3, options=opts, batch_initial_conditions=ic, return_best_only=False)
    Xo, Vo = optimize_acqf(oracle_acq, bounds, 1, 3, options=opts, batch_initial_conditions=ic,
                           return_best_only=False)
    torch.testing.assert_close(Vd, Vo, rtol=1e-5, atol=1e-9 * float(Vo.abs().max()))
    torch.testing.assert_close(Xd, Xo, rtol=0, atol=1e-4)


@pytest.mark.parametrize("batch_limit", [1, 10])
def test_spec_full_evaluation_production_settings(batch_limit):
    model, W = small_model()
    spec = DiscreteKgOptimisationSpec(n_discretisation_points_per_axis=11, num_restarts=10, raw_samples=32,
                                      batch_limit=batch_limit, max_iter=200, device=DEV, seed=7)
    x, v = spec.optimize_for_full_evaluation(model, 2, scalarisation_weights=W)
    assert x.shape == (1, 2) and bool((x >= 0).all() and (x <= 1).all())
    acq = DiscreteKnowledgeGradient(model, make_torch_std_grid(11, 2, {"dtype": torch.double}), W, device=DEV)
    raw = draw_sobol_samples(torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double), 32, 1, seed=7)
    with torch.no_grad():
        assert float(acq(x.unsqueeze(0))) == pytest.approx(float(v), rel=1e-12)
        assert float(v) >= float(acq(raw).max()) * (1 - 1e-12)


def test_spec_single_objective_picks_best_kg_per_cost():
    model, W = small_model()
    spec = DiscreteKgOptimisationSpec(11, 4, 16, 4, 50, device=DEV, seed=3)
    x, i, kg_per_cost = spec.optimize_for_single_objective(model, [1.0, 2.0], 2, scalarisation_weights=W)
    assert i in (0, 1) and x.shape == (1, 2)
    acq = DiscreteKnowledgeGradient(model, make_torch_std_grid(11, 2, {"dtype": torch.double}), W,
                                    target_output_ix=i, device=DEV)
    with torch.no_grad():
        assert float(acq(x.unsqueeze(0))) / [1.0, 2.0][i] == pytest.approx(float(kg_per_cost), rel=1e-12)
