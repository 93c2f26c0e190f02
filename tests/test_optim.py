"""The optimize_acqf restatement (dkg_amd.optim) on the CPU.

BoTorch (botorch@c14808f) is not installed, so these check the restated
algorithm's contract: Boltzmann initial conditions that keep the best raw
point, L-BFGS-B inside the bounds, chunking by batch_limit, and the
reference's objective choice (acquisition_optimisation_strategy.py:143-163).
The acquisition functions here are an analytic bowl and the oracle's
discrete KG (test infrastructure); the device KG runs in test_gpu_optim.py.
"""

import pytest
import torch

from dkg_amd.optim import (DiscreteKgOptimisationSpec, draw_sobol_samples, gen_batch_initial_conditions,
                           initialize_q_batch, optimize_acqf)


def bowl(center):
    c = torch.as_tensor(center, dtype=torch.double)

    def f(X):  # [*batch, 1, d] -> [*batch]
        return -((X.squeeze(-2) - c) ** 2).sum(-1)

    return f


def test_draw_sobol_samples_in_bounds_and_seeded():
    b = torch.tensor([[0.2, -1.0], [0.4, 3.0]], dtype=torch.double)
    X = draw_sobol_samples(b, 64, 1, seed=3)
    assert X.shape == (64, 1, 2)
    assert bool((X >= b[0]).all() and (X <= b[1]).all())
    assert torch.equal(X, draw_sobol_samples(b, 64, 1, seed=3))


def test_initialize_q_batch_keeps_best_and_shapes():
    X = torch.rand(50, 1, 3)
    Y = torch.randn(50)
    for _ in range(20):
        out = initialize_q_batch(X, Y, 5)
        assert out.shape == (5, 1, 3)
        assert any(torch.equal(r, X[int(torch.argmax(Y))]) for r in out)
    assert torch.equal(initialize_q_batch(X, Y, 50), X)
    with pytest.raises(RuntimeError):
        initialize_q_batch(X, Y, 51)
    with pytest.warns(RuntimeWarning):
        assert initialize_q_batch(X, torch.zeros(50), 4).shape == (4, 1, 3)


@pytest.mark.parametrize("batch_limit", [1, 3, 10])
def test_optimize_acqf_finds_bowl_minimum(batch_limit):
    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double)
    x, v = optimize_acqf(bowl([0.3, 0.7]), bounds, q=1, num_restarts=6, raw_samples=32,
                         options={"batch_limit": batch_limit, "maxiter": 100, "seed": 0})
    assert x.shape == (1, 2)
    torch.testing.assert_close(x, torch.tensor([[0.3, 0.7]], dtype=torch.double), atol=1e-5, rtol=0)
    assert float(v) == pytest.approx(0.0, abs=1e-9)


def test_optimize_acqf_respects_bounds():
    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double)
    X, V = optimize_acqf(bowl([1.5, -0.2]), bounds, q=1, num_restarts=4, raw_samples=16,
                         options={"maxiter": 100, "seed": 1}, return_best_only=False)
    assert X.shape == (4, 1, 2) and V.shape == (4,)
    assert bool((X >= 0).all() and (X <= 1).all())
    torch.testing.assert_close(X[int(V.argmax())], torch.tensor([[1.0, 0.0]], dtype=torch.double), atol=1e-6,
                               rtol=0)


def test_optimize_acqf_on_oracle_kg_beats_raw_samples():
    """The restated optimiser on the oracle's discrete KG (small problem): the optimum is at
    least as good as every raw sample (the starts include the best one)."""
    from oracle.discretekg import discrete_kg_forward
    from oracle.gp import ModelList, OutputGP

    g = torch.Generator().manual_seed(2)
    Xtr = torch.rand(12, 2, generator=g, dtype=torch.double)
    om = ModelList([OutputGP(Xtr, torch.sin(6 * Xtr[:, 0]) + Xtr[:, 1], 0.3, 1.0, 1e-3),
                    OutputGP(Xtr, torch.cos(5 * Xtr[:, 1]), 0.4, 1.0, 1e-3)])
    D = torch.rand(25, 2, generator=g, dtype=torch.double)
    W = torch.tensor([[0.3, 0.7], [0.8, 0.2]], dtype=torch.double)

    def acq(X):
        return discrete_kg_forward(om, X, D, W)

    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double)
    opts = {"batch_limit": 2, "maxiter": 30, "seed": 5}
    x, v = optimize_acqf(acq, bounds, q=1, num_restarts=2, raw_samples=16, options=opts)
    X_raw = draw_sobol_samples(bounds, 16, 1, seed=5)
    with torch.no_grad():
        best_raw = acq(X_raw).max()
    assert float(v) >= float(best_raw) - 1e-12
    with torch.no_grad():
        assert float(acq(x.unsqueeze(0))) == pytest.approx(float(v), rel=1e-12)


def test_gen_batch_initial_conditions_uses_acq_values():
    bounds = torch.tensor([[0.0], [1.0]], dtype=torch.double)
    ic = gen_batch_initial_conditions(bowl([0.5]), bounds, 1, 3, 64, {"seed": 0})
    X_raw = draw_sobol_samples(bounds, 64, 1, seed=0)
    best = X_raw[int(torch.argmax(bowl([0.5])(X_raw)))]
    assert ic.shape == (3, 1, 1)
    assert any(torch.equal(r, best) for r in ic)


def test_choose_best_objective_matches_reference_rule():
    pick = DiscreteKgOptimisationSpec._choose_best_objective
    x0, x1, x2 = (torch.full((1, 2), float(i)) for i in range(3))
    cands = [(0, x0, torch.tensor(0.2)), (1, x1, torch.tensor(0.3)), (2, x2, torch.tensor(0.1))]
    i, x, v = pick(cands, [1.0, 3.0, 0.25])
    assert i == 2 and torch.equal(x, x2) and float(v) == pytest.approx(0.4)
    # equal value per cost (0.2 / 1 = 0.1 / 0.5): the cheaper objective wins
    i, x, v = pick(cands, [1.0, 3.0, 0.5])
    assert i == 2 and float(v) == pytest.approx(0.2)
    # negative values clip to 0; ties go to the cheapest objective
    neg = [(0, x0, torch.tensor(-0.5)), (1, x1, torch.tensor(-0.1))]
    i, _, v = pick(neg, [2.0, 1.0])
    assert i == 1 and float(v) == pytest.approx(-0.1)
