"""dKG/dX through the C ABI (dkg_plan_forward_grad) vs the oracle's autograd.

The reference's forward is differentiable (test_discretekg.py:110-135 runs
gradcheck on it; optimize_acqf's L-BFGS-B needs dKG/dX).  The oracle is the
structure-faithful restatement; torch.autograd through it is the gradient
reference (its own gradcheck passes in test_oracle_kats.py).

Tolerance, stated like the KG's (tests/helpers.grad_tol): per candidate and coordinate
|g - g_ref| <= 1e-6 |g_ref| + 64 eps G, with G = |da_0/dx| + max_k |db_k/dx| the magnitude of the terms
the gradient sums (helpers.grad_scale): the fp64 cancellation floor of that sum, as 64 eps max|a| is
KG's.  Measured worst ratio 0.072 at the headline, 0.0011 on headline_nd (profiles/r03/grad_probe.json).
"""

import pytest
import torch

from dkg_amd import DiscreteKnowledgeGradient
from dkg_amd.synthetic import WORKLOADS, make_problem
from helpers import assert_within, grad_scale, grad_tol, load_golden, stated_tol, to_oracle
from oracle.discretekg import discrete_kg_batched, lines_batched

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def oracle_grad(om, X, D, W, target):
    Xr = X.clone().requires_grad_(True)
    kg, _ = discrete_kg_batched(om, Xr, D, W, target)
    (g,) = torch.autograd.grad(kg.sum(), Xr)
    return kg.detach(), g


def native_grad(state, X, D, W, target):
    acq = DiscreteKnowledgeGradient(state, D, W, target_output_ix=target, device=DEV)
    Xr = X.clone().to(DEV).requires_grad_(True)
    kg = acq(Xr.unsqueeze(-2))
    (g,) = torch.autograd.grad(kg.sum(), Xr)
    return kg.detach().cpu(), g.cpu()


def assert_grad_close(g, ref, G):
    """|g - ref| <= 1e-6 |ref| + 64 eps G per candidate (G from helpers.grad_scale); returns the worst ratio."""
    err = (g - ref).abs()
    tol = grad_tol(ref, G)
    ratio = err / tol
    assert bool((err <= tol).all()), f"max err {err.max():.3e}, worst err/tol {ratio.max():.3f}"
    return float(ratio.max())


@pytest.mark.parametrize("workload", ["small", "parity6d"])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_grad_vs_oracle(workload, target):
    w = WORKLOADS[workload]
    model, D, X, W = make_problem(w)
    X, W = X[:12], W[:8]
    om = to_oracle(model)
    kg_ref, g_ref = oracle_grad(om, X, D, W, target)
    kg, g = native_grad(model, X, D, W, target)
    assert g.shape == X.shape
    assert_grad_close(g, g_ref, grad_scale(om, X, D, W, target))


@pytest.mark.parametrize("name", ["lengthscales0", "observationnoise0"])
@pytest.mark.parametrize("target", [None, 1])
def test_grad_golden_problems(name, target):
    state, om, D, W, X, _ = load_golden(name)
    X = X[:10]
    _, g_ref = oracle_grad(om, X, D, W, target)
    _, g = native_grad(state, X, D, W, target)
    assert_grad_close(g, g_ref, grad_scale(om, X, D, W, target))


def test_grad_matches_central_differences():
    """The analytic device gradient against central differences of the device forward."""
    model, D, X, W = make_problem(WORKLOADS["small"])
    X = X[:6]
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    Xr = X.clone().to(DEV).requires_grad_(True)
    (g,) = torch.autograd.grad(acq(Xr.unsqueeze(-2)).sum(), Xr)
    h = 1e-6
    fd = torch.zeros_like(X)
    for j in range(X.shape[1]):
        e = torch.zeros_like(X)
        e[:, j] = h
        up = acq((X + e).to(DEV).unsqueeze(-2)).cpu()
        dn = acq((X - e).to(DEV).unsqueeze(-2)).cpu()
        fd[:, j] = (up - dn) / (2 * h)
    torch.testing.assert_close(g.cpu(), fd, rtol=1e-4, atol=1e-7 * fd.abs().max().item())


@pytest.mark.parametrize("workload", ["headline", "headline_nd"])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_grad_vs_oracle_headline_all_candidates(workload, target):
    """Headline sizes (n 256, N 1024, S 16), every one of the 128 candidates: the value the gradient plan
    returns (stated tolerance) and dKG/dx against the oracle's autograd.  headline_nd (d = 6) has KG > 0 on
    every pair, so every value and gradient there is a walked envelope's."""
    w = WORKLOADS[workload]
    model, D, X, W = make_problem(w)
    om = to_oracle(model)
    kg_ref, g_ref = oracle_grad(om, X, D, W, target)
    kg, g = native_grad(model, X, D, W, target)
    assert g.shape == X.shape == (128, w.d)
    if workload == "headline_nd":
        assert int((kg_ref > 0).sum()) >= 120  # full: all 128; decoupled paths: 126 (two exact zeros)
    amax = lines_batched(om, X, D, W, target)[0].abs().amax((-1, -2))
    kr = assert_within(kg, kg_ref, stated_tol(kg_ref, amax), "KG of the gradient plan (stated tolerance)")
    gr = assert_grad_close(g, g_ref, grad_scale(om, X, D, W, target))
    print(f"{workload} target={target}: KG worst err/tol {kr:.3g}, gradient worst err/tol {gr:.3g}")


def test_grad_headline_batch_consistent():
    """Headline-size batch: gradient rows equal those of the same candidates evaluated alone."""
    model, D, X, W = make_problem(WORKLOADS["headline"])
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    Xr = X.clone().to(DEV).requires_grad_(True)
    kg = acq(Xr.unsqueeze(-2))
    (g,) = torch.autograd.grad(kg.sum(), Xr)
    kg_plain = acq(X.to(DEV).unsqueeze(-2))
    # same KG with and without the gradient path (edge sums in a different order: rounding only)
    torch.testing.assert_close(kg.detach(), kg_plain, rtol=1e-12, atol=1e-300)
    Xs = X[:5].clone().to(DEV).requires_grad_(True)
    (gs,) = torch.autograd.grad(acq(Xs.unsqueeze(-2)).sum(), Xs)
    assert torch.equal(gs, g[:5])


def test_grad_flows_with_batch_shape_and_weights():
    """[*batch, 1, d] input and a weighted sum of outputs backpropagate exactly."""
    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    Xb = X[:6].reshape(2, 3, 1, 2).clone().to(DEV).requires_grad_(True)
    wts = torch.arange(1.0, 7.0, dtype=torch.double, device=DEV).reshape(2, 3)
    (g,) = torch.autograd.grad((acq(Xb) * wts).sum(), Xb)
    X0 = X[:6].clone().to(DEV).requires_grad_(True)
    (g0,) = torch.autograd.grad(acq(X0.unsqueeze(-2)).sum(), X0)
    torch.testing.assert_close(g.reshape(6, 2), g0 * wts.reshape(6, 1), rtol=0, atol=0)


# test_discretekg.py:110-135 through the device path: gradcheck of the module
# functions at xnew = (0.51, 0.51) on the reference test models.
@pytest.fixture(scope="module")
def ref_models():
    from oracle.fit import make_reference_test_model, reference_test_discretisation

    return {True: make_reference_test_model(use_noise=True), False: make_reference_test_model(use_noise=False),
            "disc": reference_test_discretisation()}


@pytest.mark.parametrize("noisy", [True, False], ids=["noisy", "noiseless"])
@pytest.mark.parametrize("weights", [[[0.6, 0.4]], [[0.7, 0.3], [0.6, 0.4], [0.5, 0.5]]], ids=["single", "trio"])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_reference_gradcheck(ref_models, noisy, weights, target):
    from dkg_amd import calculate_discrete_kg, calculate_discrete_kg_conditioning_on_single_output
    from helpers import to_state

    state = to_state(ref_models[noisy])
    disc = ref_models["disc"]
    W = torch.tensor(weights, dtype=torch.double)
    xnew = torch.tensor([0.51, 0.51], dtype=torch.double, device=DEV, requires_grad=True)
    if target is None:
        fn = lambda x: calculate_discrete_kg(state, x, disc, W)  # noqa: E731
    else:
        fn = lambda x: calculate_discrete_kg_conditioning_on_single_output(state, x, target, disc, W)  # noqa: E731
    assert torch.autograd.gradcheck(fn, (xnew,), raise_exception=True)


@pytest.mark.parametrize("workload", ["small", "parity6d"])
@pytest.mark.parametrize("target", [None, 1])
def test_overflow_walk_path_value_and_grad(workload, target):
    """DKG_PLAN_FORCE_WALK: the envelope's list-overflow path (gift wrap over all
    lines, discretekg.py:382-401 walk) for every pair gives the oracle's KG and gradient."""
    model, D, X, W = make_problem(WORKLOADS[workload])
    X, W = X[:12], W[:8]
    om = to_oracle(model)
    kg_ref, g_ref = oracle_grad(om, X, D, W, target)
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    tgt = -1 if target is None else target
    Xd = X.to(DEV)
    plan_fwd = acq._state.plan(acq._W, target, 16, force_walk=True)
    kg = plan_fwd.forward(Xd).cpu()
    plan_grad = acq._state.plan(acq._W, target, 16, grad=True, force_walk=True)
    kg2, g = plan_grad.forward_grad(Xd)
    assert tgt == plan_fwd.target
    amax = lines_batched(om, X, D, W, target)[0].abs().amax((-1, -2))
    assert_within(kg, kg_ref, stated_tol(kg_ref, amax), "force-walk KG")
    assert_within(kg2.cpu(), kg_ref, stated_tol(kg_ref, amax), "force-walk KG (gradient plan)")
    assert_grad_close(g.cpu(), g_ref, grad_scale(om, X, D, W, target))


@pytest.mark.parametrize("target", [None, 1])
def test_flat_early_out_matches_the_full_gradient_path(target):
    """The gradient envelope settles flat pairs (every breakpoint beyond +-48) without the filter and hull:
    KG and dKG/dx against the full path (DKG_PLAN_FORCE_WALK, no early-out) on the headline batch, where 89 %
    of the pairs are flat, plus candidates placed on discretisation points (line 0 duplicated by a line k)."""
    model, D, X, W = make_problem(WORKLOADS["headline"])
    X = X.clone()
    X[:8] = D[torch.tensor([0, 37, 100, 333, 512, 700, 901, 1023])]
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    Xd = X.to(DEV).contiguous()
    kg, g = acq._plan_for(X.shape[0], grad=True).forward_grad(Xd)
    full = acq._state.plan(acq._W, acq._target, X.shape[0], grad=True, force_walk=True)
    kg_f, g_f = full.forward_grad(Xd)
    torch.testing.assert_close(kg, kg_f, rtol=1e-12, atol=0.0)
    assert_grad_close(g.cpu(), g_f.cpu(), grad_scale(to_oracle(model), X, D, W, target))
    # off the discretisation, KG = 0 leaves at most denormal-scale gradient terms (breakpoints at 37-40
    # standard deviations, where psi rounds to 0 before phi does) on either path
    zero = kg_f == 0
    zero[:8] = False
    assert float(g[zero].abs().max()) <= 1e-250 and float(g_f[zero].abs().max()) <= 1e-250


def _faithful_grad(om, X, D, W, target):
    """The oracle's structure-faithful forward (oracle.discretekg.discrete_kg_forward: the reference's joint
    posterior over [x; D] per candidate) with autograd: at x = z_k its lines 0 and k + 1 are exact copies."""
    from oracle.discretekg import discrete_kg_forward

    Xr = X.clone().unsqueeze(-2).requires_grad_(True)
    kg = discrete_kg_forward(om, Xr, D, W, target)
    (g,) = torch.autograd.grad(kg.sum(), Xr)
    return kg.detach(), g.squeeze(-2)


@pytest.mark.parametrize("case", ["small", "parity6d", "headline", "smoke_grid"])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_candidates_on_discretisation_points(case, target):
    """Candidates exactly on discretisation points (L-BFGS-B stops on box corners, and the reference's grids
    hold them).  The reference's joint posterior over [x_b; D] makes line 0 and line k + 1 exact copies there
    (rows 0 and k + 1 of one covariance matrix), so its walk takes line 0, the lowest index, and torch.max
    splits the gradient of max a between the copies.  The device builds line 0 from record k (Plan::dup, set
    by the covariance stage where r^2 = 0): KG (stated tolerance) and dKG/dx against the faithful oracle's
    autograd, and line 0 equal to line k + 1 bit for bit in the exported lines."""
    from dkg_amd.utils import make_torch_std_grid

    if case == "smoke_grid":  # the SMOKE run's problem and 3 x 3 grid (bo_loop.py:122-131): every grid point
        state, om, _, W, X, _ = load_golden("lengthscales0")
        model = state
        D = make_torch_std_grid(3, 2, {"dtype": torch.double})
        idx = torch.arange(D.shape[0])
        X = torch.cat([D, X[:3]])
    else:
        model, D, X, W = make_problem(WORKLOADS[case])
        om = to_oracle(model)
        idx = torch.linspace(0, D.shape[0] - 1, 9).round().long()
        X = torch.cat([D[idx], X[:3]])
    W = W[:8]
    kg_ref, g_ref = _faithful_grad(om, X, D, W, target)
    kg, g = native_grad(model, X, D, W, target)
    amax = lines_batched(om, X, D, W, target)[0].abs().amax((-1, -2))
    assert_within(kg, kg_ref, stated_tol(kg_ref, amax), "KG at discretisation points")
    r = assert_grad_close(g, g_ref, grad_scale(om, X, D, W, target))
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    a, b = acq._plan_for(X.shape[0]).lines(X.to(DEV).contiguous())
    for row, k in enumerate(idx.tolist()):
        assert torch.equal(a[row, :, 0], a[row, :, k + 1]) and torch.equal(b[row, :, 0], b[row, :, k + 1]), row
    print(f"{case} target={target}: gradient worst err/tol {r:.3g}")
