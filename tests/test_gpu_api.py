"""The reference's DiscreteKnowledgeGradient surface around the forward (discretekg.py:33-159).

create_with_sobol_sample seeds like draw_sobol_samples (torch's global RNG); set_X_pending
raises UnsupportedError; target_output_ix indexes the outputs as the reference's
posteriors[obj_idx_new] does (negative counts from the end, out of range -> IndexError at
evaluation); the model is read live (a mutated model gives the new model's KG).
"""

import pytest
import torch

from dkg_amd import DiscreteKnowledgeGradient
from dkg_amd.errors import UnsupportedError
from dkg_amd.model import ModelListGPState, SingleTaskGPState
from dkg_amd.optim import draw_sobol_samples
from dkg_amd.synthetic import WORKLOADS, make_problem

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def test_create_with_sobol_sample_is_seeded_by_the_global_rng():
    model, _, X, W = make_problem(WORKLOADS["small"])
    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double)
    torch.manual_seed(123)
    a1 = DiscreteKnowledgeGradient.create_with_sobol_sample(model, bounds, 64, W)
    torch.manual_seed(123)
    a2 = DiscreteKnowledgeGradient.create_with_sobol_sample(model, bounds, 64, W)
    assert torch.equal(a1.x_discretisation, a2.x_discretisation)
    # the discretisation is draw_sobol_samples(bounds, N, q=1).squeeze(1) (discretekg.py:56-58)
    torch.manual_seed(123)
    ref = draw_sobol_samples(bounds, 64, q=1).squeeze(1)
    assert torch.equal(a1.x_discretisation, ref)
    assert a1.x_discretisation.shape == (64, 2) and a1.x_discretisation.dtype == bounds.dtype
    torch.manual_seed(124)
    a3 = DiscreteKnowledgeGradient.create_with_sobol_sample(model, bounds, 64, W)
    assert not torch.equal(a1.x_discretisation, a3.x_discretisation)
    kg1 = a1(X[:8].unsqueeze(-2))
    kg2 = a2(X[:8].unsqueeze(-2))
    assert torch.equal(kg1, kg2)
    # scaled bounds land inside the box
    b2 = torch.tensor([[-2.0, 1.0], [3.0, 1.5]], dtype=torch.double)
    a4 = DiscreteKnowledgeGradient.create_with_sobol_sample(model, b2, 32, W, target_output_ix=1)
    assert bool(((a4.x_discretisation >= b2[0]) & (a4.x_discretisation <= b2[1])).all())
    assert a4.target_output_ix == 1


def test_set_x_pending_raises():
    model, D, _, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W)
    with pytest.raises(UnsupportedError, match="does not account for X_pending"):
        acq.set_X_pending(torch.rand(2, 2, dtype=torch.double))
    with pytest.raises(UnsupportedError):
        acq.set_X_pending(None)


def test_negative_target_counts_from_the_end():
    model, D, X, W = make_problem(WORKLOADS["small"])
    Xb = X[:16].unsqueeze(-2)
    last = DiscreteKnowledgeGradient(model, D, W, target_output_ix=model.num_outputs - 1)(Xb)
    neg = DiscreteKnowledgeGradient(model, D, W, target_output_ix=-1)(Xb)
    assert torch.equal(last, neg)
    first = DiscreteKnowledgeGradient(model, D, W, target_output_ix=-model.num_outputs)(Xb)
    assert torch.equal(first, DiscreteKnowledgeGradient(model, D, W, target_output_ix=0)(Xb))
    full = DiscreteKnowledgeGradient(model, D, W)(Xb)
    assert not torch.equal(neg, full)  # -1 is the last output, not the full evaluation


def test_target_out_of_range_raises_index_error_at_evaluation():
    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=model.num_outputs)  # constructs, as the reference
    with pytest.raises(IndexError):
        acq(X[:4].unsqueeze(-2))


def test_model_is_read_live():
    """A refit (new hyperparameters), new training data and an in-place edit are all seen by forward."""
    model, D, X, W = make_problem(WORKLOADS["small"])
    Xb = X[:16].unsqueeze(-2)
    acq = DiscreteKnowledgeGradient(model, D, W)
    before = acq(Xb)
    # refit: replace an output's hyperparameters
    m0 = model.models[0]
    model.models[0] = SingleTaskGPState(m0.train_x, m0.train_y, m0.lengthscale * 1.5, m0.outputscale, m0.noise,
                                        m0.mean_constant, m0.kernel, m0.nu, m0.y_mean, m0.y_std)
    after = acq(Xb)
    fresh = DiscreteKnowledgeGradient(model, D, W)(Xb)
    assert torch.equal(after, fresh) and not torch.equal(after, before)
    # in-place edit of the training targets
    model.models[1].train_y.mul_(2.0)
    edited = acq(Xb)
    assert torch.equal(edited, DiscreteKnowledgeGradient(model, D, W)(Xb))
    assert not torch.equal(edited, after)
    # unchanged model: the cached state is reused (same values, no rebuild)
    st = acq._state
    acq(Xb)
    assert acq._state is st


@pytest.mark.parametrize("where", ["cpu", DEV])
def test_weights_are_read_live(where):
    """The scalarisation weights are read at every forward, as the reference's forward reads
    self.scalarisation_weights: an in-place edit (host) or a newly assigned tensor (host or device) gives the
    new weights' KG, while the plans keep their own snapshot (an edit never reaches a plan directly)."""
    from helpers import assert_within, stated_tol
    from oracle.discretekg import discrete_kg_batched, lines_batched
    from oracle.gp import ModelList, OutputGP

    model, D, X, W = make_problem(WORKLOADS["small"])
    om = ModelList([OutputGP(m.train_x, m.train_y, m.lengthscale, m.outputscale, m.noise, m.mean_constant,
                             m.kernel, m.nu, m.y_mean, m.y_std) for m in model.models])
    Xb = X[:8]
    Wl = W.clone().to(where)
    acq = DiscreteKnowledgeGradient(model, D, Wl)
    base = acq(Xb.unsqueeze(-2)).cpu()
    W2 = W.flip(-1).contiguous()
    if where == "cpu":
        Wl.data.copy_(W2)         # in place through .data (no version bump): seen by value
    else:
        acq.scalarisation_weights = W2.to(where)
    got = acq(Xb.unsqueeze(-2)).cpu()
    ref, _ = discrete_kg_batched(om, Xb, D, W2)
    fresh = DiscreteKnowledgeGradient(model, D, W2)(Xb.unsqueeze(-2)).cpu()
    assert torch.equal(got, fresh)
    assert not torch.equal(got, base)
    assert_within(got, ref, stated_tol(ref, lines_batched(om, Xb, D, W2)[0].abs().amax((-1, -2))))
    # a plan's weights are its own copy: editing the tensor a plan was built from changes nothing in it
    Wd = W.to(DEV)
    plan = acq._state.plan(Wd, None, 8)
    k1 = plan.forward(Xb.to(DEV)).cpu()
    Wd.mul_(0.5)
    assert torch.equal(plan.forward(Xb.to(DEV)).cpu(), k1)


def test_single_output_model_without_weights():
    g = torch.Generator().manual_seed(2)
    Xt = torch.rand(30, 2, generator=g, dtype=torch.double)
    st = SingleTaskGPState(Xt, torch.sin(4 * Xt[:, 0]), [0.3, 0.4], 1.0, 1e-3)
    D = torch.rand(50, 2, generator=g, dtype=torch.double)
    a = DiscreteKnowledgeGradient(st, D)
    assert torch.equal(a.scalarisation_weights, torch.tensor([[1.0]], dtype=torch.double))
    b = DiscreteKnowledgeGradient(ModelListGPState(st), D, torch.tensor([[1.0]], dtype=torch.double))
    Xc = torch.rand(5, 1, 2, generator=g, dtype=torch.double)
    assert torch.equal(a(Xc), b(Xc))


@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("B", [1, 5, 16])
def test_value_and_grad_host_matches_forward_and_autograd(B, graph):
    """value_and_grad_host (one round trip, graph-replayed launches): the same bits as forward + autograd."""
    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=1 if B == 5 else None)
    for rep in range(3):  # repeated calls replay the captured graph on new inputs
        Xb = X.roll(7 * rep, 0)[:B].clone()
        Xg = Xb.to(DEV).unsqueeze(-2).requires_grad_(True)
        kg_ref = acq(Xg)
        (g_ref,) = torch.autograd.grad(kg_ref.sum(), Xg)
        plan = acq._plan_for(B, grad=True)
        kg, g = plan.forward_grad_host(Xb, graph=graph)
        assert kg.device.type == "cpu" and g.shape == (B, 2)
        assert torch.equal(kg, kg_ref.detach().cpu())
        assert torch.equal(g, g_ref.squeeze(-2).cpu())
        kg2, g2 = acq.value_and_grad_host(Xb.unsqueeze(-2))
        assert kg2.shape == (B,) and g2.shape == (B, 1, 2)
        assert torch.equal(kg2, kg) and torch.equal(g2.squeeze(-2), g)


def test_value_and_grad_host_input_forms():
    """value_and_grad_host takes X as [B, d], [*batch, 1, d], fp32 or a non-contiguous view: results shaped
    like the batch and like X, the bits of the contiguous fp64 call."""
    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W)
    Xb = X[:6].clone()
    kg, g = acq.value_and_grad_host(Xb.reshape(3, 2, 1, 2))
    assert kg.shape == (3, 2) and g.shape == (3, 2, 1, 2)
    kg2, g2 = acq.value_and_grad_host(Xb)
    assert kg2.shape == (6,) and g2.shape == (6, 2)
    assert torch.equal(kg.reshape(-1), kg2) and torch.equal(g.reshape(6, 2), g2)
    wide = torch.zeros(6, 4, dtype=torch.double)
    wide[:, ::2] = Xb
    kg3, g3 = acq.value_and_grad_host(wide[:, ::2])  # non-contiguous
    assert torch.equal(kg3, kg2) and torch.equal(g3, g2)
    X32 = Xb.float()
    kg4, g4 = acq.value_and_grad_host(X32.unsqueeze(-2))
    kg5, g5 = acq.value_and_grad_host(X32.double().unsqueeze(-2))
    assert torch.equal(kg4, kg5) and torch.equal(g4, g5)


def test_value_and_grad_host_follows_a_refit_model():
    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W)
    kg0, _ = acq.value_and_grad_host(X[:1])
    m0 = model.models[0]
    model.models[0] = SingleTaskGPState(m0.train_x, m0.train_y, m0.lengthscale * 1.5, m0.outputscale, m0.noise,
                                        m0.mean_constant, m0.kernel, m0.nu, m0.y_mean, m0.y_std)
    kg1, g1 = acq.value_and_grad_host(X[:1])
    Xg = X[:1].to(DEV).unsqueeze(-2).requires_grad_(True)
    kg_ref = DiscreteKnowledgeGradient(model, D, W)(Xg)
    (g_ref,) = torch.autograd.grad(kg_ref.sum(), Xg)
    assert torch.equal(kg1, kg_ref.detach().cpu()) and torch.equal(g1, g_ref.squeeze(-2).cpu())
    assert not torch.equal(kg0, kg1)


@pytest.mark.parametrize("B", [1, 3, 16])
def test_host_route_matches_device_route(B):
    """forward of a host X (the call optimize_acqf makes: host candidates with requires_grad, then backward)
    runs _HostForwardFn -- one round trip, host backward -- and gives the device route's bits."""
    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=0 if B == 3 else None)
    for rep in range(2):
        Xb = X.roll(5 * rep, 0)[:B].clone().reshape(B, 1, 1, 2)  # batch shape (B, 1)
        Xh = Xb.clone().requires_grad_(True)
        kg_h = acq(Xh)
        assert kg_h.device.type == "cpu" and kg_h.shape == (B, 1) and kg_h.requires_grad
        (g_h,) = torch.autograd.grad((kg_h * 2.0).sum(), Xh)
        Xd = Xb.to(DEV).requires_grad_(True)
        kg_d = acq(Xd)
        (g_d,) = torch.autograd.grad((kg_d * 2.0).sum(), Xd)
        assert torch.equal(kg_h.detach(), kg_d.detach().cpu())
        assert torch.equal(g_h, g_d.cpu())
        # without grad: the forward-only plan, same values as the device route's forward-only plan
        with torch.no_grad():
            assert torch.equal(acq(Xb), acq(Xb.to(DEV)).cpu())
    # float32 host candidates: computed in fp64, returned in the input's dtype (as the device route)
    X32 = X[:B].float().unsqueeze(-2)
    assert torch.equal(acq(X32), acq(X32.to(DEV)).cpu())
    assert acq(X[:0].unsqueeze(-2)).shape == (0,)


@pytest.mark.parametrize("S", [8, 16, 24])
@pytest.mark.parametrize("B", [1, 10, 11])
def test_candidates_in_kernel_arguments_match_the_copy_path(B, S):
    """forward_grad_host with B * d <= DKG_XARG_MAX passes the candidates in the first kernel's arguments
    (dkg_plan_forward_grad_hostx) and gets [KG | dKG/dx] written into its pinned buffer by the envelope
    kernel (one workgroup per candidate at S = 8, the second of two at S = 16; copies after it at S = 24);
    past the bound, a pinned copy in: all give dkg_plan_forward_grad's bits (d = 6: B = 10 is inside,
    B = 11 past the bound)."""
    from dkg_amd import _lib
    from dkg_amd.utils import sample_simplex

    model, D, X, _ = make_problem(WORKLOADS["parity6d"])
    W = sample_simplex(2, S, qmc=True, seed=5)
    acq = DiscreteKnowledgeGradient(model, D, W)
    plan = acq._plan_for(B, grad=True)
    assert (B * 6 <= _lib.DKG_XARG_MAX) == (B <= 10)
    for rep in range(3):
        Xb = X.roll(3 * rep, 0)[:B].clone()
        kg_ref, g_ref = plan.forward_grad(Xb.to(DEV))
        kg, g = plan.forward_grad_host(Xb)
        assert torch.equal(kg, kg_ref.cpu()) and torch.equal(g, g_ref.cpu())
        # a strided host view of the same candidates
        Xs = torch.stack([Xb, Xb], -1)[..., 0]
        kg2, g2 = plan.forward_grad_host(Xs)
        assert torch.equal(kg2, kg) and torch.equal(g2, g)


def test_acquisitions_on_one_model_share_the_device_state():
    """One DeviceGPState per (model, discretisation): the per-output acquisitions the reference builds on
    one fitted model (acquisition_optimisation_strategy.py:209-216) share it; a changed model or grid
    gets its own, and the values are those of a fresh state."""
    from dkg_amd.gp_state import DeviceGPState

    model, D, X, W = make_problem(WORKLOADS["small"])
    a0 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=0)
    a1 = DiscreteKnowledgeGradient(model, D.clone(), W, target_output_ix=1)
    af = DiscreteKnowledgeGradient(model, D, W)
    assert a0._state is a1._state is af._state
    Xb = X[:8].unsqueeze(-2)
    fresh = DeviceGPState(model, D)
    for acq, t in ((a0, 0), (a1, 1), (af, None)):
        assert torch.equal(acq(Xb).cpu(), fresh.forward(X[:8].to(DEV), W, t).cpu())
    other = DiscreteKnowledgeGradient(model, D + 0.01, W)
    assert other._state is not a0._state
    model.models[0].train_y.add_(1.0)  # an in-place edit: the next forward rebuilds, the old entry stays put
    a0(Xb)
    assert a0._state is not a1._state
