"""HIP path vs the CPU oracle on identical inputs (needs a real MI355X).

Every check goes through the C ABI (``include/dkg.h``) via ``dkg_amd``.
Tolerance (BASELINE.md "Accuracy"): |KG_gpu - KG_oracle| <= 1e-6 |KG_oracle|
+ 64 eps max|a|, asserted as stated, end to end and on every candidate.  The device lines must also
stay within helpers.LINE_RTOL of the oracle's, and the envelope kernel alone is held to the stated
tolerance on identical lines (helpers.parity_case).  The line gap's Lipschitz bound
(helpers.kg_line_floor) is printed as a diagnostic only.  Worst ratios: profiles/r03_parity.json
(tools/parity_report.py).
"""

import math

import pytest
import torch

from helpers import assert_within, check_parity_case, parity_case, stated_tol, to_oracle, to_state
from oracle.discretekg import (
    _kg_from_lines,
    calculate_discrete_kg,
    calculate_discrete_kg_conditioning_on_single_output,
    discrete_kg_forward,
    lines_batched,
)
from oracle.fit import make_reference_test_model, reference_test_discretisation

pytestmark = pytest.mark.gpu

DEV = "cuda"
TRIO = [[0.7, 0.3], [0.6, 0.4], [0.5, 0.5]]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def test_mfma_f64_lane_maps():
    from dkg_amd import _lib

    lib = _lib.load()
    g = torch.Generator().manual_seed(0)
    A = torch.randint(-8, 8, (16, 4), generator=g).double()
    Bm = torch.randint(-8, 8, (4, 16), generator=g).double()
    a, b = A.to(DEV), Bm.to(DEV)
    c = torch.empty(16, 16, dtype=torch.double, device=DEV)
    _lib.check(lib.dkg_debug_mfma_f64(_lib.ptr(a), _lib.ptr(b), _lib.ptr(c), 0), "debug")
    torch.cuda.synchronize()
    assert torch.equal(c.cpu(), A @ Bm)


# ---------------------------------------------------------------- envelope stage
def _oracle_lines_kg(a, b):
    return torch.stack([_kg_from_lines(a[p], b[p]) for p in range(a.shape[0])])


# reference epigraph / expectation KAT line sets (test_discretekg.py:150-327)
KAT_SETS = [
    ([1.0, 1.5], [0.0, 0.0]),
    ([1.5], [-1.9]),
    ([1.5, 0.0], [-0.5, 0.0]),
    ([0.0, 1.5], [0.0, -0.5]),
    ([0.0, 0.0, -0.5, 0.0], [-1.0, -1.0, 0.0, 1.5]),
    ([0.0, -1.0, 0.0], [-2.0, -1.0, 0.0]),
    ([-1.0, 0.0, 0.0], [-1.0, 0.0, -2.0]),
    ([1.5, 0.0], [0.0, 1e-12]),
    ([1.5, 0.0], [-0.5, -0.5]),
    ([0.0, 0.0], [0.0, 1.0]),
]


@pytest.mark.parametrize("idx", range(len(KAT_SETS)))
def test_lines_kg_reference_kats(idx):
    from dkg_amd import kg_from_lines

    a, b = (torch.tensor(v, dtype=torch.double) for v in KAT_SETS[idx])
    got = kg_from_lines(a.to(DEV), b.to(DEV)).cpu()
    ref = _kg_from_lines(a, b)
    assert abs(float(got) - float(ref)) <= 1e-12 + 1e-9 * abs(float(ref))


def test_lines_kg_relu_exact():
    from dkg_amd import kg_from_lines

    got = kg_from_lines(torch.tensor([0.0, 0.0], device=DEV), torch.tensor([0.0, 1.0], device=DEV))
    assert abs(float(got) - 1 / math.sqrt(2 * math.pi)) < 1e-15


@pytest.mark.parametrize("L", [1, 2, 3, 17, 64, 65, 200, 1025, 2112])
def test_lines_kg_random_sets(L):
    from dkg_amd import kg_from_lines

    g = torch.Generator().manual_seed(L)
    P = 64
    a = torch.randn(P, L, generator=g, dtype=torch.double)
    b = torch.randn(P, L, generator=g, dtype=torch.double)
    b[:4] = 0.0                       # short-circuit sets
    b[4:8] = b[4:8].round()           # many equal slopes
    a[8:12] = a[8:12].round()         # many equal intercepts
    b[12:14] = 1e-10 * b[12:14]       # |b| < 1e-9 everywhere
    got = kg_from_lines(a.to(DEV), b.to(DEV)).cpu()
    ref = _oracle_lines_kg(a, b)
    assert_within(got, ref, stated_tol(ref, a.abs().amax(-1)))
    assert bool((got >= 0).all())


def test_lines_kg_parabola_many_hull_lines():
    """Every line on the envelope (tangents of a parabola): survivor overflow path."""
    from dkg_amd import kg_from_lines

    L = 1025
    s = torch.linspace(-3, 3, L, dtype=torch.double)
    a, b = -0.5 * s * s, s  # tangent lines of z^2/2
    perm = torch.randperm(L, generator=torch.Generator().manual_seed(0))
    a, b = a[perm][None], b[perm][None]
    got, hull = kg_from_lines(a.to(DEV), b.to(DEV), return_hull_size=True)
    ref = _oracle_lines_kg(a, b)
    assert_within(got.cpu(), ref, stated_tol(ref, a.abs().amax(-1)))
    assert int(hull) == L


def test_lines_kg_empty_raises():
    from dkg_amd import kg_from_lines

    with pytest.raises(ValueError, match="at least one line"):
        kg_from_lines(torch.empty(3, 0, device=DEV), torch.empty(3, 0, device=DEV))


# ---------------------------------------------------------------- posterior stage
def test_cross_root_matches_dense_product():
    from dkg_amd.gp_state import DeviceGPState
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["small"])
    st = DeviceGPState(model, D)
    om = to_oracle(model)
    for c, o in zip(st.outputs, om.models):
        ref_mu = (o.covar(D, o.train_x) @ o.cache()["alpha"] + o.mean_constant)
        torch.testing.assert_close(c.disc_mean[: D.shape[0]].cpu(), ref_mu, rtol=1e-9, atol=1e-9)
        n = o.train_x.shape[0]
        Qd = o.covar(D, o.train_x) @ o.cache()["R"]
        N = D.shape[0]
        npad = (n + 15) // 16 * 16
        Npad = (N + 15) // 16 * 16
        # pair-packed: [t][j][l>>4][l&15][h] = P[16t + (l&15)][4(2j+h) + (l>>4)]
        F = c.disc_frag.cpu().reshape(Npad // 16, npad // 8, 4, 16, 2)
        dense = F.permute(0, 3, 1, 4, 2).reshape(Npad, npad)[:N, :n]
        torch.testing.assert_close(dense, Qd, rtol=1e-8, atol=1e-8)


# ---------------------------------------------------------------- end to end
@pytest.fixture(scope="module")
def ref_model():
    return make_reference_test_model(use_noise=True)


def test_reference_kat_table_full(ref_model):
    """test_discretekg.py:50-63 through the HIP path."""
    from dkg_amd import DiscreteKnowledgeGradient

    X = torch.tensor([[[[0.5, 0.5]], [[0, 1]], [[0, 0.5]]], [[[0, 0]], [[1, 0]], [[0.5, 0]]]], dtype=torch.double)
    acq = DiscreteKnowledgeGradient(to_state(ref_model), reference_test_discretisation(), torch.tensor(TRIO))
    kg = acq(X)
    torch.testing.assert_close(kg, torch.tensor([[0.0383, 0.0224, 0.0130], [0.0005, 0.0058, 0.0015]]),
                               atol=1e-4, rtol=1e-3)
    check_parity_case(parity_case(to_state(ref_model), reference_test_discretisation(), torch.tensor(TRIO),
                                  X.reshape(-1, 2), None))


def test_reference_kat_table_single_output(ref_model):
    """test_discretekg.py:65-79 through the HIP path."""
    from dkg_amd import DiscreteKnowledgeGradient

    X = torch.tensor([[[[0.5, 0.5]], [[0, 1]], [[0, 0.5]]], [[[0, 0]], [[1, 0]], [[0.5, 0]]]], dtype=torch.double)
    acq = DiscreteKnowledgeGradient(to_state(ref_model), reference_test_discretisation(), torch.tensor(TRIO),
                                    target_output_ix=0)
    kg = acq(X)
    torch.testing.assert_close(kg, torch.tensor([[0.0297, 0.0084, 0.0048], [0.0002, 0.0030, 0.0006]]),
                               atol=1e-4, rtol=1e-3)


def test_reference_kat_scalars(ref_model):
    """test_discretekg.py:87-108: the rel-1e-6 known answers."""
    from dkg_amd import calculate_discrete_kg as gpu_kg
    from dkg_amd import calculate_discrete_kg_conditioning_on_single_output as gpu_kg1

    D = reference_test_discretisation()
    W = torch.tensor(TRIO)
    x = torch.tensor([0.5, 0.5])
    assert float(gpu_kg(to_state(ref_model), x, D, W)) == pytest.approx(0.038261974207699244, rel=1e-6)
    assert float(gpu_kg1(to_state(ref_model), x, 0, D, W)) == pytest.approx(0.02968190595713936, rel=1e-6)
    assert float(calculate_discrete_kg(ref_model, x, D, W)) == pytest.approx(0.038261974207699244)
    assert float(calculate_discrete_kg_conditioning_on_single_output(ref_model, x, 0, D, W)) == pytest.approx(
        0.02968190595713936)


@pytest.mark.parametrize("workload", ["small", "parity6d"])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_forward_vs_faithful_oracle(workload, target):
    """The per-candidate, dense-covariance oracle (the reference's structure), stated tolerance alone."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS[workload])
    X = X[:16]
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)
    got = acq(X.unsqueeze(-2))
    om = to_oracle(model)
    ref = discrete_kg_forward(om, X.unsqueeze(-2), D, W, target)
    a_ref, _ = lines_batched(om, X, D, W, target)
    assert_within(got, ref, stated_tol(ref, a_ref.abs().amax((-1, -2))), "KG vs faithful oracle (stated tolerance)")
    assert bool((got >= 0).all())


@pytest.mark.parametrize("workload,nX", [("small", 32), ("parity6d", 32), ("headline", 128), ("headline_nd", 128)])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_forward_vs_oracle_all_candidates(workload, nX, target):
    """Every candidate of the workload: lines within LINE_RTOL of the oracle's, the envelope at the
    stated tolerance on identical lines, and KG end to end (helpers.parity_case)."""
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS[workload])
    res = parity_case(model, D, W, X[:nX], target)
    if workload == "headline_nd":
        # the envelopes are walked there (KG > 0 on all but a few candidates): the assertion is not a zero check
        assert res["kg_zero_frac"] <= 0.05
    print(f"{workload} target={target}: " + ", ".join(f"{k}={v:.3g}" for k, v in res.items()
                                                     if not k.startswith("_") and isinstance(v, float)))
    check_parity_case(res)


@pytest.mark.parametrize("target", [None, 0, 1])
def test_headline_pairs_and_mean(target):
    """KG per (candidate, scalarisation) of the headline batch; the forward's KG is their mean."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["headline"])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)
    pairs = acq.forward_pairs(X.unsqueeze(-2)).cpu()
    got = acq(X.unsqueeze(-2)).cpu()
    torch.testing.assert_close(got, pairs.mean(-1), rtol=1e-14, atol=1e-300)


def test_forward_deterministic_and_permutation_equivariant():
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["headline"])
    acq = DiscreteKnowledgeGradient(model, D, W)
    k1 = acq(X.unsqueeze(-2))
    k2 = acq(X.unsqueeze(-2))
    assert torch.equal(k1, k2)
    perm = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(3))
    k3 = acq(X[perm].unsqueeze(-2))
    assert torch.equal(k3, k1[perm])
    # scalarisation order does not change the mean beyond rounding
    acq2 = DiscreteKnowledgeGradient(model, D, W.flip(0))
    torch.testing.assert_close(acq2(X.unsqueeze(-2)), k1, rtol=1e-13, atol=1e-300)


def test_odd_sizes_and_padding():
    """n, N, B, S not multiples of 16, d = 3, three outputs with different n."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.model import ModelListGPState, SingleTaskGPState

    g = torch.Generator().manual_seed(5)
    outs = []
    for i, n in enumerate([37, 50, 23]):
        X = torch.rand(n, 3, generator=g, dtype=torch.double)
        y = torch.sin(3 * X.sum(-1) + i) + 0.1 * torch.randn(n, generator=g, dtype=torch.double)
        outs.append(SingleTaskGPState(X, y, [0.3, 0.5, 0.7][: 3], 1.0 + i, 1e-3, 0.1 * i,
                                      kernel=["matern", "matern", "rbf"][i], nu=[2.5, 1.5, None][i],
                                      y_mean=0.3 * i, y_std=1.0 + 0.5 * i))
    model = ModelListGPState(*outs)
    D = torch.rand(77, 3, generator=g, dtype=torch.double)
    W = torch.rand(5, 3, generator=g, dtype=torch.double)
    W = W / W.sum(-1, keepdim=True)
    Xc = torch.rand(19, 3, generator=g, dtype=torch.double)
    for target in (None, 0, 2):
        check_parity_case(parity_case(model, D, W, Xc, target))
        DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)(Xc.unsqueeze(-2))


def test_matern12_single_output_and_no_weights():
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.model import ModelListGPState, SingleTaskGPState

    g = torch.Generator().manual_seed(9)
    X = torch.rand(40, 2, generator=g, dtype=torch.double)
    y = torch.cos(4 * X[:, 0]) * X[:, 1]
    model = ModelListGPState(SingleTaskGPState(X, y, [0.4, 0.3], 2.0, 1e-2, 0.0, kernel="matern", nu=0.5))
    D = torch.rand(100, 2, generator=g, dtype=torch.double)
    Xc = torch.rand(10, 1, 2, generator=g, dtype=torch.double)
    got = DiscreteKnowledgeGradient(model, D)(Xc)
    res = parity_case(model, D, torch.tensor([[1.0]], dtype=torch.double), Xc.squeeze(1), None)
    check_parity_case(res)
    torch.testing.assert_close(got.cpu(), res["_tensors"][0], rtol=0, atol=0)


def test_lines_match_oracle_lines_headline():
    """The KG per (candidate, scalarisation) equals the reference epigraph on oracle lines."""
    from dkg_amd import DiscreteKnowledgeGradient, kg_from_lines
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["headline"])
    om = to_oracle(model)
    a, b = lines_batched(om, X[:8], D, W, None)
    got = kg_from_lines(a.to(DEV), b.to(DEV)).cpu()
    ref = torch.stack([torch.stack([_kg_from_lines(a[i, j], b[i, j]) for j in range(a.shape[1])])
                       for i in range(a.shape[0])])
    assert_within(got, ref, stated_tol(ref, a.abs().amax(-1)))
    del DiscreteKnowledgeGradient


def test_wave_butterfly_primitives():
    """DPP + permlane butterfly steps pair every lane with the mirror lane of the other half-group."""
    from dkg_amd import _lib

    lib = _lib.load()
    x = torch.arange(64, dtype=torch.double) * 3.0 + 1.0
    xin = x.to(DEV)
    out = torch.empty(512, dtype=torch.double, device=DEV)
    _lib.check(lib.dkg_debug_wave_ops(_lib.ptr(xin), _lib.ptr(out), 0), "debug_wave")
    torch.cuda.synchronize()
    o = out.cpu().reshape(8, 64)
    lanes = torch.arange(64)
    expected_partner = [lanes ^ 1, lanes ^ 2, (lanes & ~7) | (7 - (lanes & 7)), (lanes & ~15) | (15 - (lanes & 15)),
                        lanes ^ 16, lanes ^ 32]
    for s, p in enumerate(expected_partner):
        assert torch.equal(o[s], x[p]), f"step {s}: got lanes {((o[s] - 1) / 3).long().tolist()}"
    assert torch.equal(o[6], torch.full((64,), float(x.sum()), dtype=torch.double))
    assert torch.equal(o[7], torch.full((64,), float(x.max()), dtype=torch.double))


# ---------------------------------------------------------------- stress sizes
@pytest.mark.parametrize("target", [None, 2])
def test_stress_config_parity(target):
    """BASELINE.json configs[4] shape (m=3, n=1024, N=4096 = 64^2 grid, S=32), fp64, 64 candidates: the 48
    with the largest device KG (KG > 0: walked envelopes) and the 16 smallest; stated tolerance on every one.
    Measured worst KG err/tol 0.042 (full) / 0.061 (target 2) (profiles/r03/grad_probe.json)."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["stress"])
    kg = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)(X.to(DEV).unsqueeze(-2)).cpu()
    order = torch.argsort(kg, descending=True)
    pick = torch.cat([order[:48], order[-16:]])
    assert int((kg[pick] > 0).sum()) >= 48
    check_parity_case(parity_case(model, D, W, X[pick], target))


@pytest.mark.parametrize("target", [None, 1])
def test_stress_refinement_parity(target):
    """Streaming envelope at the stress shape over 24 candidates x 32 scalarisations (noise 1e-3 s: many
    lines near the upper hull; the sample chain keeps up to a few hundred of the 4097 lines per pair)."""
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["stress32"])
    check_parity_case(parity_case(model, D, W, X[:24], target))


@pytest.mark.parametrize("workload,target", [("stress32", None), ("stress", 2)])
def test_stress_sample_chain_matches_overflow_path(workload, target):
    """The streaming envelope's one staged pass filters against the chain of a strided sample's quickhull
    vertices (dkg_device.h chain_keep); DKG_PLAN_NO_CHAIN sends every pair through the overflow path
    instead (extremes from the streamed lines, quickhull refinement, the walks).  Both walks are the
    reference walk, so KG per pair and the envelope sizes must agree bit for bit."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS[workload])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    Xd = X[:32].to(DEV).contiguous()
    chain = acq._state.plan(acq._W, acq._target, 32)
    plain = acq._state.plan(acq._W, acq._target, 32, no_chain=True)
    kg_c, pairs_c, hull_c = chain.forward_stats(Xd)
    kg_p, pairs_p, hull_p = plain.forward_stats(Xd)
    assert int((pairs_c > 0).sum()) > 0
    assert torch.equal(pairs_c, pairs_p)
    assert torch.equal(hull_c, hull_p)
    assert torch.equal(kg_c, kg_p)


# ---------------------------------------------------------------- fp32 contractions (DKG_PLAN_F32)
# SURVEY.md 8(d) asks for rel 1e-3 against the fp64 build.  cov = s k(x, z) - Q_X . Q_D loses the factor
# c = s / (posterior variance) of relative precision to cancellation, so fp32 contractions (unit roundoff
# 6e-8, n ~ 10^2..10^3 terms) give slopes good to ~c * 1e-6.  Measured (tools/f32_check.py,
# profiles/r02/r02k_f32_check.txt): c <= 34 (parity6d, headline_nd) -> max rel 1e-4 over the candidates
# with KG >= 1e-3 of the batch maximum; c ~ 10^3..10^6 (headline, BASELINE configs[4] stress32 with
# noise 1e-3 s) -> rel 1e-2..1.  The 1e-3 target is therefore attainable only for c <~ 10^2, and these
# tests hold the fp32 mode to it there; at the stress conditioning it is unattainable in fp32 (DESIGN.md
# 4.6) and the stress config is computed in fp64.
F32_RTOL = 1e-3


def _f32_vs_f64(workload, target, nX):
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS[workload])
    Xd = X[:nX].to(DEV).unsqueeze(-2)
    k64 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)(Xd).cpu()
    acq32 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV, precision="fp32")
    k32 = acq32(Xd).cpu()
    assert acq32._plan.f32
    return k32, k64


@pytest.mark.parametrize("target", [None, 0, 1])
@pytest.mark.parametrize("workload,nX", [("parity6d", 32), ("headline_nd", 128)])
def test_f32_meets_1e3_when_conditioning_allows(workload, nX, target):
    k32, k64 = _f32_vs_f64(workload, target, nX)
    d = (k32 - k64).abs()
    keep = k64.abs() >= 1e-3 * k64.abs().max()
    assert int(keep.sum()) >= nX // 4
    rel = (d / k64.abs())[keep]
    assert float(rel.max()) <= F32_RTOL, f"max rel {float(rel.max()):.3e}"
    assert bool((d <= F32_RTOL * k64.abs().max()).all())


def test_f32_stress32_error_model():
    """BASELINE configs[4]'s shape (stress32: m 3, n 1024, N 4096, S 32, B 256) in the fp32-contraction mode,
    every candidate and path held to DESIGN.md 4.6's error model: the fp32 contraction leaves each slope with
    ~c_b 1e-6 relative error, c_b = max_i s_i / v_i(x_b) the posterior's cancellation factor (from the
    oracle's R), so |KG32 - KG64| <= c_b 1e-6 sqrt(2/pi) max_k |b_k| (KG's Lipschitz constant in the slopes
    times the slope error).  Measured worst ratio 0.0044 (profiles/r04/f32_stress.json); the distribution
    is printed.  Relative errors are not asserted: with c_b ~ 1e3..6e4 rel 1e-3 is out of fp32's reach
    (DESIGN.md 4.6), and the stress config is reported in fp64."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["stress32"])
    om = to_oracle(model)
    canc = []
    for o in om.models:
        q = o.covar(X, o.train_x) @ o.cache()["R"]
        canc.append(o.outputscale / (o.outputscale - (q * q).sum(-1)).clamp_min(1e-300))
    canc = torch.stack(canc)                                  # [m, B]
    Xd = X.to(DEV).unsqueeze(-2)
    qs = torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=torch.double)
    for target in (None, 0, 2):
        acq64 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
        k64 = acq64(Xd).cpu()
        acq32 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV, precision="fp32")
        k32 = acq32(Xd).cpu()
        assert acq32._plan.f32
        _, b = acq64._plan_for(X.shape[0]).lines(X.to(DEV).contiguous())
        bmax = b.abs().amax((-1, -2)).cpu()
        del b
        c = canc.amax(0) if target is None else canc[target]
        bound = c * 1e-6 * math.sqrt(2 / math.pi) * bmax
        ratio = (k32 - k64).abs() / bound
        print(f"stress32 fp32 target={target}: KG>0 on {int((k64 > 0).sum())} of {X.shape[0]}; "
              f"err / (c 1e-6 sqrt(2/pi) max|b|) quantiles 0.5/0.9/0.99/max {ratio.quantile(qs).tolist()}")
        assert bool((ratio <= 1.0).all()), f"target={target}: worst ratio {float(ratio.max()):.3g}"


def test_f32_refuses_gradient():
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.errors import UnsupportedError
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV, precision="fp32")
    Xg = X[:4].to(DEV).unsqueeze(-2).requires_grad_(True)
    with pytest.raises(UnsupportedError):
        acq(Xg)


# ---------------------------------------------------------------- envelope sizes (dkg_plan_hull_sizes)
# The forward's envelope sizes equal the reference walk's on the same lines exactly:
# tests/test_gpu_epigraph.py::test_forward_envelopes_are_the_reference_walk.


def test_concurrent_plans_on_streams_match_single_stream():
    """bench.py's --streams / --graph path: four plans (own Q_X / cov workspace each) run interleaved batches on
    four HIP streams; every batch's KG is bit-identical to the same batch run alone on one stream."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    w = WORKLOADS["headline"]
    model, D, X, W = make_problem(w)
    dev = torch.device("cuda", 0)
    acq = DiscreteKnowledgeGradient(model, D, W, device=dev)
    base = acq._plan_for(w.B)
    batches = [torch.quasirandom.SobolEngine(w.d, scramble=True, seed=11 + k).draw(w.B, dtype=torch.double)
               .to(dev).contiguous() for k in range(12)]
    want = []
    for Xb in batches:
        kg = torch.empty(w.B, dtype=torch.double, device=dev)
        base.forward_into(Xb, kg)
        want.append(kg)
    torch.cuda.synchronize()
    main = torch.cuda.current_stream(dev)
    streams = [main] + [torch.cuda.Stream(dev) for _ in range(3)]
    plans = [base] + [acq._state.plan(acq._W, acq._target, base.max_B) for _ in range(3)]
    got = torch.full((len(batches), w.B), float("nan"), dtype=torch.double, device=dev)
    for s in streams[1:]:
        s.wait_stream(main)
    for k, Xb in enumerate(batches):
        with torch.cuda.stream(streams[k % 4]):
            plans[k % 4].forward_into(Xb, got[k])
    for s in streams[1:]:
        main.wait_stream(s)
    torch.cuda.synchronize()
    for k in range(len(batches)):
        assert torch.equal(got[k], want[k]), k

    # bench.py --graph: the same interleaving captured once as a HIP graph, replayed twice
    got.fill_(float("nan"))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream(dev)
        lanes = [cs] + streams[1:]
        for s in lanes[1:]:
            s.wait_stream(cs)
        for k, Xb in enumerate(batches):
            with torch.cuda.stream(lanes[k % 4]):
                plans[k % 4].forward_into(Xb, got[k])
        for s in lanes[1:]:
            cs.wait_stream(s)
    for _ in range(2):
        got.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        for k in range(len(batches)):
            assert torch.equal(got[k], want[k]), k
