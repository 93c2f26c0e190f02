"""The reference's epigraph and expectation functions on the device, exactly (needs a real MI355X).

``dkg_amd.calculate_epigraph_indices`` runs the reference walk (``discretekg.py:341-412``) in the
HIP envelope code (``dkg_walk.h``).  It is index work, so the bar is bit-exactness: the same line
indices and the same IEEE intersections as the oracle's restatement of the walk
(``oracle.discretekg.calculate_epigraph_indices``) on the same lines, for the reference's own KATs
(``tests/modules/acquisition/test_discretekg.py:139-260``), random sets with ties, sets that
overflow the candidate list, and the lines the forward plans build at the small / headline /
stress workloads.  The forward's envelope sizes (``dkg_plan_hull_sizes``) must equal the walk's
on the same lines.

Exact duplicate lines: for more than 16 lines the reference's first ``torch.sort`` (unstable on
CPU) may return any one of a set of identical lines; the build and the oracle return the lowest
index.  Every set below with duplicates of the walked lines is compared to the
oracle, which sorts stably.
"""

import math
import re

import pytest
import torch

from helpers import to_oracle
from oracle.discretekg import calculate_epigraph_indices as ref_epigraph
from oracle.discretekg import calculate_expected_value_of_piecewise_linear_function as ref_expectation

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _epi(a, b):
    from dkg_amd import calculate_epigraph_indices

    i, x = calculate_epigraph_indices(torch.as_tensor(a, dtype=torch.double).to(DEV),
                                      torch.as_tensor(b, dtype=torch.double).to(DEV))
    return i.cpu(), x.cpu()


def _assert_same_walk(a, b):
    gi, gx = _epi(a, b)
    ri, rx = ref_epigraph(torch.as_tensor(a, dtype=torch.double), torch.as_tensor(b, dtype=torch.double))
    assert torch.equal(gi, ri), f"indices {gi.tolist()} != {ri.tolist()}"
    assert torch.equal(gx, rx.to(gx.dtype)), f"intersections differ: max |d| {float((gx - rx).abs().max()):.3e}"
    return len(ri)


# ---------------------------------------------------------------- reference KATs (test_discretekg.py:139-260)
def test_epigraph_empty_raises():
    from dkg_amd import calculate_epigraph_indices

    msg = "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0."
    with pytest.raises(ValueError, match=re.escape(msg)):
        calculate_epigraph_indices(torch.tensor([], device=DEV), torch.tensor([], device=DEV))


def test_epigraph_zero_slopes():
    i, x = _epi([1, 1.5], [0, 0])
    assert i.tolist() == [1] and x.numel() == 0


def test_epigraph_single_line():
    i, x = _epi([1.5], [-1.9])
    assert i.tolist() == [0] and x.numel() == 0


@pytest.mark.parametrize("ordered", [True, False])
def test_epigraph_two_lines(ordered):
    a, b = [1.5, 0.0], [-0.5, 0.0]
    if not ordered:
        a, b = a[::-1], b[::-1]
    i, x = _epi(a, b)
    assert i.tolist() == ([0, 1] if ordered else [1, 0])
    assert x.tolist() == [3.0]


def test_epigraph_two_equal_slopes():
    i, x = _epi([0, 0, -0.5, 0], [-1, -1, 0, 1.5])
    assert i.tolist() == [0, 3] and x.tolist() == [0.0]


@pytest.mark.parametrize("order,expected", [([0, 1, 2], [0, 2]), ([1, 2, 0], [2, 1])])
def test_epigraph_ignores_lines_below(order, expected):
    a = torch.tensor([0.0, -1.0, 0.0])[order]
    b = torch.tensor([-2.0, -1.0, 0.0])[order]
    i, x = _epi(a, b)
    assert i.tolist() == expected and x.tolist() == [0.0]


@pytest.mark.parametrize("slopes", [[-0.5, 0.0], [0.0, 1e-12], [-0.5, -0.5]])
def test_epigraph_gradients(slopes):
    """test_discretekg.py:213-228: gradcheck of the intersections w.r.t. intercepts and slopes."""
    from dkg_amd import calculate_epigraph_indices

    a = torch.tensor([1.5, 0.0], dtype=torch.double, device=DEV, requires_grad=True)
    b = torch.tensor(slopes, dtype=torch.double, device=DEV, requires_grad=True)
    torch.autograd.gradcheck(lambda *t: calculate_epigraph_indices(*t)[1], (a, b), raise_exception=True)


@pytest.mark.parametrize("offset", [0.0, 1.0])
def test_epigraph_gradients_two_of_four_identical(offset):
    """test_discretekg.py:230-260."""
    from dkg_amd import calculate_epigraph_indices

    a = torch.tensor([offset, offset, -0.5, 0.0], dtype=torch.double, device=DEV, requires_grad=True)
    b = torch.tensor([-1.0, -1.0, 0.0, 1.5], dtype=torch.double, device=DEV, requires_grad=True)
    _, x = calculate_epigraph_indices(a, b)
    only = x.squeeze(0)
    assert only.ndim == 0
    (gb,) = torch.autograd.grad(only, b, retain_graph=True)
    (ga,) = torch.autograd.grad(only, a, retain_graph=True)
    torch.testing.assert_close(gb.cpu(), torch.tensor([0.16 * offset, 0.0, 0.0, -0.16 * offset], dtype=torch.double))
    torch.testing.assert_close(ga.cpu(), torch.tensor([0.4, 0.0, 0.0, -0.4], dtype=torch.double))


# ---------------------------------------------------------------- expectation KATs (test_discretekg.py:263-342)
def _pwl(a, b, c, **kw):
    from dkg_amd import calculate_expected_value_of_piecewise_linear_function

    t = lambda v: torch.tensor(v, dtype=torch.double, device=DEV, **kw)  # noqa: E731
    return calculate_expected_value_of_piecewise_linear_function(t(a), t(b), t(c))


def test_expectation_empty_raises():
    msg = "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0."
    with pytest.raises(ValueError, match=re.escape(msg)):
        _pwl([], [], [])


@pytest.mark.parametrize("a,b,c,want", [
    ([1.5], [0.0], [], 1.5),
    ([0.0], [1.0], [], 0.0),
    ([0.0, 0.0], [0.0, 1.0], [0.0], 1 / math.sqrt(2 * math.pi)),
    ([0.0, 1.0, 1.0, 0.0], [0.0, 1.0, -1.0, 0.0], [-1.0, 0.0, 1.0],
     math.erf(1 / math.sqrt(2)) - (1 - math.exp(-0.5)) * math.sqrt(2 / math.pi)),
])
def test_expectation_kats(a, b, c, want):
    got = float(_pwl(a, b, c))
    ref = float(ref_expectation(*(torch.tensor(v, dtype=torch.double) for v in (a, b, c))))
    assert got == pytest.approx(want, rel=1e-12, abs=1e-15)
    assert got == pytest.approx(ref, rel=1e-12, abs=1e-15)


def test_expectation_gradients():
    """test_discretekg.py:329-342 (the hump): gradcheck w.r.t. intercepts, slopes and boundaries."""
    from dkg_amd import calculate_expected_value_of_piecewise_linear_function

    t = lambda v: torch.tensor(v, dtype=torch.double, device=DEV, requires_grad=True)  # noqa: E731
    torch.autograd.gradcheck(calculate_expected_value_of_piecewise_linear_function,
                             (t([0.0, 1.0, 1.0, 0.0]), t([0.0, 1.0, -1.0, 0.0]), t([-1.0, 0.0, 1.0])),
                             raise_exception=True)


def test_expectation_random_batches_vs_oracle():
    from dkg_amd import _lib
    from dkg_amd.gp_state import current_stream_ptr

    g = torch.Generator().manual_seed(3)
    for m in (1, 2, 5, 63, 64, 65, 300):
        P = 8
        a = torch.randn(P, m, generator=g, dtype=torch.double)
        b = torch.randn(P, m, generator=g, dtype=torch.double)
        c = torch.sort(torch.randn(P, max(m - 1, 1), generator=g, dtype=torch.double) * 2, dim=-1).values[:, : m - 1]
        ad, bd, cd = a.to(DEV), b.to(DEV), c.contiguous().to(DEV)
        out = torch.empty(P, dtype=torch.double, device=DEV)
        lib = _lib.load()
        _lib.check(lib.dkg_pwl_expectation(_lib.ptr(ad), _lib.ptr(bd), _lib.ptr(cd) if m > 1 else 0, P, m,
                                           _lib.ptr(out), current_stream_ptr(torch.device(DEV))), "pwl")
        ref = torch.stack([ref_expectation(a[p], b[p], c[p]) for p in range(P)])
        scale = (a.abs().sum(-1) + b.abs().sum(-1))
        assert bool(((out.cpu() - ref).abs() <= 1e-14 * scale).all()), m


# ---------------------------------------------------------------- random and adversarial sets
@pytest.mark.parametrize("L", [1, 2, 3, 16, 17, 64, 65, 200, 1025, 2112, 3000])
def test_epigraph_random_sets_exact(L):
    g = torch.Generator().manual_seed(100 + L)
    for rep in range(6):
        a = torch.randn(L, generator=g, dtype=torch.double)
        b = torch.randn(L, generator=g, dtype=torch.double)
        if rep == 1:
            b = b.round()            # many equal slopes
        elif rep == 2:
            a = a.round()            # many equal intercepts
        elif rep == 3:
            b = 1e-10 * b            # every |b| < 1e-9: short-circuit
        elif rep == 4 and L >= 4:    # exact duplicates and lines concurrent at a breakpoint
            a[L // 2:] = a[: L - L // 2].clone()
            b[L // 2:] = b[: L - L // 2].clone()
            a[1] = 0.0
            b[1] = 0.0
            a[2] = 1.0
            b[2] = -1.0
            a[3] = 1.0
            b[3] = 1.0               # lines 1..3 meet... 2 and 3 cross at z = 0 where line 1 = 0 < 1
        elif rep == 5:
            a = (a * 4).round() / 4  # coarse grid: many ties in the intersections
            b = (b * 4).round() / 4
        _assert_same_walk(a, b)


def test_epigraph_parabola_every_line_on_the_envelope():
    """Every line is an envelope line (tangents of z^2/2, shuffled): the candidate list overflows and
    the walk runs over all lines."""
    for L in (130, 1025, 2500):
        s = torch.linspace(-3, 3, L, dtype=torch.double)
        perm = torch.randperm(L, generator=torch.Generator().manual_seed(L))
        assert _assert_same_walk((-0.5 * s * s)[perm], s[perm]) == L


def test_epigraph_concurrent_lines():
    """Many lines through one point: the reference's argmin-first rule visits them all (zero-length
    segments), in slope order."""
    k = torch.arange(-8, 9, dtype=torch.double)
    a = 1.0 - 0.5 * k       # every line passes through (z = 0.5, y = 1)
    b = k
    perm = torch.randperm(len(k), generator=torch.Generator().manual_seed(0))
    n = _assert_same_walk(a[perm], b[perm])
    assert n >= 2


def test_epigraph_batched_matches_single():
    from dkg_amd import calculate_epigraph_indices_batched

    g = torch.Generator().manual_seed(7)
    a = torch.randn(5, 40, generator=g, dtype=torch.double)
    b = torch.randn(5, 40, generator=g, dtype=torch.double)
    idx, xs, cnt = calculate_epigraph_indices_batched(a.to(DEV), b.to(DEV))
    for p in range(5):
        ri, rx = ref_epigraph(a[p], b[p])
        m = int(cnt[p])
        assert torch.equal(idx[p, :m].cpu(), ri) and torch.equal(xs[p, : m - 1].cpu(), rx)


def test_epigraph_far_breakpoints_redo_and_padding():
    """Envelope breakpoints near 1e10 and 1e11 (two nearly parallel lines on the hull): the first list walk
    leaves the 2^30 guard and is redone over a list filtered at the wider margin that covers it; the result
    is the reference walk, and every index / intersection past the count is -1 / NaN."""
    from dkg_amd import calculate_epigraph_indices_batched

    g = torch.Generator().manual_seed(11)
    a = torch.cat([torch.tensor([-5.0, 1.0, 1.0 - 1e-3, -1e11], dtype=torch.double),
                   -10.0 - torch.rand(60, generator=g, dtype=torch.double)])
    b = torch.cat([torch.tensor([-2.0, 0.0, 1e-13, 1.0], dtype=torch.double),
                   2.0 * torch.rand(60, generator=g, dtype=torch.double) - 1.0])
    assert _assert_same_walk(a, b) >= 3
    A, Bm = torch.stack([a, a.flip(0)]), torch.stack([b, b.flip(0)])
    idx, xs, cnt = calculate_epigraph_indices_batched(A.to(DEV), Bm.to(DEV))
    idx, xs, cnt = idx.cpu(), xs.cpu(), cnt.cpu()
    for p in range(2):
        ri, rx = ref_epigraph(A[p], Bm[p])
        m = int(cnt[p])
        assert m == len(ri) and torch.equal(idx[p, :m], ri) and torch.equal(xs[p, : m - 1], rx)
        assert bool((idx[p, m:] == -1).all()) and bool(xs[p, m - 1:].isnan().all())
        assert float(rx.abs().max()) > 2.0 ** 30


def test_epigraph_padding_past_the_count():
    """Every set of a random batch: indices past the count are -1 and intersections past count - 1 NaN."""
    from dkg_amd import calculate_epigraph_indices_batched

    g = torch.Generator().manual_seed(12)
    for L in (5, 200, 1025, 3000):
        a = torch.randn(16, L, generator=g, dtype=torch.double)
        b = torch.randn(16, L, generator=g, dtype=torch.double)
        b[:2] = 0.0  # short-circuit sets: one index, no intersection
        idx, xs, cnt = calculate_epigraph_indices_batched(a.to(DEV), b.to(DEV))
        idx, xs, cnt = idx.cpu(), xs.cpu(), cnt.cpu()
        for p in range(16):
            m = int(cnt[p])
            assert bool((idx[p, m:] == -1).all()) and bool((idx[p, :m] >= 0).all())
            assert bool(xs[p, max(m - 1, 0):].isnan().all()) and not bool(xs[p, : max(m - 1, 0)].isnan().any())


# ---------------------------------------------------------------- the forward's own lines
def _plan_lines(workload, nX, target):
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, D, X, W = make_problem(WORKLOADS[workload])
    X = X[:nX]
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    plan = acq._plan_for(nX)
    kg, pairs, hull = plan.forward_stats(X.to(DEV))
    a, b = plan.lines(X.to(DEV))
    return a, b, pairs, hull


@pytest.mark.parametrize("workload,nX,target", [("small", 32, None), ("small", 32, 1), ("parity6d", 16, None),
                                                ("headline", 128, None), ("headline", 128, 0),
                                                ("stress32", 4, None)])
def test_forward_envelopes_are_the_reference_walk(workload, nX, target):
    """On the lines the plan builds (exported bit for bit by dkg_plan_lines): the device walk returns
    the oracle walk's indices and intersections exactly, and the forward's envelope sizes
    (dkg_plan_hull_sizes) equal the walk's -- every (candidate, scalarisation) pair."""
    from dkg_amd import calculate_epigraph_indices_batched

    a, b, pairs, hull = _plan_lines(workload, nX, target)
    B, S, L = a.shape
    idx, xs, cnt = calculate_epigraph_indices_batched(a, b)
    ac, bc, idx, xs, cnt, hull = a.cpu(), b.cpu(), idx.cpu(), xs.cpu(), cnt.cpu(), hull.cpu()
    for i in range(B):
        for j in range(S):
            ri, rx = ref_epigraph(ac[i, j], bc[i, j])
            m = len(ri)
            assert int(cnt[i, j]) == m and int(hull[i, j]) == m, (i, j, int(cnt[i, j]), int(hull[i, j]), m)
            assert torch.equal(idx[i, j, :m], ri), (i, j)
            assert torch.equal(xs[i, j, : m - 1], rx), (i, j)
