"""Pin the CPU oracle against the reference's own known answers.

Every case here restates one test of the reference's
``tests/modules/acquisition/test_discretekg.py`` (cited per test) and checks
``oracle/`` against the expected values written in that file.
"""

import math
import re

import pytest
import torch

from oracle.discretekg import (
    calculate_discrete_kg,
    calculate_discrete_kg_conditioning_on_single_output,
    calculate_epigraph_indices,
    calculate_expected_value_of_piecewise_linear_function,
    discrete_kg_batched,
    discrete_kg_forward,
)
from oracle.fit import make_reference_test_model, reference_test_discretisation

TRIO = [[0.7, 0.3], [0.6, 0.4], [0.5, 0.5]]
SINGLE = [[0.6, 0.4]]


@pytest.fixture(scope="module")
def noisy_model():
    return make_reference_test_model(use_noise=True)


@pytest.fixture(scope="module")
def noiseless_model():
    return make_reference_test_model(use_noise=False)


@pytest.fixture()
def disc():
    return reference_test_discretisation()


@pytest.fixture()
def target_x():
    return torch.tensor([[[[0.5, 0.5]], [[0, 1]], [[0, 0.5]]], [[[0, 0]], [[1, 0]], [[0.5, 0]]]])


# test_discretekg.py:50-63
def test_forward_full_table(noisy_model, disc, target_x):
    kg = discrete_kg_forward(noisy_model, target_x, disc, torch.tensor(TRIO))
    exp = torch.tensor([[0.0383, 0.0224, 0.0130], [0.0005, 0.0058, 0.0015]])
    torch.testing.assert_close(kg, exp, atol=1e-4, rtol=1e-3)


# test_discretekg.py:65-79
def test_forward_single_output_table(noisy_model, disc, target_x):
    kg = discrete_kg_forward(noisy_model, target_x, disc, torch.tensor(TRIO), target_output_ix=0)
    exp = torch.tensor([[0.0297, 0.0084, 0.0048], [0.0002, 0.0030, 0.0006]])
    torch.testing.assert_close(kg, exp, atol=1e-4, rtol=1e-3)


# test_discretekg.py:87-93
def test_calculate_discrete_kg_kat(noisy_model, disc):
    kg = calculate_discrete_kg(noisy_model, torch.tensor([0.5, 0.5]), disc, torch.tensor(TRIO))
    assert kg.item() == pytest.approx(0.038261974207699244)


# test_discretekg.py:95-108
def test_calculate_discrete_kg_single_output_kat(noisy_model, disc):
    kg = calculate_discrete_kg_conditioning_on_single_output(
        noisy_model, torch.tensor([0.5, 0.5]), 0, disc, torch.tensor(TRIO))
    assert kg.item() == pytest.approx(0.02968190595713936)


def test_batched_oracle_matches_faithful(noisy_model, disc, target_x):
    X = target_x.reshape(-1, 2)
    W = torch.tensor(TRIO)
    for target in (None, 0, 1):
        kg, _ = discrete_kg_batched(noisy_model, X, disc, W, target)
        ref = discrete_kg_forward(noisy_model, target_x, disc, W, target).reshape(-1)
        torch.testing.assert_close(kg, ref, rtol=1e-10, atol=1e-13)


# test_discretekg.py:110-135
@pytest.mark.parametrize("noisy", [True, False], ids=["noisy", "noiseless"])
@pytest.mark.parametrize("weights", [SINGLE, TRIO], ids=["single", "trio"])
@pytest.mark.parametrize("target", [None, 0, 1])
def test_gradients(noisy, weights, target, noisy_model, noiseless_model, disc):
    model = noisy_model if noisy else noiseless_model
    xnew = torch.tensor([0.51, 0.51], requires_grad=True)
    W = torch.tensor(weights)
    if target is None:
        fn = lambda x: calculate_discrete_kg(model, x, disc, W)  # noqa: E731
    else:
        fn = lambda x: calculate_discrete_kg_conditioning_on_single_output(model, x, target, disc, W)  # noqa: E731
    assert torch.autograd.gradcheck(fn, (xnew,), raise_exception=True)


# test_discretekg.py:139-148
def test_epigraph_raises_on_empty_input():
    msg = "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0."
    with pytest.raises(ValueError, match=re.escape(msg)):
        calculate_epigraph_indices(torch.tensor([]), torch.tensor([]))


# test_discretekg.py:150-158
def test_epigraph_zero_slopes():
    idx, x = calculate_epigraph_indices(torch.tensor([1, 1.5]), torch.tensor([0.0, 0.0]))
    torch.testing.assert_close(idx, torch.tensor([1]))
    torch.testing.assert_close(x, torch.tensor([]))


# test_discretekg.py:160-167
def test_epigraph_single_line():
    idx, x = calculate_epigraph_indices(torch.tensor([1.5]), torch.tensor([-1.9]))
    torch.testing.assert_close(idx, torch.tensor([0]))
    torch.testing.assert_close(x, torch.tensor([]))


# test_discretekg.py:169-182
@pytest.mark.parametrize("ordered", [True, False])
def test_epigraph_two_lines(ordered):
    a = torch.tensor([1.5, 0])
    b = torch.tensor([-0.5, 0])
    if not ordered:
        a, b = torch.flip(a, [0]), torch.flip(b, [0])
    idx, x = calculate_epigraph_indices(a, b)
    torch.testing.assert_close(idx, torch.tensor([0, 1] if ordered else [1, 0]))
    torch.testing.assert_close(x, torch.tensor([3.0]))


# test_discretekg.py:184-196
def test_epigraph_two_equal_slopes():
    idx, x = calculate_epigraph_indices(torch.tensor([0, 0, -0.5, 0]), torch.tensor([-1, -1, 0, 1.5]))
    torch.testing.assert_close(idx, torch.tensor([0, 3]))
    torch.testing.assert_close(x, torch.tensor([0.0]))


# test_discretekg.py:198-215
@pytest.mark.parametrize(("order", "expected"), [([0, 1, 2], [0, 2]), ([1, 2, 0], [2, 1])])
def test_epigraph_ignores_lines_below(order, expected):
    a = torch.tensor([0.0, -1, 0])[order]
    b = torch.tensor([-2.0, -1, 0])[order]
    idx, x = calculate_epigraph_indices(a, b)
    torch.testing.assert_close(idx, torch.tensor(expected))
    torch.testing.assert_close(x, torch.tensor([0.0]))


# test_discretekg.py:217-235
@pytest.mark.parametrize("slopes", [[-0.5, 0], [0, 1e-12], [-0.5, -0.5]], ids=["normal", "tiny", "identical"])
def test_epigraph_gradients(slopes):
    a = torch.tensor([1.5, 0], requires_grad=True)
    b = torch.tensor(slopes, requires_grad=True)
    assert torch.autograd.gradcheck(lambda *args: calculate_epigraph_indices(*args)[1], (a, b))


# test_discretekg.py:237-260
@pytest.mark.parametrize("offset", [0, 1])
def test_epigraph_gradients_two_of_four_identical(offset):
    a = torch.tensor([offset, offset, -0.5, 0], dtype=torch.double, requires_grad=True)
    b = torch.tensor([-1, -1, 0, 1.5], dtype=torch.double, requires_grad=True)
    _, x = calculate_epigraph_indices(a, b)
    only = x.squeeze(0)
    assert only.ndim == 0
    (gb,) = torch.autograd.grad(only, b, retain_graph=True)
    (ga,) = torch.autograd.grad(only, a, retain_graph=True)
    torch.testing.assert_close(gb, torch.tensor([0.16 * offset, 0.0, 0.0, -0.16 * offset]))
    torch.testing.assert_close(ga, torch.tensor([0.4, 0.0, 0.0, -0.4]))


# test_discretekg.py:264-276
def test_expectation_raises_on_empty():
    e = torch.tensor([])
    msg = "Expected inputs to specify at least one line. Got intercepts.shape[-1]=0."
    with pytest.raises(ValueError, match=re.escape(msg)):
        calculate_expected_value_of_piecewise_linear_function(e, e, e)


# test_discretekg.py:278-309
@pytest.mark.parametrize(("a", "b", "c", "expected"), [
    ([1.5], [0.0], [], 1.5),
    ([0.0], [1.0], [], 0.0),
    ([0.0, 0.0], [0.0, 1.0], [0.0], 1 / math.sqrt(2 * math.pi)),
    ([0.0, 1, 1, 0], [0.0, 1, -1, 0], [-1.0, 0, 1],
     math.erf(1 / math.sqrt(2)) - (1 - math.exp(-1 / 2)) * math.sqrt(2 / math.pi)),
], ids=["constant", "sloped", "relu", "hump"])
def test_expectation_kats(a, b, c, expected):
    v = calculate_expected_value_of_piecewise_linear_function(torch.tensor(a), torch.tensor(b), torch.tensor(c))
    assert v == pytest.approx(expected)


# test_discretekg.py:329-342
def test_expectation_gradients():
    a = torch.tensor([0.0, 1, 1, 0], requires_grad=True)
    b = torch.tensor([0.0, 1, -1, 0], requires_grad=True)
    c = torch.tensor([-1.0, 0, 1], requires_grad=True)
    assert torch.autograd.gradcheck(calculate_expected_value_of_piecewise_linear_function, (a, b, c))
