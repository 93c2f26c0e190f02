"""Host-side pieces of the drop-in surface that need no device (CPU)."""

import torch

from dkg_amd.discretekg import _fingerprint
from dkg_amd.model import ModelListGPState, SingleTaskGPState
from dkg_amd.optim import draw_sobol_samples


def test_draw_sobol_samples_follows_the_global_rng():
    b = torch.tensor([[0.0, -1.0], [2.0, 1.0]], dtype=torch.double)
    torch.manual_seed(7)
    a = draw_sobol_samples(b, 16, q=1)
    torch.manual_seed(7)
    c = draw_sobol_samples(b, 16, q=1)
    assert a.shape == (16, 1, 2) and torch.equal(a, c)
    assert bool(((a >= b[0]) & (a <= b[1])).all())
    torch.manual_seed(8)
    assert not torch.equal(a, draw_sobol_samples(b, 16, q=1))


def test_fingerprint_tracks_refits_and_in_place_edits():
    x = torch.rand(10, 2, dtype=torch.double)
    m = ModelListGPState(SingleTaskGPState(x, torch.rand(10, dtype=torch.double), [0.2, 0.3], 1.0, 1e-4))
    fp = _fingerprint(m)
    assert _fingerprint(m) == fp
    m.models[0].train_y.add_(1.0)
    fp2 = _fingerprint(m)
    assert fp2 != fp
    m.models[0].noise = 1e-3
    assert _fingerprint(m) != fp2


def test_fingerprint_sees_hyperparameters_written_through_data():
    """gpytorch's initialize() / constraint setters write hyperparameters through .data (no version bump):
    small tensors are fingerprinted by value too, so the shared device state is not reused stale."""
    x = torch.rand(10, 2, dtype=torch.double)
    m = ModelListGPState(SingleTaskGPState(x, torch.rand(10, dtype=torch.double), [0.2, 0.3], 1.0, 1e-4))
    fp = _fingerprint(m)
    m.models[0].lengthscale.data.copy_(torch.tensor([0.25, 0.3], dtype=torch.double))
    assert _fingerprint(m) != fp
    mod = torch.nn.Module()
    mod.raw = torch.nn.Parameter(torch.zeros(3, dtype=torch.double))
    f1 = _fingerprint(mod)
    mod.raw.data.copy_(torch.ones(3, dtype=torch.double))
    assert _fingerprint(mod) != f1


def test_clear_state_cache():
    from dkg_amd import clear_state_cache
    from dkg_amd.discretekg import _STATE_CACHE

    _STATE_CACHE.append(("fp", None, None, None, None))
    clear_state_cache()
    assert _STATE_CACHE == []
