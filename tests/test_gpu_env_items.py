"""Multi-candidate envelope workgroups (include/dkg.h dkg_debug_env_items).

With ipw > 1 a staged-forward envelope workgroup stages mu_D's records once and runs ipw candidates in turn,
DMA-ing the next candidate's covariance records into a second LDS buffer while the current candidate's pairs
run.  Every value of ipw must give the bits of one candidate per workgroup: KG per candidate and per pair,
for batched and single launches, ragged last blocks (B not a multiple of ipw), candidates on discretisation
points (line 0 copied from a staged record), the decoupled path and walked pairs (headline_nd).
"""

import pytest
import torch

from dkg_amd import DiscreteKnowledgeGradient, _lib
from dkg_amd.synthetic import WORKLOADS, make_problem

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def _run(wname, B, K, target, on_grid, ipw, seed=5):
    lib = _lib.load()
    prev = lib.dkg_debug_env_items(ipw)
    try:
        model, D, _, W = make_problem(WORKLOADS[wname])
        acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
        d = D.shape[1]
        X = torch.quasirandom.SobolEngine(d, scramble=True, seed=seed).draw(K * B, dtype=torch.double)
        if on_grid:
            X[:on_grid] = D[torch.arange(on_grid) * 5 % D.shape[0]]
        X = X.to(DEV)
        big = acq._state.plan(acq._W, acq._target, K * B)
        kg = torch.full((K * B,), float("nan"), dtype=torch.double, device=DEV)
        big.forward_batches_into(X, kg, B)
        pairs = torch.full((B, W.shape[0]), float("nan"), dtype=torch.double, device=DEV)
        one = acq._state.plan(acq._W, acq._target, B)
        one_kg = torch.full((B,), float("nan"), dtype=torch.double, device=DEV)
        one.forward_into(X[:B], one_kg)
        one.forward(X[:B], kg_pairs=pairs)
        torch.cuda.synchronize()
        return kg.cpu(), one_kg.cpu(), pairs.cpu()
    finally:
        lib.dkg_debug_env_items(prev)


@pytest.mark.parametrize("wname,B,K,target,on_grid", [
    ("headline", 128, 5, None, 0),
    ("headline", 77, 2, 0, 4),        # ragged: 77 candidates over blocks of ipw
    ("small", 37, 3, None, 3),
    ("small", 1, 4, 1, 1),
    ("parity6d", 23, 3, None, 0),
    ("headline_nd", 128, 2, 1, 0),    # KG > 0 on every pair: walked envelopes
])
@pytest.mark.parametrize("ipw", [2, 3, 8])
def test_multi_candidate_envelope_gives_the_same_bits(wname, B, K, target, on_grid, ipw):
    ref = _run(wname, B, K, target, on_grid, 1)
    got = _run(wname, B, K, target, on_grid, ipw)
    for r, g in zip(ref, got):
        assert not torch.isnan(r).any()
        assert torch.equal(g, r)


def test_env_items_hook_reads_and_clamps():
    lib = _lib.load()
    prev = lib.dkg_debug_env_items(-1)
    try:
        assert lib.dkg_debug_env_items(4) == prev
        assert lib.dkg_debug_env_items(-1) == 4
        lib.dkg_debug_env_items(100)
        assert lib.dkg_debug_env_items(-1) == 8
    finally:
        lib.dkg_debug_env_items(prev)
