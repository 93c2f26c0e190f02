"""K forward batches in one launch per stage (include/dkg.h dkg_plan_forward_batches).

Each batch keeps its own candidates and its own result row: the batched launch must write, bit for bit,
what one dkg_plan_forward per batch writes (the reference's forward is per batch, discretekg.py:131-159).
Covers batch sizes that are not multiples of the 16-candidate tiles, the decoupled path, candidates on
discretisation points (the per-tile clearing of the coincidence marks), a launch large enough that the
whole launch would take the other covariance block shape (the block shape is chosen per batch), and the
stress shape (64 x 64 covariance blocks).
"""

import pytest
import torch

from dkg_amd import DiscreteKnowledgeGradient, _lib
from dkg_amd.errors import BotorchTensorDimensionError
from dkg_amd.synthetic import WORKLOADS, make_problem

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


# The batched launches with every fp64 covariance block kernel enabled that their shapes take (the defaults, the
# 64 x 32 blocks, the register-operand and whole-record blocks: dkg_debug_cov_kernels); every one must give the
# per-batch bits (one dkg_plan_forward per batch, the narrow blocks).
COV_KERNELS = {"default": 0, "blk": _lib.DKG_COV_ENABLE_BLK, "rec2": _lib.DKG_COV_ENABLE_REC2,
               "reg": _lib.DKG_COV_ENABLE_REG}


@pytest.fixture(params=list(COV_KERNELS))
def cov_kernels(request):
    lib = _lib.load()
    prev = lib.dkg_debug_cov_kernels(COV_KERNELS[request.param])
    yield request.param
    torch.cuda.synchronize()
    lib.dkg_debug_cov_kernels(prev)


def _batched_vs_single(wname, B, K, target, on_grid=0, seed=3, fused=False, precision="fp64"):
    """fused: the per-batch reference plan is a DKG_PLAN_FUSED one (its forward is the one-launch kernel; the
    batched launch runs the stage kernels).  precision "fp32": both plans DKG_PLAN_F32."""
    model, D, _, W = make_problem(WORKLOADS[wname])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV, precision=precision)
    f32 = precision == "fp32"
    d = D.shape[1]
    X = torch.quasirandom.SobolEngine(d, scramble=True, seed=seed).draw(K * B, dtype=torch.double)
    if on_grid:  # some candidates exactly on discretisation points, in the middle batch
        k = K // 2
        X[k * B:k * B + on_grid] = D[torch.arange(on_grid) * 7 % D.shape[0]]
    X = X.to(DEV)
    big = acq._state.plan(acq._W, acq._target, K * B, f32=f32)
    one = acq._state.plan(acq._W, acq._target, B, fused=fused, f32=f32)
    kg = torch.full((K * B,), float("nan"), dtype=torch.double, device=DEV)
    big.forward_batches_into(X, kg, B)
    ref = torch.full_like(kg, float("nan"))
    for j in range(K):
        one.forward_into(X[j * B:(j + 1) * B], ref[j * B:(j + 1) * B])
    # twice: the second launch on the same plan must not see the first one's accumulators or marks
    kg2 = torch.full_like(kg, float("nan"))
    big.forward_batches_into(X, kg2, B)
    torch.cuda.synchronize()
    return kg.cpu(), kg2.cpu(), ref.cpu()


@pytest.mark.parametrize("wname,B,K,target,on_grid", [
    ("headline", 128, 20, None, 0),    # 2,560 candidates: as one forward it would take the 64 x 64 blocks
    ("headline", 128, 4, 0, 5),
    ("small", 37, 5, None, 3),         # batches straddle the 16-candidate tiles
    ("small", 1, 9, 1, 1),
    ("parity6d", 23, 3, None, 0),
    ("headline_nd", 128, 3, 1, 0),
])
def test_batched_launch_writes_the_per_batch_bits(wname, B, K, target, on_grid, cov_kernels):
    kg, kg2, ref = _batched_vs_single(wname, B, K, target, on_grid)
    assert not torch.isnan(ref).any()
    assert torch.equal(kg, ref)
    assert torch.equal(kg2, ref)
    if wname != "headline" or on_grid:
        assert (ref > 0).any()


@pytest.mark.parametrize("wname,B,K", [("headline", 128, 5), ("small", 37, 3), ("small", 1, 4)])
def test_batched_launch_matches_a_fused_plan(wname, B, K):
    """include/dkg.h promises the per-batch bits for a DKG_PLAN_FUSED plan too: its dkg_plan_forward is the
    one-launch forward (dkg_fused.h), the batched launch the three stage kernels."""
    model, D, _, W = make_problem(WORKLOADS[wname])
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    one = acq._state.plan(acq._W, acq._target, B, fused=True)
    assert one.fused, "the reference plan must take the one-launch forward"
    del one
    kg, kg2, ref = _batched_vs_single(wname, B, K, None, on_grid=2 if B > 2 else 0, fused=True)
    assert not torch.isnan(ref).any()
    assert torch.equal(kg, ref) and torch.equal(kg2, ref)


@pytest.mark.parametrize("wname,B,K", [("stress32", 256, 2), ("headline_nd", 128, 5)])
def test_batched_launch_fp32_plan(wname, B, K):
    """F32 plans keep the per-batch bits as well: a batched launch takes the fp32 block kernels
    (posterior_cov_big32 / cross_big32) exactly where one batch would (stress32: both; headline_nd: neither)."""
    kg, kg2, ref = _batched_vs_single(wname, B, K, None, precision="fp32")
    assert not torch.isnan(ref).any()
    assert torch.equal(kg, ref) and torch.equal(kg2, ref)


def test_batched_launch_stress_shape(cov_kernels):
    kg, kg2, ref = _batched_vs_single("stress", 256, 2, None, 0)
    assert torch.equal(kg, ref) and torch.equal(kg2, ref)


def test_batched_launch_arguments():
    model, D, X0, W = make_problem(WORKLOADS["small"])
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    plan = acq._state.plan(acq._W, acq._target, 64)
    X = X0.to(DEV).repeat(3, 1).contiguous()
    kg = torch.empty(96, dtype=torch.double, device=DEV)
    with pytest.raises(ValueError):
        plan.forward_batches_into(X[:95], kg, 32)          # not whole batches
    with pytest.raises(BotorchTensorDimensionError):  # DKG_ERR_ARG
        plan.forward_batches_into(X, kg, 32)               # 96 > plan capacity 64
    plan.forward_batches_into(X[:0], kg, 32)               # no batches: nothing to do


@pytest.mark.parametrize("kernel,nu", [("matern", 2.5), ("rbf", None)])
def test_batched_launch_outputs_of_different_sizes(kernel, nu, cov_kernels):
    """Outputs with different training-set sizes (ragged n: 100, 300 and 37 points) in a launch that takes the
    K(x, X) fill and the 64 x 32 cross blocks (5 x 128 = 640 candidates), against one forward per batch (the
    in-workgroup fill of cross_root_plan_kernel): the blocks of the smaller outputs past their own tiles return
    early, and every output's K(x, X) uses its own k-block count."""
    from dkg_amd.model import ModelListGPState, SingleTaskGPState

    g = torch.Generator().manual_seed(5)
    outs = []
    for n, ls in ((100, [0.3, 0.5]), (300, [0.2, 0.4]), (37, [0.6, 0.3])):
        X = torch.rand(n, 2, generator=g, dtype=torch.double)
        y = torch.sin(3 * X[:, 0]) + X[:, 1] ** 2 + 0.01 * torch.randn(n, generator=g, dtype=torch.double)
        outs.append(SingleTaskGPState(X, y, ls, 1.3, 1e-3, 0.1, kernel=kernel, nu=nu))
    model = ModelListGPState(*outs)
    D = torch.rand(200, 2, generator=g, dtype=torch.double)
    W = torch.rand(6, 3, generator=g, dtype=torch.double)
    W = W / W.sum(-1, keepdim=True)
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    B, K = 128, 5
    X = torch.quasirandom.SobolEngine(2, scramble=True, seed=7).draw(K * B, dtype=torch.double).to(DEV)
    big = acq._state.plan(acq._W, acq._target, K * B)
    one = acq._state.plan(acq._W, acq._target, B)
    kg = torch.full((K * B,), float("nan"), dtype=torch.double, device=DEV)
    big.forward_batches_into(X, kg, B)
    ref = torch.full_like(kg, float("nan"))
    for j in range(K):
        one.forward_into(X[j * B:(j + 1) * B], ref[j * B:(j + 1) * B])
    torch.cuda.synchronize()
    assert not torch.isnan(ref).any()
    assert torch.equal(kg.cpu(), ref.cpu())
    assert (ref > 0).any()


@pytest.mark.parametrize("K,kernel,nu", [(5, "matern", 2.5), (4, "rbf", None), (5, "matern", 1.5)])
def test_batched_launch_two_outputs_whole_records(K, kernel, nu, cov_kernels):
    """Two outputs of different (odd-half) training sizes, N = 1000 lines: K = 5 / 4 batches of 128 take the
    block kernel that writes both outputs' records from one workgroup (posterior_cov_rec2_kernel, RT = 5 / 4:
    256 blocks), whose K halves are 7 and 4 words here; its rows must be the per-batch bits (narrow blocks)."""
    from dkg_amd.model import ModelListGPState, SingleTaskGPState

    g = torch.Generator().manual_seed(11)
    outs = []
    for n, ls in ((100, [0.3, 0.5]), (61, [0.2, 0.4])):
        X = torch.rand(n, 2, generator=g, dtype=torch.double)
        y = torch.sin(3 * X[:, 0]) + X[:, 1] ** 2 + 0.01 * torch.randn(n, generator=g, dtype=torch.double)
        outs.append(SingleTaskGPState(X, y, ls, 1.3, 1e-3, 0.1, kernel=kernel, nu=nu))
    model = ModelListGPState(*outs)
    D = torch.rand(1000, 2, generator=g, dtype=torch.double)
    D[7] = torch.tensor([0.25, 0.75], dtype=torch.double)
    W = torch.rand(8, 2, generator=g, dtype=torch.double)
    W = W / W.sum(-1, keepdim=True)
    acq = DiscreteKnowledgeGradient(model, D, W, device=DEV)
    B = 128
    X = torch.quasirandom.SobolEngine(2, scramble=True, seed=9).draw(K * B, dtype=torch.double)
    X[130] = D[7]  # a candidate on a discretisation point (Plan::dup from the record kernel)
    X = X.to(DEV)
    big = acq._state.plan(acq._W, acq._target, K * B)
    one = acq._state.plan(acq._W, acq._target, B)
    kg = torch.full((K * B,), float("nan"), dtype=torch.double, device=DEV)
    big.forward_batches_into(X, kg, B)
    ref = torch.full_like(kg, float("nan"))
    for j in range(K):
        one.forward_into(X[j * B:(j + 1) * B], ref[j * B:(j + 1) * B])
    torch.cuda.synchronize()
    assert not torch.isnan(ref).any()
    assert torch.equal(kg.cpu(), ref.cpu())
    assert (ref > 0).any()
