"""On-device state preparation (dkg_prepare_output) vs LAPACK on the host.

The reference's posterior caches come from GPyTorch's exact prediction
strategy and linear_operator's ``psd_safe_cholesky`` (call sites
``discretekg.py:182-185, 275-284``): L = chol(K + noise I) with absolute
jitter 1e-8 * 10**i retries, R = L^{-T}, alpha = K^{-1}(y - c).  The library
computes them with its own HIP kernels (csrc/dkg_linalg.hip); this file checks
them against torch.linalg on the CPU (LAPACK) through the C ABI.

Tolerances are backward-error style (independent of conditioning):
  |L L^T - K|_max        <= 64 eps n |K|_max
  |L Linv - I|_max       <= 64 eps n |L|_max |Linv|_max
  |K alpha - r|_max      <= 64 eps n (|K|_max |alpha|_max + |r|_max)
plus forward errors against LAPACK where the matrix is well conditioned.
"""

import ctypes

import pytest
import torch

from dkg_amd import _lib
from dkg_amd.errors import NotPSDError
from dkg_amd.gp_state import _base_struct, _pad16
from dkg_amd.model import SingleTaskGPState
from oracle.gp import OutputGP, psd_safe_cholesky

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
EPS = torch.finfo(torch.double).eps


def run_prepare(st: SingleTaskGPState, max_tries: int = 3):
    lib = _lib.load()
    n, d = st.train_x.shape
    X = st.train_x.to(DEV).contiguous()
    inv_ls = (1.0 / st.lengthscale).to(DEV).contiguous()
    o = _base_struct(st, inv_ls, X)
    y = st.train_y.to(DEV).contiguous()
    L = torch.empty(n, n, dtype=torch.double, device=DEV)
    work = torch.empty(lib.dkg_prepare_workspace(n), dtype=torch.uint8, device=DEV)
    alpha = torch.empty(_pad16(n), dtype=torch.double, device=DEV)
    root = torch.empty(lib.dkg_frag_elems(n, n), dtype=torch.double, device=DEV)
    jit = ctypes.c_double(-1.0)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    _lib.check(lib.dkg_prepare_output(o, d, _lib.ptr(y), max_tries, _lib.ptr(L), _lib.ptr(work), work.numel(),
                                      _lib.ptr(alpha), _lib.ptr(root), ctypes.byref(jit), stream),
               "dkg_prepare_output")
    torch.cuda.synchronize()
    linv = work[: n * n * 8].view(torch.double).reshape(n, n).cpu()
    return L.cpu(), linv, alpha.cpu(), root.cpu(), jit.value


def problem(n, d=2, ls=0.3, s=1.0, noise=1e-4, seed=0, c=0.25):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, d, generator=g, dtype=torch.double)
    y = torch.randn(n, generator=g, dtype=torch.double)
    return SingleTaskGPState(X, y, ls, s, noise, c)


def host_K(st):
    og = OutputGP(st.train_x, st.train_y, st.lengthscale, st.outputscale, st.noise, st.mean_constant)
    K = og.covar(st.train_x, st.train_x)
    return K + st.noise * torch.eye(K.shape[0], dtype=torch.double)


def check_backward_errors(st, L, linv, alpha, jit=0.0):
    n = st.num_train
    K = host_K(st) + jit * torch.eye(n, dtype=torch.double)
    scale = 64 * EPS * n
    assert torch.equal(L.triu(1), torch.zeros_like(L))
    assert (L @ L.T - K).abs().max() <= scale * K.abs().max()
    assert (L @ linv - torch.eye(n, dtype=torch.double)).abs().max() <= scale * L.abs().max() * linv.abs().max()
    r = st.train_y - st.mean_constant
    res = (K @ alpha[:n] - r).abs().max()
    assert res <= scale * (K.abs().max() * alpha[:n].abs().max() + r.abs().max())
    assert torch.equal(alpha[n:], torch.zeros(_pad16(n) - n, dtype=torch.double))
    return K


@pytest.mark.parametrize("n", [1, 5, 16, 31, 32, 33, 64, 100, 256, 300, 1000])
def test_prepare_matches_lapack(n):
    st = problem(n, noise=1e-2)
    L, linv, alpha, root, jit = run_prepare(st)
    assert jit == 0.0
    K = check_backward_errors(st, L, linv, alpha)
    # forward errors vs LAPACK (well conditioned: noise 1e-2)
    L_ref = torch.linalg.cholesky(K)
    torch.testing.assert_close(L, L_ref, rtol=1e-10, atol=1e-11 * L_ref.abs().max().item())
    r = st.train_y - st.mean_constant
    a_ref = torch.cholesky_solve(r.unsqueeze(-1), L_ref).squeeze(-1)
    torch.testing.assert_close(alpha[:n], a_ref, rtol=1e-8, atol=1e-9 * a_ref.abs().max().item())


@pytest.mark.parametrize("kernel,nu", [("matern", 0.5), ("matern", 1.5), ("rbf", None)])
def test_prepare_other_kernels(kernel, nu):
    g = torch.Generator().manual_seed(5)
    X = torch.rand(70, 3, generator=g, dtype=torch.double)
    st = SingleTaskGPState(X, torch.randn(70, generator=g, dtype=torch.double), [0.3, 0.5, 0.9], 2.0, 1e-3, -0.4,
                           kernel, 2.5 if nu is None else nu)
    L, linv, alpha, _, jit = run_prepare(st)
    og = OutputGP(st.train_x, st.train_y, st.lengthscale, st.outputscale, st.noise, st.mean_constant, kernel,
                  2.5 if nu is None else nu)
    K = og.covar(X, X) + st.noise * torch.eye(70, dtype=torch.double)
    assert (L @ L.T - K).abs().max() <= 64 * EPS * 70 * K.abs().max()
    assert jit == 0.0


def test_prepare_ill_conditioned_headline_state():
    """The headline GP (l = 1.8, s = 50, noise 1e-4, n = 256): backward errors hold."""
    from dkg_amd.synthetic import WORKLOADS, make_problem

    model, _, _, _ = make_problem(WORKLOADS["headline"])
    for st in model.models:
        L, linv, alpha, _, jit = run_prepare(st)
        check_backward_errors(st, L, linv, alpha, jit)


def test_root_frag_matches_pack_root():
    """root_frag from L^{-1} equals dkg_pack_root of R = L^{-T} (the layout the kernels read)."""
    lib = _lib.load()
    st = problem(50, noise=1e-3)
    L, linv, _, root, _ = run_prepare(st)
    R = linv.T.contiguous().to(DEV)
    ref = torch.empty(lib.dkg_frag_elems(50, 50), dtype=torch.double, device=DEV)
    _lib.check(lib.dkg_pack_root(_lib.ptr(R), 50, _lib.ptr(ref), torch.cuda.current_stream(DEV).cuda_stream),
               "dkg_pack_root")
    torch.cuda.synchronize()
    assert torch.equal(root, ref.cpu())


def test_jitter_retry_follows_psd_safe_cholesky():
    """Duplicated inputs with a slightly negative diagonal shift: the plain
    factorisation fails and the first jitter (1e-8) repairs it, as
    linear_operator's psd_safe_cholesky (oracle restatement) does."""
    X = torch.rand(12, 2, generator=torch.Generator().manual_seed(3), dtype=torch.double)
    X = torch.cat([X, X[:4]])
    st = SingleTaskGPState(X, torch.randn(16, dtype=torch.double), 0.5, 1.0, -5e-9, 0.0)
    L, linv, alpha, _, jit = run_prepare(st)
    K = host_K(st)
    _, info = torch.linalg.cholesky_ex(K)
    assert int(info) != 0  # the plain factorisation fails on the host too
    L_ref = psd_safe_cholesky(K)
    assert jit == pytest.approx(1e-8)
    Kj = K + jit * torch.eye(16, dtype=torch.double)
    assert (L @ L.T - Kj).abs().max() <= 64 * EPS * 16 * K.abs().max()
    assert (L_ref @ L_ref.T - Kj).abs().max() <= 64 * EPS * 16 * K.abs().max()


def test_not_positive_definite_raises():
    with pytest.raises(NotPSDError, match="not positive definite"):
        run_prepare(problem(20, noise=-1.0))
    # duplicated inputs: K has a zero eigenvalue, so a -1e-9 shift is indefinite;
    # with max_tries = 0 there is no jitter retry
    X = torch.rand(8, 2, generator=torch.Generator().manual_seed(9), dtype=torch.double)
    st = SingleTaskGPState(torch.cat([X, X[:2]]), torch.randn(10, dtype=torch.double), 0.5, 1.0, -1e-9, 0.0)
    with pytest.raises(NotPSDError):
        run_prepare(st, max_tries=0)
    assert run_prepare(st, max_tries=1)[4] == pytest.approx(1e-8)


def test_prepare_outputs_batched_matches_one_by_one():
    """dkg_prepare_outputs (every output's factorisation in one chain, one status check, jitter retries per
    failing output) gives each output's dkg_prepare_output results bit for bit: outputs of different n, a
    kernel family each, one of them needing the first jitter retry."""
    from dkg_amd.gp_state import prepare_outputs

    g = torch.Generator().manual_seed(11)
    X0 = torch.rand(37, 2, generator=g, dtype=torch.double)
    Xj = torch.rand(12, 2, generator=g, dtype=torch.double)
    Xj = torch.cat([Xj, Xj[:4]])  # duplicated inputs with a slightly negative shift: needs jitter
    X2 = torch.rand(70, 2, generator=g, dtype=torch.double)
    states = [SingleTaskGPState(X0, torch.randn(37, generator=g, dtype=torch.double), [0.3, 0.5], 2.0, 1e-3, 0.1,
                                "matern", 2.5),
              SingleTaskGPState(Xj, torch.randn(16, generator=g, dtype=torch.double), 0.5, 1.0, -5e-9, 0.0),
              SingleTaskGPState(X2, torch.randn(70, generator=g, dtype=torch.double), [0.2, 0.9], 0.7, 1e-4, -0.3,
                                "rbf")]
    D = torch.rand(50, 2, generator=g, dtype=torch.double).to(DEV)
    together = prepare_outputs(states, D)
    for st, got in zip(states, together):
        (alone,) = prepare_outputs([st], D)
        assert got.jitter == alone.jitter
        for name in ("L", "alpha", "root_frag", "disc_frag", "disc_mean"):
            assert torch.equal(getattr(got, name), getattr(alone, name)), name
    assert together[1].jitter == pytest.approx(1e-8) and together[0].jitter == 0.0 and together[2].jitter == 0.0
