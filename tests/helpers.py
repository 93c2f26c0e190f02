"""Shared test helpers: product <-> oracle model conversion and the parity tolerance."""

import torch

from oracle.gp import ModelList, OutputGP

EPS = torch.finfo(torch.double).eps


def to_oracle(state) -> ModelList:
    """dkg_amd ModelListGPState -> oracle ModelList (same fitted state)."""
    return ModelList([OutputGP(m.train_x, m.train_y, m.lengthscale, m.outputscale, m.noise, m.mean_constant,
                               m.kernel, m.nu, m.y_mean, m.y_std) for m in state.models])


def to_state(oracle_model):
    from dkg_amd.model import ModelListGPState, SingleTaskGPState

    return ModelListGPState(*[SingleTaskGPState(o.train_x, o.train_y, o.lengthscale.reshape(-1), o.outputscale,
                                                o.noise, o.mean_constant, o.kernel, o.nu, o.y_mean, o.y_std)
                              for o in oracle_model.models])


def rounding_floor(om: ModelList, X: torch.Tensor, D: torch.Tensor, W: torch.Tensor, target=None,
                   c: float = 64.0) -> torch.Tensor:
    """Absolute fp64 floor of the parity tolerance, per candidate [B].

    Two fp64 implementations of the same KG differ by their rounding errors,
    whose standard bound is ~ n*eps times the *absolute* sums behind each
    quantity: KG = E[max] - max(a) cancels at |a| (discretekg.py:233), the
    posterior mean c + K alpha cancels at sum_l |k_l alpha_l|, and the
    covariance k - q.Q_D at sum_l |q_l| |Q_D,kl|.  The floor is
    c * eps * (max|a| + n * (sum_i |w_i| sd_i sum_l |k_l alpha_l|
                            + max_k sum_i |beta_i| sd_i^2 sum_l |q_l||Q_D,kl|)),
    taken over scalarisations (DESIGN.md "Parity tolerance").
    """
    B = X.shape[0]
    mag_a = torch.zeros(B, dtype=torch.double)
    mag_mu = torch.zeros(B, dtype=torch.double)
    mag_cov = torch.zeros(B, dtype=torch.double)
    for i, o in enumerate(om.models):
        cch = o.cache()
        n = o.train_x.shape[0]
        Kx = o.covar(X, o.train_x)
        Kd = o.covar(D, o.train_x)
        Qx = (Kx @ cch["R"]).abs()
        Qd = (Kd @ cch["R"]).abs()
        muabs = (Kx.abs() @ cch["alpha"].abs()) * n
        covabs = (Qx @ Qd.mT).max(dim=1).values * n
        mu_d = (Kd @ cch["alpha"] + o.mean_constant) * o.y_std + o.y_mean
        w = W[:, i].abs().max()
        mag_a += w * (mu_d.abs().max() + (Kx @ cch["alpha"]).abs() * o.y_std + abs(o.y_mean))
        mag_mu += w * o.y_std * muabs
        if target is None or target == i:
            v = o.outputscale - (Kx @ cch["R"]).pow(2).sum(-1)
            beta = o.y_std / torch.sqrt(o.y_std**2 * (v + o.noise)).clamp_min(1e-300)
            mag_cov += w * o.y_std * beta * covabs
    return c * EPS * (mag_a + mag_mu + mag_cov)


def assert_kg_close(got: torch.Tensor, ref: torch.Tensor, floor: torch.Tensor, rtol: float = 1e-6):
    got = got.detach().cpu().double().reshape(-1)
    ref = ref.detach().cpu().double().reshape(-1)
    floor = floor.reshape(-1)
    tol = rtol * ref.abs() + floor
    err = (got - ref).abs()
    bad = err > tol
    assert not bool(bad.any()), (
        f"{int(bad.sum())}/{bad.numel()} KG values outside rtol={rtol}+floor: "
        f"max err/tol={float((err / tol).max()):.3g}; worst got={got[bad][:4].tolist()} ref={ref[bad][:4].tolist()}")
    return float((err / tol).max())


def load_golden(name: str):
    """tests/golden/<name>.npz -> (state, oracle ModelList, D, W, X, arrays dict)."""
    import os

    import numpy as np

    from dkg_amd.model import ModelListGPState, SingleTaskGPState

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{name}.npz")
    z = dict(np.load(path))
    t = {k: torch.from_numpy(v) for k, v in z.items()}
    state = ModelListGPState(*[
        SingleTaskGPState(t["train_x"], t["train_y"][:, i], t["lengthscale"][i], float(t["outputscale"][i]),
                          float(t["noise"][i]), float(t["mean_constant"][i]))
        for i in range(t["train_y"].shape[1])])
    return state, to_oracle(state), t["D"], t["W"], t["X"], t
