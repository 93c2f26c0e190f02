"""ORACLE (test infrastructure only) — restatement of the reference KG path.

Restates ``src/decoupledbo/modules/acquisition/discretekg.py`` (reference
snapshot 2025-08-24) on top of the posterior restatement in ``oracle/gp.py``.
Structure is deliberately faithful (per-candidate Python loop, full (N+1)^2
posterior covariance, per-scalarisation loop, the sort + argmin-walk epigraph)
so that it doubles as the timed CPU baseline of ``bench.py``.

Each function cites the reference lines it follows.
"""

from __future__ import annotations

import math

import torch
from torch import Tensor

from .gp import DTYPE, ModelList


class BotorchTensorDimensionError(Exception):
    """Stand-in for ``botorch.exceptions.BotorchTensorDimensionError``."""


class UnsupportedError(Exception):
    """Stand-in for ``botorch.exceptions.UnsupportedError``."""


# ---------------------------------------------------------------------------
# discretekg.py:455-470
def _check_lines(intercepts: Tensor, slopes: Tensor) -> None:
    if intercepts.dim() != 1 or slopes.dim() != 1:
        raise BotorchTensorDimensionError(
            f"Expected 'intercepts' and 'slopes' to both be one-dimensional tensors. "
            f"Got {intercepts.dim()=} and {slopes.dim()=}."
        )
    if intercepts.shape != slopes.shape:
        raise BotorchTensorDimensionError(
            f"Expected 'intercepts' and 'slopes' to have the same shape. "
            f"Got {intercepts.shape=} and {slopes.shape=}."
        )
    if intercepts.shape[-1] == 0:
        raise ValueError(
            f"Expected inputs to specify at least one line. "
            f"Got {intercepts.shape[-1]=}."
        )


# ---------------------------------------------------------------------------
# discretekg.py:341-412
def calculate_epigraph_indices(intercepts: Tensor, slopes: Tensor):
    """Upper envelope of the lines ``a_k + b_k z`` (reference algorithm).

    Short-circuit when every |b| < 1e-9 (:363-367); otherwise order the lines
    by slope ascending, ties broken by intercept descending (:370-374; both
    sorts are taken stable here, matching CPU torch on the KATs), then walk
    from the first line, each step jumping to the later line with a different
    slope whose intersection comes first (:382-401).
    Returns (indices into the inputs, left-to-right; intersection abscissae).
    """
    _check_lines(intercepts, slopes)
    if bool(torch.all(slopes.abs() < 1e-9)):
        top = torch.argmax(intercepts).reshape(1)
        return top, torch.tensor([], dtype=torch.double)

    by_a = torch.sort(intercepts, descending=True, stable=True).indices
    by_b = torch.sort(slopes[by_a], stable=True).indices
    perm = by_a[by_b]
    a = intercepts[perm]
    b = slopes[perm]

    n = a.shape[0]
    walk = [0]
    cuts = []
    cur = 0
    while cur < n - 1:
        later = torch.arange(cur + 1, n)
        keep = later[b[cur] != b[cur + 1:]]
        if keep.numel() == 0:
            break
        x = (a[keep] - a[cur]) / (b[cur] - b[keep])
        pick = int(torch.argmin(x))
        cur = int(keep[pick])
        walk.append(cur)
        cuts.append(x[pick])

    idx = perm[torch.tensor(walk, dtype=torch.long)]
    if cuts:
        return idx, torch.stack(cuts)
    return idx, torch.tensor([], dtype=torch.double)


# ---------------------------------------------------------------------------
# discretekg.py:415-452
def calculate_expected_value_of_piecewise_linear_function(intercepts: Tensor, slopes: Tensor,
                                                          boundaries: Tensor) -> Tensor:
    """E[f(Z)], Z ~ N(0,1), f piecewise linear: sum_j a_j dPhi_j - b_j dphi_j."""
    _check_lines(intercepts, slopes)
    if boundaries.shape != (len(intercepts) - 1,):
        raise BotorchTensorDimensionError(
            f"Expected 'boundaries' to be a one-dimensional tensor with "
            f"{len(intercepts)} elements. Got {boundaries.shape=}."
        )
    inf = torch.tensor([math.inf], dtype=boundaries.dtype)
    z = torch.cat([-inf, boundaries, inf])
    std_normal = torch.distributions.Normal(torch.zeros((), dtype=z.dtype), torch.ones((), dtype=z.dtype))
    pdf = torch.exp(std_normal.log_prob(z))
    cdf = std_normal.cdf(z)
    return torch.sum(intercepts * (cdf[1:] - cdf[:-1]) - slopes * (pdf[1:] - pdf[:-1]))


def _check_weights(w: Tensor) -> None:
    if w.dim() != 2:
        raise BotorchTensorDimensionError(
            "Expected 'scalarisation_weights' to have two dimensions: The first "
            "indexing different scalarisations to be averaged over and the second "
            "indexing coordinates of the objective space."
        )


def _kg_from_lines(intercepts: Tensor, slopes: Tensor) -> Tensor:
    idx, cuts = calculate_epigraph_indices(intercepts, slopes)
    e = calculate_expected_value_of_piecewise_linear_function(intercepts[idx], slopes[idx], cuts)
    return e - torch.max(intercepts)


# ---------------------------------------------------------------------------
# Candidates on discretisation points.  The reference evaluates one joint posterior over [x; D]
# (discretekg.py:182-184, 275-281): at x = z_k rows 0 and k + 1 of its covariance, and entries 0 and
# k + 1 of its mean, are the same numbers in exact arithmetic, and identical bits whenever the BLAS
# computes equal input rows identically (it does on this container's CPU; the GPU box's CPU BLAS was
# seen not to, for one of nine grid points, profiles/r04/dup_probe.txt).  Line 0 and line k + 1 are then
# exact copies: the walk takes line 0 (the lowest index among copies, :370-401) and torch.max splits the
# gradient of max a between them (:225-233).  The restatement fixes that reading independently of BLAS
# rounding: line 0 takes line k + 1's values (k the lowest coincident index) and keeps its own gradient.
def coincident_index(xnew: Tensor, discretisation: Tensor):
    """The lowest k with discretisation[k] == xnew exactly, or None."""
    if discretisation.shape[0] == 0:
        return None
    hit = (discretisation == xnew.detach()).all(-1).nonzero()
    return int(hit[0]) if hit.numel() else None


def copy_row(v: Tensor, k: int) -> Tensor:
    """v with entry 0 given entry k's value (its own gradient kept)."""
    return torch.cat([(v[0] + (v[k] - v[0]).detach()).unsqueeze(0), v[1:]])


# ---------------------------------------------------------------------------
# discretekg.py:162-235
def calculate_discrete_kg(model: ModelList, xnew: Tensor, discretisation: Tensor,
                          scalarisation_weights: Tensor) -> Tensor:
    """Full-evaluation discrete KG at one candidate (coupled observation)."""
    _check_weights(scalarisation_weights)
    Xt = torch.cat([xnew.unsqueeze(0), discretisation])
    post = model.posterior_list(Xt, observation_noise=False)            # :182-184
    post_noisy = model.posterior_list(xnew.unsqueeze(0), observation_noise=True)  # :185
    kc = coincident_index(xnew, discretisation)
    if kc is not None:  # line 0 an exact copy of line kc + 1 (see coincident_index)
        post = [(copy_row(p[0], kc + 1), torch.cat([copy_row(p[1][0], kc + 1)[None], p[1][1:]])) for p in post]
    means = torch.stack([p[0] for p in post], dim=-1)                    # (N+1) x m
    S = scalarisation_weights.shape[0]
    kg = torch.zeros(S, dtype=scalarisation_weights.dtype)
    for j in range(S):                                                   # :200
        w = scalarisation_weights[j]
        # ScalarizedPosteriorTransform on independent outputs: mean @ w,
        # covariance sum_i w_i^2 Cov_i (botorch scalarize_posterior).
        mean = means @ w                                                 # :211
        cov_row0 = sum(w[i] ** 2 * post[i][1][0] for i in range(len(post)))  # :212
        var_noisy = sum(w[i] ** 2 * post_noisy[i][1][0, 0] for i in range(len(post)))  # :213
        slopes = cov_row0 / var_noisy.sqrt()                             # :223
        kg[j] = _kg_from_lines(mean, slopes)                             # :225-233
    return kg.mean()                                                     # :235


# ---------------------------------------------------------------------------
# discretekg.py:238-338
def calculate_discrete_kg_conditioning_on_single_output(model: ModelList, xnew: Tensor, obj_idx_new: int,
                                                        discretisation: Tensor,
                                                        scalarisation_weights: Tensor) -> Tensor:
    """Decoupled discrete KG: only output ``obj_idx_new`` is observed at xnew."""
    _check_weights(scalarisation_weights)
    if not isinstance(model, ModelList):
        raise UnsupportedError(f"Input 'model' must be a 'ModelListGP'. Got {type(model)=}.")
    Xt = torch.cat([xnew.unsqueeze(0), discretisation])
    post = [m.posterior(Xt, observation_noise=False) for m in model.models]           # :275-281
    post_noisy = [m.posterior(xnew.unsqueeze(0), observation_noise=True) for m in model.models]  # :282-284
    kc = coincident_index(xnew, discretisation)
    if kc is not None:  # line 0 an exact copy of line kc + 1 (see coincident_index)
        post = [(copy_row(p[0], kc + 1), torch.cat([copy_row(p[1][0], kc + 1)[None], p[1][1:]])) for p in post]
    means = torch.stack([p[0] for p in post], dim=-1)                    # :300
    cov_i = post[obj_idx_new][1][0]                                      # :301
    var_i = post_noisy[obj_idx_new][1][0, 0]                             # :302
    znew = cov_i / var_i.sqrt()                                          # :313
    m = scalarisation_weights.shape[-1]
    weights = scalarisation_weights.view(-1, 1, m)
    intercepts = torch.sum(weights * means, dim=-1)                      # :320
    slopes = weights[..., obj_idx_new] * znew                            # :321
    S = scalarisation_weights.shape[0]
    kg = torch.zeros(S, dtype=scalarisation_weights.dtype)
    for j in range(S):                                                   # :329-336
        kg[j] = _kg_from_lines(intercepts[j], slopes[j])
    return kg.mean()                                                     # :338


# ---------------------------------------------------------------------------
# discretekg.py:62-123, 131-159
def check_init(model: ModelList, x_discretisation: Tensor, scalarisation_weights=None):
    """Validation of ``DiscreteKnowledgeGradient.__init__`` (:92-119)."""
    if x_discretisation.dim() != 2:
        raise BotorchTensorDimensionError(
            f"Expected 'x_discretisation' to have two dimensions. Got {x_discretisation.dim()=}."
        )
    if scalarisation_weights is None:
        if model.num_outputs != 1:
            raise UnsupportedError("Models with more than one output must specify 'scalarisation_weights'.")
        scalarisation_weights = torch.tensor([[1.0]], dtype=x_discretisation.dtype)
    if scalarisation_weights.dim() != 2:
        raise BotorchTensorDimensionError("Expected 'scalarisation_weights' to have two dimensions")
    if scalarisation_weights.shape[-1] != model.num_outputs:
        raise BotorchTensorDimensionError("Expected the last dimension of 'scalarisation_weights' to "
                                          "have one element per objective.")
    return scalarisation_weights


def discrete_kg_forward(model: ModelList, X: Tensor, x_discretisation: Tensor,
                        scalarisation_weights=None, target_output_ix=None) -> Tensor:
    """``DiscreteKnowledgeGradient.forward`` (:131-159): X [*batch, 1, d] -> [*batch]."""
    W = check_init(model, x_discretisation, scalarisation_weights)
    if X.dim() < 2:
        raise ValueError("X must have at least 2 dimensions")
    if X.dim() == 2:
        X = X.unsqueeze(0)
    if X.shape[-2] != 1:
        raise AssertionError(f"Expected X to be `batch_shape x q=1 x d`, but got X with shape {X.shape}.")
    batch_shape, d = X.shape[:-2], X.shape[-1]
    if d != x_discretisation.shape[-1]:
        raise RuntimeError(
            f"Expected X to have last dimension matching 'self.x_discretisation'. "
            f"Got {X.shape[-1]=}, {x_discretisation.shape[-1]=}."
        )
    out = torch.zeros(batch_shape.numel(), dtype=X.dtype)
    for i, xnew in enumerate(X.reshape(-1, d)):
        if target_output_ix is not None:
            out[i] = calculate_discrete_kg_conditioning_on_single_output(
                model, xnew, target_output_ix, x_discretisation, W)
        else:
            out[i] = calculate_discrete_kg(model, xnew, x_discretisation, W)
    return out.reshape(batch_shape)


# ---------------------------------------------------------------------------
# Vectorised restatement of the same lines (tests at larger sizes).  Same
# formulas as above; the posterior rows are computed for all candidates at
# once instead of materialising the (N+1)^2 covariance per candidate.
def lines_batched(model: ModelList, X: Tensor, D: Tensor, W: Tensor, target=None):
    """Intercepts/slopes for every (candidate, scalarisation): a, b of shape [B, S, N+1]."""
    B = X.shape[0]
    mus, covs, var_noisy = [], [], []
    for om in model.models:
        c = om.cache()
        n = om.train_x.shape[0]
        Kx = om.covar(X, torch.cat([om.train_x, X], 0))[:, :n]          # B x n
        Kd = om.covar(D, torch.cat([om.train_x, D], 0))[:, :n]          # N x n
        Qx = Kx @ c["R"]
        Qd = Kd @ c["R"]
        mu_x = Kx @ c["alpha"] + om.mean_constant
        mu_d = Kd @ c["alpha"] + om.mean_constant
        kxd = om.covar(X, D)                                            # B x N
        v = om.outputscale - (Qx * Qx).sum(-1)                          # B
        cov = torch.cat([v[:, None], kxd - Qx @ Qd.mT], dim=1)         # B x (N+1)
        mu = torch.cat([mu_x[:, None], mu_d[None, :].expand(B, -1)], dim=1)
        mus.append(mu * om.y_std + om.y_mean)
        covs.append(cov * om.y_std**2)
        var_noisy.append((v + om.noise) * om.y_std**2)
    mus = torch.stack(mus, -1)           # B x (N+1) x m
    covs = torch.stack(covs, -1)         # B x (N+1) x m
    for bi in range(B):  # candidates on discretisation points: line 0 a copy of line k + 1 (coincident_index)
        kc = coincident_index(X[bi], D)
        if kc is not None:
            mus = torch.cat([mus[:bi], copy_row(mus[bi], kc + 1)[None], mus[bi + 1:]])
            covs = torch.cat([covs[:bi], copy_row(covs[bi], kc + 1)[None], covs[bi + 1:]])
    var_noisy = torch.stack(var_noisy, -1)  # B x m
    a = torch.einsum("bkm,sm->bsk", mus, W)
    if target is None:
        num = torch.einsum("bkm,sm->bsk", covs, W**2)
        den = torch.einsum("bm,sm->bs", var_noisy, W**2).sqrt()
        b = num / den[..., None]
    else:
        zc = covs[..., target] / var_noisy[:, target, None].sqrt()     # B x (N+1)
        b = W[None, :, target, None] * zc[:, None, :]
    return a, b


def kg_pairs_from_lines(a: Tensor, b: Tensor) -> Tensor:
    """KG per (candidate, scalarisation) with the reference epigraph/expectation."""
    B, S, _ = a.shape
    out = torch.zeros(B, S, dtype=a.dtype)
    for i in range(B):
        for j in range(S):
            out[i, j] = _kg_from_lines(a[i, j], b[i, j])
    return out


def discrete_kg_batched(model: ModelList, X: Tensor, D: Tensor, W: Tensor, target=None):
    """Vectorised oracle forward: returns (kg[B], kg_pairs[B,S])."""
    a, b = lines_batched(model, X, D, W, target)
    pairs = kg_pairs_from_lines(a, b)
    return pairs.mean(-1), pairs
