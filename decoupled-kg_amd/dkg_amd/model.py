"""GP model state consumed by the Discrete-KG path (host side, plain tensors).

Mirrors the model family the reference builds in
``src/decoupledbo/modules/model/factory.py:24-151``: a ModelListGP of
independent SingleTaskGPs, each ``ScaleKernel(Matern(nu) | RBF, ARD)`` with a
``ConstantMean``, a homoskedastic ``GaussianLikelihood`` and an optional
``Standardize(m=1)`` outcome transform.  The reference's KG reads the model
only through ``model.num_outputs``, ``model.models`` and ``posterior``
(``discretekg.py:99,114,182-185,270-284``); here the fitted state is read once
and handed to the device (``dkg_amd.gp_state``).

Three ways in:
  * construct ``SingleTaskGPState``/``ModelListGPState`` directly;
  * ``from_botorch(model)`` when BoTorch/GPyTorch are importable;
  * ``from_state_dict(...)`` for the reference's on-disk GP-problem format
    (``pipeline/data_catalog.py:99-111``).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import torch

KERNELS = {("matern", 0.5): 0, ("matern", 1.5): 1, ("matern", 2.5): 2, ("rbf", None): 3}


def kernel_id(kind: str, nu) -> int:
    key = (kind, None if kind == "rbf" else float(nu))
    if key not in KERNELS:
        raise ValueError(f"Unsupported kernel {kind!r} (nu={nu}); catalog is matern(0.5|1.5|2.5), rbf")
    return KERNELS[key]


@dataclass
class SingleTaskGPState:
    """Fitted hyperparameters + data of one output (model space targets)."""

    train_x: torch.Tensor
    train_y: torch.Tensor
    lengthscale: torch.Tensor
    outputscale: float
    noise: float
    mean_constant: float = 0.0
    kernel: str = "matern"
    nu: float = 2.5
    y_mean: float = 0.0
    y_std: float = 1.0

    def __post_init__(self):
        self.train_x = torch.as_tensor(self.train_x, dtype=torch.double).detach().cpu()
        self.train_y = torch.as_tensor(self.train_y, dtype=torch.double).detach().cpu().reshape(-1)
        d = self.train_x.shape[-1]
        ls = torch.as_tensor(self.lengthscale, dtype=torch.double).detach().cpu().reshape(-1)
        if ls.numel() == 1:
            ls = ls.repeat(d)
        if ls.numel() != d:
            raise ValueError(f"lengthscale has {ls.numel()} entries for d={d}")
        self.lengthscale = ls
        if self.train_x.dim() != 2 or self.train_x.shape[0] != self.train_y.shape[0]:
            raise ValueError("train_x must be n x d and train_y must have n entries")
        kernel_id(self.kernel, self.nu)

    @property
    def num_train(self) -> int:
        return self.train_x.shape[0]


@dataclass
class ModelListGPState:
    models: List[SingleTaskGPState]

    def __init__(self, *models: SingleTaskGPState):
        if len(models) == 1 and isinstance(models[0], (list, tuple)):
            models = tuple(models[0])
        self.models = list(models)
        dims = {m.train_x.shape[-1] for m in self.models}
        if len(dims) != 1:
            raise ValueError("all outputs must share the input dimension")

    @property
    def num_outputs(self) -> int:
        return len(self.models)

    @property
    def input_dim(self) -> int:
        return self.models[0].train_x.shape[-1]


def from_botorch(model) -> ModelListGPState:
    """Read the fitted state of a BoTorch ModelListGP / SingleTaskGP."""
    subs: Sequence = getattr(model, "models", None) or [model]
    outs = []
    for gp in subs:
        covar = gp.covar_module
        base = covar.base_kernel
        kind = "rbf" if type(base).__name__ == "RBFKernel" else "matern"
        nu = getattr(base, "nu", None)
        ot = getattr(gp, "outcome_transform", None)
        y_mean, y_std = 0.0, 1.0
        if ot is not None:
            y_mean = float(ot.means.reshape(-1)[0])
            y_std = float(ot.stdvs.reshape(-1)[0])
        outs.append(SingleTaskGPState(
            train_x=gp.train_inputs[0], train_y=gp.train_targets,
            lengthscale=base.lengthscale.reshape(-1), outputscale=float(covar.outputscale),
            noise=float(gp.likelihood.noise.reshape(-1)[0]), mean_constant=float(gp.mean_module.constant),
            kernel=kind, nu=nu, y_mean=y_mean, y_std=y_std))
    return ModelListGPState(*outs)


def _per_output(v, m: int, what: str) -> list:
    """A shared tensor, or one per output."""
    if isinstance(v, (list, tuple)):
        if len(v) != m:
            raise ValueError(f"{what}: {len(v)} entries for {m} outputs")
        return [torch.as_tensor(t, dtype=torch.double) for t in v]
    t = torch.as_tensor(v, dtype=torch.double)
    if what == "train_y":
        if t.dim() == 1 and m == 1:
            return [t]
        if t.dim() != 2 or t.shape[1] != m:
            raise ValueError(f"train_y must be n x {m} (or one tensor per output); got shape {tuple(t.shape)}")
        return [t[:, i] for i in range(m)]
    return [t] * m


def _constrained(sd: dict, key: str, enforced: bool = True) -> torch.Tensor:
    """A GPyTorch constrained parameter from its raw value: Interval(lb, ub) -> sigmoid, GreaterThan /
    Positive -> softplus + lb; ``enforced=False`` (a constraint built with ``transform=None``,
    factory.py:102-104 and BoTorch's default likelihood) -> the raw value itself."""
    if key not in sd:
        raise KeyError(f"state dict has no {key!r}")
    raw = sd[key]
    if not enforced:
        return raw
    lb = sd.get(key + "_constraint.lower_bound", torch.tensor(0.0, dtype=torch.double))
    ub = sd.get(key + "_constraint.upper_bound", torch.tensor(float("inf"), dtype=torch.double))
    if bool(torch.isfinite(ub).all()):
        return lb + (ub - lb) * torch.sigmoid(raw)
    return torch.nn.functional.softplus(raw) + lb


def from_state_dict(state: dict, train_x, train_y, kernel: str = "matern", nu: float = 2.5, bounds=None,
                    noise_constraint: str = "enforced") -> ModelListGPState:
    """ModelListGP ``state_dict`` (raw GPyTorch parameters and buffers) + training data -> state.

    * ``train_x``: [n, d] shared by every output, or one [n_i, d] tensor per output (decoupled BO
      keeps a training set per objective).  With ``bounds`` [2, d] the raw inputs are normalised
      as the reference does before building each GP (``factory.py:64``), else they must already be
      in [0, 1]^d.
    * ``train_y``: [n, m], or one [n_i] tensor per output, in the problem's units (what the reference
      hands to ``SingleTaskGP``).  If the state dict holds a ``Standardize(m=1)`` outcome transform
      (``models.i.outcome_transform.means`` / ``stdvs``, ``factory.py:75-76``) the targets are
      standardised with those buffers exactly as BoTorch did at construction, and the posterior is
      untransformed with them (``y_mean`` / ``y_std``).
    * Raw parameters go through GPyTorch's constraint transforms (softplus + lower bound, or sigmoid
      for a finite interval).  ``noise_constraint="raw"`` for likelihoods whose ``GreaterThan`` was
      built with ``transform=None`` (the BO loop's models, ``factory.py:102-104``): the noise is the
      raw value.  The GP-problem fixtures (``data/shared/gp-problem``) enforce it (``raw_noise = -inf``
      maps to the lower bound).
    * The constant mean is ``mean_module.raw_constant`` (GPyTorch >= 1.9) or ``mean_module.constant``;
      a missing mean raises ``KeyError``.
    """
    if noise_constraint not in ("enforced", "raw"):
        raise ValueError(f"noise_constraint must be 'enforced' or 'raw', got {noise_constraint!r}")
    sd = {k: torch.as_tensor(v, dtype=torch.double) for k, v in state.items()}
    m = 0
    while f"models.{m}.covar_module.raw_outputscale" in sd:
        m += 1
    if m == 0:
        raise KeyError("state dict has no 'models.0.covar_module.raw_outputscale': not a ModelListGP state dict")
    xs = _per_output(train_x, m, "train_x")
    ys = _per_output(train_y, m, "train_y")
    outs = []
    for i in range(m):
        p = f"models.{i}."
        x = xs[i]
        if bounds is not None:
            bnd = torch.as_tensor(bounds, dtype=torch.double)
            x = (x - bnd[0]) / (bnd[1] - bnd[0])
        if p + "mean_module.raw_constant" in sd:
            c = float(sd[p + "mean_module.raw_constant"].reshape(-1)[0])
        elif p + "mean_module.constant" in sd:
            c = float(sd[p + "mean_module.constant"].reshape(-1)[0])
        else:
            raise KeyError(f"state dict has no constant mean for output {i} "
                           f"({p}mean_module.raw_constant / {p}mean_module.constant)")
        y = ys[i].reshape(-1)
        y_mean, y_std = 0.0, 1.0
        if p + "outcome_transform.means" in sd:
            if p + "outcome_transform.stdvs" not in sd:
                raise KeyError(f"{p}outcome_transform.means without {p}outcome_transform.stdvs")
            y_mean = float(sd[p + "outcome_transform.means"].reshape(-1)[0])
            y_std = float(sd[p + "outcome_transform.stdvs"].reshape(-1)[0])
            y = (y - y_mean) / y_std                      # Standardize.forward (BoTorch)
        outs.append(SingleTaskGPState(
            train_x=x, train_y=y,
            lengthscale=_constrained(sd, p + "covar_module.base_kernel.raw_lengthscale").reshape(-1),
            outputscale=float(_constrained(sd, p + "covar_module.raw_outputscale")),
            noise=float(_constrained(sd, p + "likelihood.noise_covar.raw_noise",
                                     noise_constraint == "enforced").reshape(-1)[0]),
            mean_constant=c, kernel=kernel, nu=nu, y_mean=y_mean, y_std=y_std))
    return ModelListGPState(*outs)


def _inv_softplus(x: torch.Tensor) -> torch.Tensor:
    """GPyTorch's ``inv_softplus``: the raw value whose softplus is ``x`` (x > 0)."""
    return x + torch.log(-torch.expm1(-x))


# factory.py:15-20: the noise floor of a fitted / a fixed-hyperparameter ("never") surrogate
MIN_NOISE_SE = 1e-2
MIN_NOISE_SE_FIXED = 1e-4


def _prior_buffers(prior_cfg) -> Dict[str, float]:
    """The buffers of a prior the reference's config names (``factory.py:138-151``: only ``gamma``):
    gpytorch's ``GammaPrior`` registers ``concentration`` and ``rate``."""
    if prior_cfg is None:
        return {}
    if prior_cfg["type"] != "gamma":
        raise ValueError(f"Unsupported prior 'type'. Got {prior_cfg['type']!r}.")
    return {"concentration": float(prior_cfg["args"]["concentration"]), "rate": float(prior_cfg["args"]["rate"])}


def to_state_dict(model: ModelListGPState, model_config: Optional[dict] = None) -> Dict[str, torch.Tensor]:
    """The ``ModelListGP.state_dict()`` the reference checkpoints (``bo_loop.py:281-290``,
    ``data_catalog.py:317-348``) for a state built here, in the raw GPyTorch parametrisation that
    ``from_state_dict(..., noise_constraint="raw")`` reads back: ``Positive`` (softplus) lengthscales and
    outputscale, the BO loop's ``GreaterThan(min_noise_se**2, transform=None)`` noise (``factory.py:95-104``:
    raw = noise; lower bound ``MIN_NOISE_SE_FIXED**2`` on the ``never`` path, ``MIN_NOISE_SE**2`` otherwise,
    ``factory.py:41-43``), ``mean_module.raw_constant``, BoTorch's ``Standardize(m=1)`` buffers when the output
    is standardised, and the ``LikelihoodList`` copies ``likelihood.likelihoods.i.*`` every ``ModelListGP``
    holds (the keys of the reference's own ``data/shared/gp-problem`` state dicts, tests/golden/ref_schema.json).

    ``model_config`` (the reference's ``model`` config section, ``bo_smoke.reference_model_config``): the
    surrogate ``build_mll_and_model`` builds from it also carries its priors' buffers
    (``<module>.<name>_prior.concentration`` / ``.rate``, ``factory.py:91-151``); without it the never-path
    floor and no priors are assumed.  The prior buffer names follow gpytorch 1.11's ``GammaPrior``, which is
    not importable here: that part of the key set is unpinned.
    ``from_state_dict(to_state_dict(m), train_x, train_y_problem_units, ...)`` rebuilds ``m`` (hyperparameters
    to the last ulp of softplus∘inv_softplus)."""
    sd: Dict[str, torch.Tensor] = {}
    f64 = dict(dtype=torch.double)
    fit = (model_config or {}).get("fit_hyperparams", "never")
    floor = (MIN_NOISE_SE_FIXED if fit == "never" else MIN_NOISE_SE) ** 2
    outs_cfg = (model_config or {}).get("outputs") or [None] * model.num_outputs
    if len(outs_cfg) != model.num_outputs:
        raise ValueError(f"model_config has {len(outs_cfg)} outputs for a {model.num_outputs}-output model")
    lik_list: Dict[str, torch.Tensor] = {}
    for i, st in enumerate(model.models):
        p = f"models.{i}."
        cfg = outs_cfg[i] or {}
        lik = {"noise_covar.raw_noise": torch.tensor([st.noise], **f64),
               "noise_covar.raw_noise_constraint.lower_bound": torch.tensor(floor, **f64),
               "noise_covar.raw_noise_constraint.upper_bound": torch.tensor(float("inf"), **f64)}
        for k, v in _prior_buffers((cfg.get("likelihood") or {}).get("noise_prior")).items():
            lik["noise_covar.noise_prior." + k] = torch.tensor(v, **f64)
        for k, v in lik.items():
            sd[p + "likelihood." + k] = v
            lik_list[f"likelihood.likelihoods.{i}." + k] = v.clone()
        sd[p + "mean_module.raw_constant"] = torch.tensor(float(st.mean_constant), **f64)
        sd[p + "covar_module.raw_outputscale"] = _inv_softplus(torch.tensor(float(st.outputscale), **f64))
        sd[p + "covar_module.base_kernel.raw_lengthscale"] = _inv_softplus(
            torch.as_tensor(st.lengthscale, **f64).reshape(1, -1).clone())
        for k in ("covar_module.raw_outputscale_constraint", "covar_module.base_kernel.raw_lengthscale_constraint"):
            sd[p + k + ".lower_bound"] = torch.tensor(0.0, **f64)
            sd[p + k + ".upper_bound"] = torch.tensor(float("inf"), **f64)
        kcfg = cfg.get("kernel") or {}
        for name, mod in (("lengthscale_prior", "covar_module.base_kernel."), ("outputscale_prior", "covar_module.")):
            for k, v in _prior_buffers(kcfg.get(name)).items():
                sd[p + mod + name + "." + k] = torch.tensor(v, **f64)
        if st.y_mean != 0.0 or st.y_std != 1.0:
            sd[p + "outcome_transform.means"] = torch.tensor([[st.y_mean]], **f64)
            sd[p + "outcome_transform.stdvs"] = torch.tensor([[st.y_std]], **f64)
            sd[p + "outcome_transform._stdvs_sq"] = torch.tensor([[st.y_std ** 2]], **f64)
    sd.update(lik_list)
    return sd
