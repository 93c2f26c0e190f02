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
from typing import List, Sequence

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


def from_state_dict(state: dict, train_x: torch.Tensor, train_y: torch.Tensor,
                    kernel: str = "matern", nu: float = 2.5) -> ModelListGPState:
    """ModelListGP ``state_dict`` (raw GPyTorch parameters) + data -> state.

    Raw parameters go through GPyTorch's constraint transform (softplus +
    lower bound); ``raw_noise = -inf`` therefore maps to the noise lower bound.
    """
    sd = {k: torch.as_tensor(v, dtype=torch.double) for k, v in state.items()}
    outs = []
    i = 0
    sp = torch.nn.functional.softplus
    while f"models.{i}.covar_module.raw_outputscale" in sd:
        p = f"models.{i}."

        def cons(key):
            lb = sd.get(p + key + "_constraint.lower_bound", torch.tensor(0.0, dtype=torch.double))
            return sp(sd[p + key]) + lb

        outs.append(SingleTaskGPState(
            train_x=train_x, train_y=train_y[:, i],
            lengthscale=cons("covar_module.base_kernel.raw_lengthscale").reshape(-1),
            outputscale=float(cons("covar_module.raw_outputscale")),
            noise=float(cons("likelihood.noise_covar.raw_noise").reshape(-1)[0]),
            mean_constant=float(sd.get(p + "mean_module.raw_constant", torch.tensor(0.0))),
            kernel=kernel, nu=nu))
        i += 1
    return ModelListGPState(*outs)
