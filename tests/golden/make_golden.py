"""Generate tests/golden/*.npz: fixed-state Discrete-KG golden vectors.

Inputs come from the reference's own GP-problem fixtures
(``/root/reference/data/shared/gp-problem/{lengthscales,observationnoise}/0.pt``,
format of ``src/decoupledbo/pipeline/data_catalog.py:99-111``), loaded with
``torch.load(weights_only=True)``; raw GPyTorch parameters go through the
constraint transforms (``oracle.gp.model_list_from_state_dict``).  The noise is
floored at 1e-4 (the reference's MIN_NOISE_SE**2, ``model/factory.py:15``),
because 1e-8 leaves K(X,X) numerically singular for lengthscale 1.8.

Expected outputs are the oracle restatement's (BoTorch/GPyTorch are not
importable here): the structure-faithful per-candidate path
(``calculate_discrete_kg`` / ``..._conditioning_on_single_output``) for every
candidate and scalarisation.  Run from the repo root:
    python tests/golden/make_golden.py
The .npz files are data (inputs and expected outputs); the GPU tests read them
without /root/reference.
"""

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]

from dkg_amd.utils import make_torch_std_grid, sample_simplex  # noqa: E402
from oracle.discretekg import (calculate_discrete_kg,  # noqa: E402
                               calculate_discrete_kg_conditioning_on_single_output, lines_batched)
from oracle.gp import ModelList, OutputGP, model_list_from_state_dict  # noqa: E402

REF = "/root/reference/data/shared/gp-problem"
PROBLEMS = {"lengthscales0": "lengthscales/0.pt", "observationnoise0": "observationnoise/0.pt"}
NOISE_FLOOR = 1e-4


def build(name, rel):
    torch.set_default_dtype(torch.double)
    blob = torch.load(os.path.join(REF, rel), weights_only=True)
    tx, ty = blob["train_x"].double(), blob["train_y"].double()
    ml = model_list_from_state_dict(blob["model_state_dict"], tx, ty)
    om = ModelList([OutputGP(m.train_x, m.train_y, m.lengthscale, m.outputscale, max(m.noise, NOISE_FLOOR),
                             m.mean_constant, m.kernel, m.nu) for m in ml.models])
    m, d = len(om.models), tx.shape[1]
    D = make_torch_std_grid(16, d, {"dtype": torch.double})
    W = sample_simplex(m, 8, qmc=True, seed=21)
    X = torch.quasirandom.SobolEngine(d, scramble=True, seed=22).draw(24, dtype=torch.double)
    out = {
        "train_x": tx.numpy(), "train_y": ty.numpy(),
        "lengthscale": torch.stack([mm.lengthscale.reshape(-1) for mm in om.models]).numpy(),
        "outputscale": np.array([mm.outputscale for mm in om.models]),
        "noise": np.array([mm.noise for mm in om.models]),
        "mean_constant": np.array([mm.mean_constant for mm in om.models]),
        "D": D.numpy(), "W": W.numpy(), "X": X.numpy(),
    }
    for key, target in (("full", None), ("t0", 0), ("t1", 1)):
        kg = []
        for x in X:
            if target is None:
                kg.append(float(calculate_discrete_kg(om, x, D, W)))
            else:
                kg.append(float(calculate_discrete_kg_conditioning_on_single_output(om, x, target, D, W)))
        out[f"kg_{key}"] = np.array(kg)
    a, b = lines_batched(om, X[:4], D, W, None)   # lines of the first 4 candidates, full path: [4, S, N+1]
    out["lines_a"], out["lines_b"] = a.numpy(), b.numpy()
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, "kg_full", out["kg_full"][:4], "max", out["kg_full"].max())


if __name__ == "__main__":
    for n, r in PROBLEMS.items():
        build(n, r)
