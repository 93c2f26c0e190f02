"""fp32-contraction plan (DKG_PLAN_F32) against the fp64 plan on stress-shaped GPs.

Run on the GPU box:  python tools/f32_check.py
Prints, per GP variant and path, the median and max relative difference over
the candidates whose KG is at least 1e-3 of the batch maximum.
"""
import dataclasses
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

base = WORKLOADS["stress32"]
variants = {
    "stress32 (l=.2/1.8/.6, noise 1e-3 s)": base,
    "noise 1e-2 s": dataclasses.replace(base, noise_rel=1e-2),
    "l=.2/.5/.3, noise 1e-3 s": dataclasses.replace(base, lengthscales=(0.2, 0.5, 0.3)),
    "l=.2/.5/.3, noise 1e-2 s": dataclasses.replace(base, lengthscales=(0.2, 0.5, 0.3), noise_rel=1e-2),
}
for name, w in variants.items():
    model, D, X, W = make_problem(w)
    Xd = X[:128].cuda().unsqueeze(-2)
    for target in (None, 0, 1):
        k64 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)(Xd).cpu()
        k32 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, precision="fp32")(Xd).cpu()
        keep = k64.abs() >= 1e-3 * k64.abs().max()
        rel = ((k32 - k64).abs() / k64.abs())[keep]
        print(f"{name:32s} target={target}: {int(keep.sum())} candidates, max KG {float(k64.max()):.3e}, "
              f"rel median {float(rel.median()):.2e} max {float(rel.max()):.2e}", flush=True)
