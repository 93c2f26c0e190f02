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

sys.path.insert(0, os.path.join(REPO, "tests"))
from helpers import to_oracle  # noqa: E402

base = WORKLOADS["stress32"]
variants = {
    "small": WORKLOADS["small"],
    "parity6d": WORKLOADS["parity6d"],
    "headline": WORKLOADS["headline"],
    "headline_nd": WORKLOADS["headline_nd"],
    "stress32 (l=.2/1.8/.6, noise 1e-3 s)": base,
    "noise 1e-2 s": dataclasses.replace(base, noise_rel=1e-2),
    "l=.2/.5/.3, noise 1e-3 s": dataclasses.replace(base, lengthscales=(0.2, 0.5, 0.3)),
    "l=.2/.5/.3, noise 1e-2 s": dataclasses.replace(base, lengthscales=(0.2, 0.5, 0.3), noise_rel=1e-2),
}
for name, w in variants.items():
    model, D, X, W = make_problem(w)
    Xd = X[:128].cuda().unsqueeze(-2)
    # cancellation factor of the posterior: prior variance s over the smallest noiseless posterior variance
    # at the candidates (cov = s k - Q_X . Q_D loses that factor of relative precision)
    canc = []
    for o in to_oracle(model).models:
        q = o.covar(X[:128], o.train_x) @ o.cache()["R"]
        v = o.outputscale - (q * q).sum(-1)
        canc.append(float(o.outputscale / v.clamp_min(1e-300).min()))
    print(f"{name}: cancellation s / min var at the candidates per output: " + ", ".join(f"{c:.3g}" for c in canc))
    for target in (None, 0, 1):
        k64 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)(Xd).cpu()
        k32 = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, precision="fp32")(Xd).cpu()
        keep = k64.abs() >= 1e-3 * k64.abs().max()
        rel = ((k32 - k64).abs() / k64.abs())[keep]
        print(f"{name:32s} target={target}: {int(keep.sum())} candidates, max KG {float(k64.max()):.3e}, "
              f"rel median {float(rel.median()):.2e} max {float(rel.max()):.2e}", flush=True)
