"""Histogram of the envelope's candidate count nc per (candidate, scalarisation) pair
(DKG_DEBUG_ENV_FLAGS=32 makes kg_pairs carry nc).  GPU box, repo root."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
os.environ["DKG_DEBUG_ENV_FLAGS"] = "32"
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

for name in sys.argv[1:] or ["headline"]:
    w = WORKLOADS[name]
    model, D, X, W = make_problem(w)
    for target in (None, 0):
        acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)
        nc = acq.forward_pairs(X.unsqueeze(-2)).cpu().numpy().ravel()
        q = np.percentile(nc, [0, 25, 50, 75, 90, 99, 100])
        print(f"{name} target={target}: nc mean {nc.mean():.1f} pct[0,25,50,75,90,99,100] {q} "
              f"overflow(>128) {(nc > 128).mean():.3f}")
