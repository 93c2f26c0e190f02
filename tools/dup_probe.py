"""Candidates on discretisation points (Plan::dup): device KG / dKG/dx against the faithful oracle, per candidate.
Run on the GPU box:  python tools/dup_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.utils import make_torch_std_grid  # noqa: E402
from helpers import load_golden  # noqa: E402
from oracle.discretekg import discrete_kg_forward  # noqa: E402

torch.set_printoptions(precision=6, linewidth=200)
state, om, _, W, X, _ = load_golden("lengthscales0")
D = make_torch_std_grid(3, 2, {"dtype": torch.double})
W = W[:8]
X = torch.cat([D, X[:3]])
for target in (None, 0, 1):
    Xr = X.clone().unsqueeze(-2).requires_grad_(True)
    kg = discrete_kg_forward(om, Xr, D, W, target)
    (g,) = torch.autograd.grad(kg.sum(), Xr)
    acq = DiscreteKnowledgeGradient(state, D, W, target_output_ix=target, device="cuda:0")
    Xd = X.clone().cuda().requires_grad_(True)
    kd = acq(Xd.unsqueeze(-2))
    (gd,) = torch.autograd.grad(kd.sum(), Xd)
    a, b = acq._plan_for(X.shape[0]).lines(X.cuda().contiguous())
    print("target", target)
    for i in range(X.shape[0]):
        print(f"  x {X[i].tolist()} kg {kg[i].item():.9e} dev {kd[i].item():.9e} g {g[i,0].tolist()} dev {gd[i].tolist()}")
    print("  line0 a", a[:9, 0, 0].tolist())
    print("  linek a", [a[r, 0, r + 1].item() for r in range(9)])
    print("  line0 b", b[:9, 0, 0].tolist())
    print("  linek b", [b[r, 0, r + 1].item() for r in range(9)])
