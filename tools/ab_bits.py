"""Bit-identity of two builds of libdkg.so (DKG_LIB A/B): forward KG, KG per pair and the value+gradient
path on several workloads.

Run on the GPU box from the repo root:  python tools/ab_bits.py <libA.so> <libB.so>
Each build runs in its own subprocess (the library is loaded once per process); prints, per output, whether
the two builds agree bit for bit.
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if len(sys.argv) > 2 and sys.argv[1] == "--dump":
    sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
    import torch

    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem

    out = {}
    for name in ("small", "parity6d", "headline", "headline_nd", "stress"):
        w = WORKLOADS[name]
        model, D, X, W = make_problem(w)
        for target in (None, 1):
            acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)
            Xd = X.cuda().unsqueeze(-2)
            out[f"{name}/{target}/kg"] = acq(Xd).cpu()
            out[f"{name}/{target}/pairs"] = acq.forward_pairs(X.cuda()).cpu()
            if name in ("small", "headline"):
                Xg = X[:16].cuda().unsqueeze(-2).requires_grad_(True)
                (g,) = torch.autograd.grad(acq(Xg).sum(), Xg)
                out[f"{name}/{target}/grad"] = g.cpu()
    torch.save(out, sys.argv[2])
    sys.exit(0)

import torch  # noqa: E402

res = []
for i, lib in enumerate(sys.argv[1:3]):
    path = f"/tmp/ab_{i}.pt"
    subprocess.run([sys.executable, __file__, "--dump", path], check=True, env=dict(os.environ, DKG_LIB=lib))
    res.append(torch.load(path))
bad = 0
for k in res[0]:
    same = torch.equal(res[0][k], res[1][k])
    bad += not same
    diff = (res[0][k] - res[1][k]).abs().max().item()
    print(f"{k:28s} {'same bits' if same else 'DIFFERENT'}  max|diff| {diff:.3e}")
print("all identical" if bad == 0 else f"{bad} outputs differ")
sys.exit(1 if bad else 0)
