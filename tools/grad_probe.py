"""Gradient and stress parity probe (GPU box, repo root): how far inside candidate tolerances the device
gradient and the stress-shape KG are, on every candidate.

usage: python tools/grad_probe.py [out.json]

Gradient: dKG/dx through the C ABI (dkg_plan_forward_grad) against the oracle's autograd, all candidates of
``headline`` and ``headline_nd``, paths full and target 1.  Per candidate the scale of the quantities the
gradient sums is G = |d a_0/dx|_inf + max_k |d b_k/dx|_inf (line 0's intercept and every slope; central
differences of the oracle's lines, a magnitude only), and the tolerance tested is
    |g - g_ref| <= 1e-6 |g_ref| + 64 eps G              (tests/helpers.grad_tol).
Stress: KG end to end at the stated tolerance on 64 candidates of the stress shape, 48 of them the largest
device KGs (so most have KG > 0).
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402
from helpers import EPS, grad_scale, parity_case, to_oracle  # noqa: E402
from oracle.discretekg import discrete_kg_batched  # noqa: E402

DEV = "cuda:0"


def grad_case(wname, target):
    model, D, X, W = make_problem(WORKLOADS[wname])
    om = to_oracle(model)
    t0 = time.time()
    Xr = X.clone().requires_grad_(True)
    kg_ref, _ = discrete_kg_batched(om, Xr, D, W, target)
    (g_ref,) = torch.autograd.grad(kg_ref.sum(), Xr)
    t_or = time.time() - t0
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    kg, g = acq._plan_for(X.shape[0], grad=True).forward_grad(X.to(DEV))
    g = g.cpu()
    G = grad_scale(om, X, D, W, target)                      # [B]
    err = (g - g_ref).abs()
    rel = 1e-6 * g_ref.abs()
    floor = 64.0 * EPS * G[:, None]
    tol = rel + floor
    ratio = err / tol
    nz = (kg_ref.detach() > 0)
    return {"workload": wname, "target": target, "B": X.shape[0], "oracle_s": t_or,
            "kg_pos": int(nz.sum()), "g_nonzero_rows": int((g_ref.abs().amax(-1) > 0).sum()),
            "ratio_max": float(ratio.max()), "ratio_max_kgpos": float(ratio[nz].max()) if nz.any() else 0.0,
            "err_max": float(err.max()), "g_ref_max": float(g_ref.abs().max()),
            "rel_only_ratio_max": float((err / rel.clamp_min(1e-300)).max()),
            "floor_over_err_min": float((floor / err.clamp_min(1e-300)).min()),
            "G_median": float(G.median()), "G_max": float(G.max())}


def stress_case(target, n=64, top=48):
    model, D, X, W = make_problem(WORKLOADS["stress"])
    acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=DEV)
    kg = acq(X.to(DEV).unsqueeze(-2)).cpu()
    order = torch.argsort(kg, descending=True)
    pick = torch.cat([order[:top], order[-(n - top):]])
    t0 = time.time()
    res = parity_case(model, D, W, X[pick], target)
    row = {k: v for k, v in res.items() if not k.startswith("_")}
    row.update({"workload": "stress", "target": target, "picked_kg_pos": int((kg[pick] > 0).sum()),
                "oracle_s": time.time() - t0})
    return row


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "grad_probe.json")
    rep = {"grad": [], "stress": []}
    for wname in ("headline", "headline_nd"):
        for target in (None, 1):
            r = grad_case(wname, target)
            rep["grad"].append(r)
            print(json.dumps(r), flush=True)
    for target in (None, 2):
        r = stress_case(target)
        rep["stress"].append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(rep, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
