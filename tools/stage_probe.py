"""Per-stage launch times of one launch over G headline batches (dkg_plan_time_stage: HIP events around
back-to-back launches of the stage alone; stage 3 = the whole forward).

usage: python tools/stage_probe.py [--workload headline] [--groups 1 10 20] [--reps 20] [--precision fp64|fp32]
(DKG_COV_WIDE=0/1 forces the covariance block shape of a launch over B candidates.)
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]

import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="headline")
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 10, 20])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    model, D, X0, W = make_problem(w)
    acq = DiscreteKnowledgeGradient(model, D, W, device=dev, precision=args.precision)
    for G in args.groups:
        plan = acq._state.plan(acq._W, acq._target, G * w.B, f32=args.precision == "fp32")
        X = X0.to(dev).repeat(G, 1).contiguous()
        t = [plan.time_stage(X, k, args.reps) * 1e3 for k in range(4)]
        print(json.dumps({"workload": args.workload, "precision": args.precision, "G": G, "candidates": G * w.B,
                          "cross_us": t[0], "cov_us": t[1], "env_us": t[2], "forward_us": t[3],
                          "per_batch_us": [round(x / G, 3) for x in t],
                          "cov_wide_env": os.environ.get("DKG_COV_WIDE")}), flush=True)
        del plan


if __name__ == "__main__":
    main()
