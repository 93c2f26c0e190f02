"""Time DiscreteKgOptimisationSpec.optimize_for_full_evaluation.

The reference's production setting (pipeline/nodes/bo_loop.py:123-131): 11 grid
points per axis, 10 restarts, 32 raw samples, batch_limit 1, maxiter 200.  The
GP is the headline synthetic state (2 outputs, n = 256, d = 2) with its 16
scalarisations.  Runs the device spec at batch_limit 1 (the reference's
setting) and batch_limit 10 (all restarts in one L-BFGS-B problem, one C call
per evaluation), and the oracle's structure-faithful CPU restatement at
batch_limit 1 on the same initial conditions (the reference's own BoTorch path
cannot run here: BoTorch is not installed).

Run on the GPU box:  python tools/bench_optimize.py [--cpu-seconds 60]
Prints one JSON line.
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]

import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient, make_torch_std_grid  # noqa: E402
from dkg_amd.optim import gen_batch_initial_conditions, optimize_acqf  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402


class Counting:
    def __init__(self, f):
        self.f, self.calls, self.points = f, 0, 0

    def __call__(self, X):
        self.calls += 1
        self.points += X.reshape(-1, X.shape[-1]).shape[0]
        return self.f(X)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-seconds", type=float, default=60.0, help="0 = skip the CPU restatement")
    ap.add_argument("--threads", type=int, default=16)
    args = ap.parse_args()
    torch.manual_seed(0)
    model, _, _, W = make_problem(WORKLOADS["headline"])
    D = make_torch_std_grid(11, 2, {"dtype": torch.double})
    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.double)
    acq = DiscreteKnowledgeGradient(model, D, W, device="cuda:0")
    ic = gen_batch_initial_conditions(acq, bounds, 1, 10, 32, {"seed": 0})
    out = {"config": {"grid": "11x11", "num_restarts": 10, "raw_samples": 32, "maxiter": 200, "m": 2,
                      "n_train": 256, "S": W.shape[0]}}
    for bl in (1, 10):
        c = Counting(acq)
        optimize_acqf(c, bounds, 1, 10, options={"batch_limit": bl, "maxiter": 200}, batch_initial_conditions=ic)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c = Counting(acq)
        x, v = optimize_acqf(c, bounds, 1, 10, options={"batch_limit": bl, "maxiter": 200},
                             batch_initial_conditions=ic)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        out[f"device_batch_limit_{bl}"] = {"seconds": dt, "acq_calls": c.calls, "points": c.points,
                                           "best_kg": float(v), "x": x.reshape(-1).tolist()}
    if args.cpu_seconds > 0:
        from oracle.discretekg import discrete_kg_forward
        from oracle.gp import ModelList, OutputGP

        torch.set_num_threads(args.threads)
        om = ModelList([OutputGP(m.train_x, m.train_y, m.lengthscale, m.outputscale, m.noise, m.mean_constant)
                        for m in model.models])
        c = Counting(lambda X: discrete_kg_forward(om, X, D, W))
        # one restart (batch_limit 1 = the reference's per-restart problem), timed, then scaled
        t0 = time.perf_counter()
        x, v = optimize_acqf(c, bounds, 1, 1, options={"batch_limit": 1, "maxiter": 200},
                             batch_initial_conditions=ic[:1])
        dt = time.perf_counter() - t0
        dev1 = out["device_batch_limit_1"]
        out["cpu_restatement_one_restart"] = {"seconds": dt, "acq_calls": c.calls, "kg": float(v),
                                              "threads": args.threads,
                                              "est_seconds_10_restarts": dt * 10}
        out["speedup_vs_cpu_restatement"] = {"batch_limit_1": dt * 10 / dev1["seconds"],
                                             "batch_limit_10": dt * 10 / out["device_batch_limit_10"]["seconds"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
