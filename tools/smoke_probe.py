"""Where a device SMOKE run and the oracle run part (tests/test_gpu_bo_smoke.py::..._matches_the_oracle_run).

Run on the GPU box from the repo root:  python tools/smoke_probe.py [seed]
Prints both trajectories, and for every L-BFGS-B run of the device's full-evaluation steps the same run
with the oracle's KG from the same start: per objective call x, the device and oracle values and gradients.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import dkg_amd.optim as optim  # noqa: E402
from dkg_amd.bo_smoke import GPProblem, run_mobo  # noqa: E402
from helpers import load_golden  # noqa: E402
from smoke_oracle import HYPER, oracle_acq_factory  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
want = json.load(open(os.path.join(REPO, "tests", "golden", "smoke_oracle.json")))["seeds"][str(seed)]
state, *_ = load_golden("lengthscales0")

orig_gen = optim.gen_candidates_scipy
orig_acq = optim.DiscreteKgOptimisationSpec._acq
cur = {}


def acq_hook(self, model, input_dim, W, target):
    a = orig_acq(self, model, input_dim, W, target)
    from dkg_amd.utils import make_torch_std_grid
    disc = make_torch_std_grid(self.n_discretisation_points_per_axis, input_dim, {"dtype": torch.double})
    cur["oracle"] = oracle_acq_factory(model, disc, W, target)
    cur["target"] = target
    return a


def gen_hook(ic, acq, lb, ub, options=None):
    if True:
        from scipy.optimize import minimize
        for name, fn in (("device", acq), ("oracle", cur["oracle"])):
            log = []

            def f(x, fn=fn, name=name):
                X = torch.from_numpy(x).view(ic.shape).contiguous().requires_grad_(True)
                if name == "device":
                    kg, g = fn.value_and_grad_host(torch.from_numpy(x).view(ic.shape))
                    v, gg = -float(kg.sum()), (-g).reshape(-1).numpy()
                else:
                    loss = -fn(X).sum()
                    (gr,) = torch.autograd.grad(loss, X)
                    v, gg = float(loss), gr.reshape(-1).numpy()
                log.append((x.copy(), v, gg.copy()))
                return v, gg

            opts = {k: v for k, v in (options or {}).items() if k not in ("method", "callback", "with_grad")}
            res = minimize(f, ic.clamp(lb, ub).reshape(-1).numpy(), method="L-BFGS-B", jac=True,
                           bounds=list(zip(lb.expand(ic.shape).reshape(-1).tolist(),
                                           ub.expand(ic.shape).reshape(-1).tolist())), options=opts)
            print(f"  [{name}] target {cur['target']} start {ic.reshape(-1).tolist()} -> x {res.x.tolist()} f {res.fun:.12e} "
                  f"nit {res.nit} nfev {res.nfev} msg {res.message}")
            cur[name + "_log"] = log
        # the oracle's value / gradient at the device's iterates
        for i, (x, v, g) in enumerate(cur["device_log"]):
            X = torch.from_numpy(x).view(ic.shape).contiguous().requires_grad_(True)
            loss = -cur["oracle"](X).sum()
            (gr,) = torch.autograd.grad(loss, X)
            print(f"    it {i:3d} x {x.tolist()} dev {v:.15e} orc {float(loss):.15e} "
                  f"dv {v - float(loss):.2e} dg {np.abs(g - gr.reshape(-1).numpy()).max():.2e} |g| {np.abs(g).max():.2e}")
    return orig_gen(ic, acq, lb, ub, options)


optim.gen_candidates_scipy = gen_hook
optim.DiscreteKgOptimisationSpec._acq = acq_hook
for mode in ("separate", "full"):
    print("=====", mode)
    got = run_mobo(GPProblem(state, device="cuda:0"), HYPER, separate=mode == "separate", seed=seed)
    print("device", mode, "x", got["x"], "acq", got["acq"], "obj", got["obj_index"])
    print("oracle", mode, "x", want[mode]["x"], "acq", want[mode]["acq"], "obj", want[mode]["obj_index"])
