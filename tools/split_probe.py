"""Split-envelope probe: the single-output / single-scalarisation / Matern-1/2 parity case (S = 1, one-wave
envelope workgroups) through the plan's forward, printing the queue counters (Plan::wqctl, the workspace's
last 256-byte block) and the values.

usage: python tools/split_probe.py            (DKG_ENV_SPLIT / DKG_ENV_SPLIT_NOWALK pick the mode)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.model import ModelListGPState, SingleTaskGPState  # noqa: E402

print("start split", os.environ.get("DKG_ENV_SPLIT"), "nowalk", os.environ.get("DKG_ENV_SPLIT_NOWALK"), flush=True)
g = torch.Generator().manual_seed(9)
X = torch.rand(40, 2, generator=g, dtype=torch.double)
y = torch.cos(4 * X[:, 0]) * X[:, 1]
model = ModelListGPState(SingleTaskGPState(X, y, [0.4, 0.3], 2.0, 1e-2, 0.0, kernel="matern", nu=0.5))
D = torch.rand(100, 2, generator=g, dtype=torch.double)
Xc = torch.rand(10, 1, 2, generator=g, dtype=torch.double)
acq = DiscreteKnowledgeGradient(model, D)
plan = acq._state.plan(acq._W, acq._target, 10)
print("plan built, ws bytes", plan.ws.numel(), flush=True)
Xd = Xc.reshape(10, 2).cuda().contiguous()
kg = torch.empty(10, dtype=torch.double, device="cuda")
plan.forward_into(Xd, kg)
torch.cuda.synchronize()
ctl = plan.ws[-256:-248].clone().view(torch.int32).cpu().tolist()
print("wqctl (queued, claimed)", ctl, flush=True)
print("kg", kg.cpu().tolist(), flush=True)
